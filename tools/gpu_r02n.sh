#!/bin/bash
# r02n: GPU octree build -- its own tests first, then the whole GPU suite and a C2 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_octree_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_oct.log 2>&1 || { echo "octree tests failed"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pt_oct.log | tail -30; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pt_oct.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_n.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_n.log; exit 1; }
grep metric gpurun_out/bench_n.log | cut -c1-900
