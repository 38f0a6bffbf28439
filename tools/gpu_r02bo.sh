#!/bin/bash
# r02bo: the whole GPU suite and smoke at HEAD, and the default bench line (with the CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_bo.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_bo.log | tail -20; tail -5 gpurun_out/pytest_gpu_bo.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_bo.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_bo.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_bo.log; exit 1; }
tail -1 gpurun_out/smoke_bo.log
timeout -k 10 400 python bench.py > gpurun_out/bench_bo.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_bo.log; exit 1; }
grep metric gpurun_out/bench_bo.log
