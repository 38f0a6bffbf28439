#!/bin/bash
# r02l: live band slots in the leaf loop -- Mo parity tests, then the C2 bench (with counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_l.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_l.log | tail -20; tail -5 gpurun_out/pt_l.log; exit 1; }
tail -1 gpurun_out/pt_l.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_l.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_l.log; exit 1; }
grep metric gpurun_out/bench_l.log
