#!/bin/bash
# r02x: the wave-queue gather with a 5088-entry near field (default) vs 4096 (MPSS_MO_WK=4096).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_x.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_x.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_x.log
for k in 5088 4096 5088 4096; do
  MPSS_MO_WK=$k timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_x$k.log 2>&1 || { echo "bench k=$k failed"; tail -20 gpurun_out/bench_x$k.log; exit 1; }
  echo "k=$k $(grep metric gpurun_out/bench_x$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
