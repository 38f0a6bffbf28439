#!/bin/bash
# r02bp: NEAR 9 (past-end lanes issue no load; exec-masked flat loads in one asm block) vs NEAR 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MPSS_MO_N9=1
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_bp.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_bp.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_bp.log
for v in 7 5 7 5; do
  if [ $v = 7 ]; then export MPSS_MO_N9=1; else unset MPSS_MO_N9; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_bp$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_bp$v.log; exit 1; }
  echo "n9=$v $(grep metric gpurun_out/bench_bp$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
