#!/bin/bash
# r02bm: steal from the group with the most units left (MPSS_MO_STEALMAX) vs the next group in order
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MPSS_MO_STEALMAX=1
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_bm.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_bm.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_bm.log
for v in 7 5 7 5; do
  if [ $v = 7 ]; then export MPSS_MO_STEALMAX=1; else unset MPSS_MO_STEALMAX; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_bm$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_bm$v.log; exit 1; }
  echo "max=$v $(grep metric gpurun_out/bench_bm$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
