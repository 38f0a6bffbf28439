#!/bin/bash
# r02bh: NEAR 8 (3-band groups spread the LDS over 3 rows of 13649 entries) with the 3-band groups
# placed on the longest reach (MPSS_MO_HEAVY3) or the shortest (default adjacent-reach deal)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MPSS_MO_N8=1 MPSS_MO_HEAVY3=1
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_bh.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_bh.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_bh.log
for v in h8 d n8 h8 d n8; do
  unset MPSS_MO_N8 MPSS_MO_HEAVY3
  if [ $v = h8 ]; then export MPSS_MO_N8=1 MPSS_MO_HEAVY3=1; fi
  if [ $v = n8 ]; then export MPSS_MO_N8=1; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_bh$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_bh$v.log; exit 1; }
  echo "v=$v $(grep metric gpurun_out/bench_bh$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"])')"
done
