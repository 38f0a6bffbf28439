#!/bin/bash
# r02av: EXPERIMENT: a no-LDS copy of the gather on a second stream sharing the wave queue
# (MPSS_MO_DUAL=n: n workgroups of 16 waves per group) beside the near-field workgroups.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MPSS_MO_DUAL=32
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_av.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_av.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_av.log
for v in 0 32 16 0 32 8; do
  if [ $v = 0 ]; then unset MPSS_MO_DUAL; else export MPSS_MO_DUAL=$v; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_av$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_av$v.log; exit 1; }
  echo "dual=$v $(grep metric gpurun_out/bench_av$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"])')"
done
