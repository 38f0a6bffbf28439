#!/bin/bash
# r02ar: TIMING EXPERIMENT (sums wrong): the gather with its table / near-field loads replaced by a
# register value (addresses still computed) -- how much of the launch the lookups' memory path costs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export MPSS_MO_DBG_NOLOAD=1; else unset MPSS_MO_DBG_NOLOAD; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ar$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ar$v.log; exit 1; }
  echo "noload=$v $(grep metric gpurun_out/bench_ar$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"])')"
done
