#!/bin/bash
# r02ak: TIMING EXPERIMENT (sums wrong): lookups with KLDS <= s < MPSS_MO_DBG_KLIM read the LDS zero
# pair instead of L2 -- how the gather time falls with a bigger near field (the 2-bands-per-group case).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in 0 20472 40944 1000000 0; do
  export MPSS_MO_DBG_KLIM=$v
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ak$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ak$v.log; exit 1; }
  echo "klim=$v $(grep metric gpurun_out/bench_ak$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
