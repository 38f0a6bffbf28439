#!/bin/bash
# r02aa: gather time vs resident workgroups per band group (MPSS_MO_WGS): is it L2-bound with
# fewer waves, leaving CU slots for other kernels?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for w in 64 56 48 40 32; do
  MPSS_MO_WGS=$w timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_aa$w.log 2>&1 || { echo "bench wgs=$w failed"; tail -20 gpurun_out/bench_aa$w.log; exit 1; }
  echo "wgs=$w $(grep metric gpurun_out/bench_aa$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
