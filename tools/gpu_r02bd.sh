#!/bin/bash
# r02bd: per-group (XCD) start / finish times of the gather (MPSS_MO_WGTIME instrumentation)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MPSS_MO_WGTIME=1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_bd.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_bd.log; exit 1; }
grep wgtime gpurun_out/bench_bd.log | tail -6
