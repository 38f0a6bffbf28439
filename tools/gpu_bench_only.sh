#!/bin/bash
# One C2 bench line (no tests, no profiling): quick A/B of a kernel change.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bench.log | head -1
grep -o '"kernel_ms_per_step": {[^}]*}' gpurun_out/bench.log
