#!/bin/bash
# r02ao: camera samples per render batch (one Mo() launch per batch): 2^26 (default) vs 2^27 / 2^25
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in 26 27 25 27 26; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --batch-log2 $v > gpurun_out/bench_ao$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ao$v.log; exit 1; }
  echo "batch=2^$v $(grep metric gpurun_out/bench_ao$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"], r["kernel_ms_per_step"])')"
done
