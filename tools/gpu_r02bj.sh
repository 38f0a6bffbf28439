#!/bin/bash
# r02bj: batch overlap (odd render batches on a second workspace + stream) now that the gather has
# VALU slack, at 2^26 / 2^25 / 2^24 samples per batch; MPSS_NO_BATCH_OVERLAP=1 is the baseline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_render_parity_gpu.py tests/test_concurrency_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_bj.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_bj.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_bj.log
for v in "26 0" "26 1" "25 1" "25 0" "24 1" "26 0"; do
  set -- $v
  if [ $2 = 0 ]; then export MPSS_NO_BATCH_OVERLAP=1; else unset MPSS_NO_BATCH_OVERLAP; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --batch-log2 $1 > gpurun_out/bench_bj.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_bj.log; exit 1; }
  echo "batch=2^$1 overlap=$2 $(grep metric gpurun_out/bench_bj.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms_per_step"])')"
done
