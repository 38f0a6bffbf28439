#!/bin/bash
# r02ap: odd render batches on a second workspace + stream (camera/direct kernels overlap the previous
# batch's gather) vs one stream (MPSS_NO_BATCH_OVERLAP=1); render parity + concurrency tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_render_parity_gpu.py tests/test_concurrency_gpu.py tests/test_golden_gpu.py tests/test_replay_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_ap.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_ap.log | tail -20; tail -3 gpurun_out/pt_ap.log; exit 1; }
tail -1 gpurun_out/pt_ap.log
for v in 1 0 1 0; do
  if [ $v = 0 ]; then export MPSS_NO_BATCH_OVERLAP=1; else unset MPSS_NO_BATCH_OVERLAP; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ap$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ap$v.log; exit 1; }
  echo "overlap=$v $(grep metric gpurun_out/bench_ap$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"], r["kernel_ms_per_step"])')"
done
