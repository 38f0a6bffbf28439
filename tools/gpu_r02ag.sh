#!/bin/bash
# r02ag: node test with the centroid distance first (box test only where it can prune; default) vs the box test first (MPSS_MO_BOXFIRST=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py tests/test_concurrency_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_ag.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_ag.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_ag.log
for v in 1 0 1 0; do
  if [ $v = 0 ]; then export MPSS_MO_BOXFIRST=1; else unset MPSS_MO_BOXFIRST; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ag$v.log 2>&1 || { echo "bench v=$v failed"; tail -20 gpurun_out/bench_ag$v.log; exit 1; }
  echo "d2first=$v $(grep metric gpurun_out/bench_ag$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
