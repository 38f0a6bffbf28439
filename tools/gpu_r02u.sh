#!/bin/bash
# r02u: node records loaded in one scalar round trip (HOIST, default) vs the r02 kernel
# (MPSS_MO_HOIST=0) -- Mo / golden / render parity, then alternating C2 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_u.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_u.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_u.log
for h in 1 0 1 0; do
  MPSS_MO_HOIST=$h timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_u$h.log 2>&1 || { echo "bench hoist=$h failed"; tail -20 gpurun_out/bench_u$h.log; exit 1; }
  echo "hoist=$h $(grep metric gpurun_out/bench_u$h.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
