#!/bin/bash
# r02p: the half-group gather (MPSS_MO_HALF=1: 2 bands per lane, 8192-entry LDS near field) --
# Mo / golden / render parity under it, then C2 bench lines for the default and the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
MPSS_MO_HALF=1 timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py tests/test_concurrency_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_half.log 2>&1 || { echo "half tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_half.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_half.log
for h in 0 1 0 1; do
  MPSS_MO_HALF=$h timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_half$h.log 2>&1 || { echo "bench half=$h failed"; tail -20 gpurun_out/bench_half$h.log; exit 1; }
  echo "half=$h $(grep metric gpurun_out/bench_half$h.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["kernel_ms_per_step"], d["config"]["mo_lane_efficiency"])')"
done
