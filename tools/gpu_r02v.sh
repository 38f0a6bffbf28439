#!/bin/bash
# r02v: the wave-queue gather (MPSS_MO_WAVEQ=1: chunks sorted by a separate kernel, waves take
# 64 queries at a time with no workgroup barrier) -- parity under it, then alternating C2 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
MPSS_MO_WAVEQ=1 timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py tests/test_concurrency_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_v.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_v.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_v.log
for w in 1 0 1 0; do
  MPSS_MO_WAVEQ=$w timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_v$w.log 2>&1 || { echo "bench waveq=$w failed"; tail -20 gpurun_out/bench_v$w.log; exit 1; }
  echo "waveq=$w $(grep metric gpurun_out/bench_v$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["config"]["mo_lane_efficiency"])')"
done
