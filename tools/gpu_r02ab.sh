#!/bin/bash
# r02ab: one gather workgroup per CU with a 10236-entry near field (MPSS_MO_WK=10236) vs two with
# 5088 -- parity under the variant, then alternating C2 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
MPSS_MO_WK=10236 timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_ab.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_ab.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_ab.log
for k in 10236 5088 10236 5088; do
  MPSS_MO_WK=$k timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ab$k.log 2>&1 || { echo "bench k=$k failed"; tail -20 gpurun_out/bench_ab$k.log; exit 1; }
  echo "k=$k $(grep metric gpurun_out/bench_ab$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
