#!/bin/bash
# r02y: past-end lanes on an LDS zero pair (NEAR 5, default) vs the table's zero pair (MPSS_MO_WNEAR=2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py tests/test_dipole_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_y.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_y.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_y.log
for n in 5 2 5 2; do
  MPSS_MO_WNEAR=$n timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_y$n.log 2>&1 || { echo "bench n=$n failed"; tail -20 gpurun_out/bench_y$n.log; exit 1; }
  echo "near=$n $(grep metric gpurun_out/bench_y$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
