#!/bin/bash
# r02ac: NEAR 5 (past-end lanes on an LDS zero pair, one select less per band) in the 10236-entry
# wave kernel (default) vs NEAR 2 (MPSS_MO_WN2=1), now that VALU is the tighter bound.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py tests/test_dipole_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_ac.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_ac.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_ac.log
for n in 5 2 5 2; do
  if [ $n = 2 ]; then export MPSS_MO_WN2=1; else unset MPSS_MO_WN2; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ac$n.log 2>&1 || { echo "bench n=$n failed"; tail -20 gpurun_out/bench_ac$n.log; exit 1; }
  echo "near=$n $(grep metric gpurun_out/bench_ac$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
