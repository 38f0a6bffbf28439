#!/bin/bash
# r02af: band row bases held in VGPRs for the whole traversal (default for the 10236-entry gather)
# vs re-copied from SGPRs per lookup (MPSS_MO_NOVROWS=1); also the 128-VGPR register target.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_af.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_af.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_af.log
for v in 1 0 1 0; do
  if [ $v = 0 ]; then export MPSS_MO_NOVROWS=1; else unset MPSS_MO_NOVROWS; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_af$v.log 2>&1 || { echo "bench v=$v failed"; tail -20 gpurun_out/bench_af$v.log; exit 1; }
  echo "vrows=$v $(grep metric gpurun_out/bench_af$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
