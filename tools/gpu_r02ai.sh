#!/bin/bash
# r02ai: FAR skip (records whose terms are +0 for the whole wave skipped; default)
# vs no skip (MPSS_MO_NOFAR=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_ai.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_ai.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_ai.log
for v in 1 0 1 0; do
  if [ $v = 0 ]; then export MPSS_MO_NOFAR=1; else unset MPSS_MO_NOFAR; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ai$v.log 2>&1 || { echo "bench v=$v failed"; tail -20 gpurun_out/bench_ai$v.log; exit 1; }
  echo "far=$v $(grep metric gpurun_out/bench_ai$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
unset MPSS_MO_NOFAR
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/prof_r02ai
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02ai/kt -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02ai/kt.log 2>&1 || { echo "kt failed"; tail -5 gpurun_out/prof_r02ai/kt.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_r02ai/kt/run_kernel_stats.csv')))[:8]: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])
"
