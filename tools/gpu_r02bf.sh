#!/bin/bash
# r02bf: adjacent-reach groups (MPSS_MO_CONTIG) under the default work stealing vs snake groups
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export MPSS_MO_CONTIG=1
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_bf.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_bf.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_bf.log
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export MPSS_MO_CONTIG=1; else unset MPSS_MO_CONTIG; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_bf$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_bf$v.log; exit 1; }
  echo "contig=$v $(grep metric gpurun_out/bench_bf$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"])')"
done
