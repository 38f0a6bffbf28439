#!/bin/bash
# r02ax: TIMING EXPERIMENT: 16 real v_add_f32 per point-pair step (XV1) / 8 per node test (XV2)

set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in 0 1 2 0 1 2; do
  unset MPSS_MO_XV1 MPSS_MO_XV2
  if [ $v = 1 ]; then export MPSS_MO_XV1=1; fi
  if [ $v = 2 ]; then export MPSS_MO_XV2=1; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ax$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ax$v.log; exit 1; }
  echo "xv=$v $(grep metric gpurun_out/bench_ax$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_ms"])')"
done
