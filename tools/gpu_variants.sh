#!/bin/bash
# Mo-gather variant sweep (env knobs of mo_kernel.hip): one C2 bench line each (no CPU leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${VARIANTS:-1024:4096:1 1024:4096:2 512:2048:1 1024:9216:1 512:0:0}; do
  IFS=: read bs k near <<< "$v"
  MPSS_MO_BS=$bs MPSS_MO_K=$k MPSS_MO_NEAR=$near timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/var.log 2>&1 || { echo "bench failed $v"; tail -20 gpurun_out/var.log; exit 1; }
  echo "$v $(grep metric gpurun_out/var.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_per_step"]["mo_band"], d["config"]["mo_lane_efficiency"], d["config"]["mo_lookup_near_fraction"])')"
done
