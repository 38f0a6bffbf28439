#!/bin/bash
# Mo-gather variant sweep, round 2: bs:k:near:pair[:batch_log2] (env knobs of mo_kernel.hip, bench --batch-log2).
# One C2 bench line each (no CPU leg): Msamples/s, mo_band ms per step, lane efficiency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${VARIANTS:-1024:4096:2:0 1024:0:0:1 1024:4096:4:1 1024:4096:4:0 1024:4096:2:1}; do
  IFS=: read bs k near pair blog <<< "$v"
  extra=""
  [ -n "$blog" ] && extra="--batch-log2 $blog"
  MPSS_MO_BS=$bs MPSS_MO_K=$k MPSS_MO_NEAR=$near MPSS_MO_PAIR=$pair timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $extra > gpurun_out/var.log 2>&1 || { echo "bench failed $v"; tail -20 gpurun_out/var.log; exit 1; }
  echo "$v $(grep metric gpurun_out/var.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"], d["config"]["mo_lane_efficiency"])')"
done
