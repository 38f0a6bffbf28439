#!/bin/bash
# PMC passes of the C2 bench (one counter group per run; kernel-trace only, no sys/runtime trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r02x}
mkdir -p gpurun_out/prof_$TAG
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $line -d gpurun_out/prof_$TAG/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$TAG/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/prof_$TAG/pmc_$i.log; exit 1; }
  echo "pass $i ok: $line"
done <<< "${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES
SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE}"
