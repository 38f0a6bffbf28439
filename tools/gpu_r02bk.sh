#!/bin/bash
# r02bk (was r02an): stall / pipe-occupancy counters of the gather (what the waves wait on), one rocprofv3 pass
# per counter group, each under its own kill timer; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=r02bk
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "== pmc $i: $line"
  timeout -s KILL 240 rocprofv3 --pmc $line -d gpurun_out/prof_$TAG/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$TAG/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/prof_$TAG/pmc_$i.log; exit 1; }
done <<< "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_LDS
SQ_BUSY_CYCLES SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT SQ_INSTS_FLAT_NO_LDS SQ_WAIT_INST_LDS
TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
SQ_LEVEL_WAVES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD SQ_CYCLES SQ_ACCUM_PREV_HIRES SQ_INSTS_SMEM_NORM"
echo ALL_OK
