#!/bin/bash
# Detailed PMC passes of the render bench for the Mo gather. Usage: bash tools/prof_mo_detail.sh TAG
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r01}
D=gpurun_out/prof_$TAG
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
run() { name=$1; shift; timeout -k 10 300 rocprofv3 --pmc "$@" -d $D/$name -o run --output-format csv -- $B > $D/$name.log 2>&1 || echo "pass $name failed"; }
run pmc_a SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run pmc_b TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
run pmc_c TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCC_BUSY_sum TCC_TAG_STALL_sum
run pmc_d SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_SALU
run pmc_e FETCH_SIZE
run pmc_f TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
echo PROF_DONE
