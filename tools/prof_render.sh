#!/bin/bash
# PMC passes of the render bench (mo_band_kernel focus). Usage: bash tools/prof_render.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r01}
D=gpurun_out/prof_$TAG
mkdir -p $D
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $D/pmc_sq -o run --output-format csv -- $B > $D/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -20 $D/pmc_sq.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum -d $D/pmc_tcp -o run --output-format csv -- $B > $D/pmc_tcp.log 2>&1 || { echo "pmc tcp failed"; tail -20 $D/pmc_tcp.log; exit 1; }

timeout -k 10 120 rocprofv3 -L > $D/counters_list.txt 2>&1 || true
echo PROF_OK
