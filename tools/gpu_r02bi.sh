#!/bin/bash
# r02bi: C5 on one GPU under the adjacent-reach groups + work stealing: kernel trace and the PMC passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=r02bi
mkdir -p gpurun_out/prof_$TAG
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/kt -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG/kt.log 2>&1 || { echo "rocprof kt failed"; tail -30 gpurun_out/prof_$TAG/kt.log; exit 1; }
grep metric gpurun_out/prof_$TAG/kt.log > gpurun_out/prof_$TAG/kt_bench.jsonl || true
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "== pmc $i: $line"
  timeout -s KILL 300 rocprofv3 --pmc $line -d gpurun_out/prof_$TAG/pmc_$i -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$TAG/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/prof_$TAG/pmc_$i.log; exit 1; }
done <<< "FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
echo ALL_OK
