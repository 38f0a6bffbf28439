#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_micro
timeout -k 10 120 ./tools/microbench/l2_gather 256 > gpurun_out/l2_gather.json 2>&1 || { echo fail; cat gpurun_out/l2_gather.json; exit 1; }
cat gpurun_out/l2_gather.json
timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/prof_micro/pmc_1 -o run --output-format csv -- ./tools/microbench/l2_gather 256 > gpurun_out/prof_micro/pmc_1.log 2>&1 || { echo pmcfail; tail -5 gpurun_out/prof_micro/pmc_1.log; exit 1; }
echo pmc ok
