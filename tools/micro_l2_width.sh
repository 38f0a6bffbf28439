#!/bin/bash
# tools/microbench/l2_width: every variant's rate, then L2 requests / TA busy under PMC for the listed
# variants (one rocprofv3 pass each) -> gpurun_out/TAG/
#   bash tools/r06_micro.sh TAG "V1 V2 ..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:?usage: r06_micro.sh TAG "variants"}
mkdir -p gpurun_out/$TAG
timeout -k 10 120 ./tools/microbench/l2_width 256 > gpurun_out/$TAG/l2_width.json 2>&1 || { cat gpurun_out/$TAG/l2_width.json; exit 1; }
cat gpurun_out/$TAG/l2_width.json
for v in $2; do
  timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum -d gpurun_out/$TAG/pmc_$v -o run --output-format csv -- ./tools/microbench/l2_width 256 $v > gpurun_out/$TAG/pmc_$v.log 2>&1 || { echo pmc $v failed; tail -5 gpurun_out/$TAG/pmc_$v.log; exit 1; }
done
echo ALL_OK
