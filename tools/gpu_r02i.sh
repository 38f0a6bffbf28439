#!/bin/bash
# r02i: Mo pair/near variants must match the oracle before they are timed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in "0 4096 2 0" "1 0 0 1" "1 4096 4 1" "0 4096 4 0"; do
  read pair k near x <<< "$v"
  MPSS_MO_PAIR=$pair MPSS_MO_K=$k MPSS_MO_NEAR=$near timeout -k 10 300 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_var.log 2>&1 || { echo "variant $v failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_var.log | tail -20; exit 1; }
  echo "variant pair=$pair k=$k near=$near: $(tail -1 gpurun_out/pt_var.log)"
done
VARIANTS="1024:4096:2:0 1024:0:0:1 1024:4096:4:1 1024:4096:4:0 1024:4096:2:1 1024:4096:2:0:26" bash tools/gpu_variants2.sh
