#!/bin/bash
# r02j: batch size and the 9216-entry near field with paired point loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
MPSS_MO_PAIR=1 MPSS_MO_K=9216 MPSS_MO_NEAR=2 timeout -k 10 300 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_var.log 2>&1 || { echo "9216 pair failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_var.log | tail -20; exit 1; }
VARIANTS="1024:4096:2:1:26 1024:4096:2:1:27 1024:9216:2:1:26 1024:4096:2:0:24" bash tools/gpu_variants2.sh
