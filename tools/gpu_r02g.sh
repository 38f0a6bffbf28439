#!/bin/bash
# r02g: GPU rho table tests first, then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_rho_gpu.py tests/test_golden_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { echo "new tests failed"; grep -E "PASSED|FAILED|Error|assert|material build" gpurun_out/pytest_new.log | tail -40; exit 1; }
grep -E "PASSED|FAILED|material build" gpurun_out/pytest_new.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
