#!/bin/bash
# r02o: rgbprofile LayeredSkin -- its GPU tests, then the Mo / render parity tests it touches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rgbprofile_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pt_rgb.log 2>&1 || { echo "rgb tests failed"; grep -E "PASSED|FAILED|Error|assert|^E " gpurun_out/pt_rgb.log | tail -30; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pt_rgb.log
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_dipole_gpu.py tests/test_render_parity_gpu.py tests/test_concurrency_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_o.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_o.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_o.log
