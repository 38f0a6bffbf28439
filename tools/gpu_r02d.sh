#!/bin/bash
# r02d: the Monte-Carlo profile work (mcprofile renderer file, diffusion check, usemontecarlo
# material) and the MC walk / C4 tests that share its kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_mcprofile_gpu.py tests/test_mc_gpu.py "tests/test_configs_gpu.py::test_c4_mcprofile_1e7_photons" -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_mc.log 2>&1 || { echo "mc tests failed"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_mc.log | tail -40; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_mc.log
