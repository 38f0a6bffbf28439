#!/bin/bash
# r02f: the new GPU tests (dipole Mo, pointsfile, golden fixtures, the reference's env map).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_dipole_gpu.py tests/test_formats_gpu.py tests/test_golden_gpu.py "tests/test_render_parity_gpu.py::test_image_parity_infinite_light" -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { echo "new tests failed"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_new.log | tail -40; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_new.log
