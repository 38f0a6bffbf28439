#!/bin/bash
# r02c: new GPU tests (configs, concurrency) first, then the whole GPU suite, smoke and a bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_concurrency_gpu.py tests/test_configs_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_new.log 2>&1 || { echo "new tests failed"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/pytest_new.log | tail -40; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
