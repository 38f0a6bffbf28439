#!/bin/bash
# r02h: reference-sampler replay tests on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_replay_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_replay.log 2>&1 || { echo "replay tests failed"; grep -E "PASSED|FAILED|Error|assert|first differing" gpurun_out/pytest_replay.log | tail -40; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_replay.log
