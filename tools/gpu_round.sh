#!/bin/bash
# One GPU session: parity/property tests, a short bench with an image, a rocprofv3 kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --out gpurun_out/skin.pfm > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
