#!/bin/bash
# GPU tests + one bench line (no profiling). Usage: bash tools/gpu_quick.sh [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then KARG="-k $K"; else KARG=""; fi
timeout -k 10 600 python -m pytest tests -m gpu -x -q $KARG > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log | grep metric
timeout -k 10 300 python tools/bench_mc.py --cpu-seconds 5 > gpurun_out/bench_mc.log 2>&1 || { echo "bench_mc failed"; tail -30 gpurun_out/bench_mc.log; exit 1; }
cat gpurun_out/bench_mc.log
