#!/bin/bash
# One GPU session: tests, bench (with CPU baseline and an image), rocprofv3 kernel trace and
# PMC passes of the bench. Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out gpurun_out/prof_${1:-r01}
export TMPDIR=/tmp
TAG=${1:-r01}
step() { echo "== $*"; }
step pytest
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
step bench
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --out gpurun_out/skin.exr > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
step rocprof-kernel-trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG/kt -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG/kt.log 2>&1 || { echo "rocprof kt failed"; tail -30 gpurun_out/prof_$TAG/kt.log; exit 1; }
step rocprof-pmc-fetch
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_$TAG/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$TAG/pmc_fetch.log 2>&1 || { echo "rocprof pmc failed"; tail -30 gpurun_out/prof_$TAG/pmc_fetch.log; exit 1; }
step rocprof-pmc-l2
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof_$TAG/pmc_l2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$TAG/pmc_l2.log 2>&1 || { echo "rocprof pmc2 failed"; tail -30 gpurun_out/prof_$TAG/pmc_l2.log; exit 1; }
echo ALL_OK
