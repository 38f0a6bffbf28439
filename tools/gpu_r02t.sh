#!/bin/bash
# r02t: single-GPU C3 and C5 lines at HEAD (batched launches, BSDF-ray sphere skip, GPU octree).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { echo "c3 failed"; tail -20 gpurun_out/bench_c3.log; exit 1; }
grep metric gpurun_out/bench_c3.log | cut -c1-300
timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/bench_c5.log; exit 1; }
grep metric gpurun_out/bench_c5.log | cut -c1-300
