#!/bin/bash
# r02m: single-GPU lines for BASELINE's other configs at HEAD: C3 (2048^2 256 spp), C5 (4096^2 512
# spp, 4 M triangles), C4 (10^8 photons MC walk vs the multipole profile).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { echo "c3 failed"; tail -20 gpurun_out/bench_c3.log; exit 1; }
grep metric gpurun_out/bench_c3.log
timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/bench_c5.log; exit 1; }
grep metric gpurun_out/bench_c5.log
timeout -k 10 300 python tools/bench_mc.py > gpurun_out/bench_c4.log 2>&1 || { echo "c4 failed"; tail -20 gpurun_out/bench_c4.log; exit 1; }
tail -3 gpurun_out/bench_c4.log
