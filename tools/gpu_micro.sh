#!/bin/bash
# Microbenchmarks of the gather's memory path (binaries built on the CPU side beforehand:
#   hipcc -O3 --offload-arch=gfx950 tools/microbench/X.hip -o tools/microbench/X).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in "$@"; do
  timeout -k 10 120 ./tools/microbench/$b 256 > gpurun_out/micro_$b.json 2>&1 || { echo "$b failed"; cat gpurun_out/micro_$b.json; exit 1; }
  cat gpurun_out/micro_$b.json
done
