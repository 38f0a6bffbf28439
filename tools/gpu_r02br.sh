#!/bin/bash
# r02br: final state -- the whole GPU suite and smoke at HEAD, C3 and C5 lines, and the C2 profile set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | tail -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { echo "c3 failed"; tail -20 gpurun_out/bench_c3.log; exit 1; }
timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/bench_c5.log; exit 1; }
for c in c3 c5; do grep metric gpurun_out/bench_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])'; done
bash tools/gpu_round.sh ${1:-r02br}
