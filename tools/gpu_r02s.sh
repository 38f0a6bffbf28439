#!/bin/bash
# r02s: atomics-free octree level assignment -- octree tests, then a C2 bench line (with the
# node / point split of the gather's wave iterations).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_octree_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_s.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_s.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_s.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_s.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_s.log; exit 1; }
grep metric gpurun_out/bench_s.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); c=d["config"]; print(d["value"], d["ms_per_step"], c["preprocess_s"], c["mo_wave_iters"], c["mo_visits"], d["roofline"]["traffic"], d["roofline"].get("traffic_source"))'
