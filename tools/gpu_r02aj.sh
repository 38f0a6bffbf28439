#!/bin/bash
# r02aj: the lerp products added by one v_add_f32 each; + a scheduling barrier after the pair loop fetches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py tests/test_render_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_aj.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_aj.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_aj.log
for v in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_aj$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_aj$v.log; exit 1; }
  echo "run=$v $(grep metric gpurun_out/bench_aj$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
done
