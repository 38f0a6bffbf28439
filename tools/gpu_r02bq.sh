#!/bin/bash
# r02bq: the instrumented (count) gather pass with work stealing: Mo tests (counters vs oracle) and
# the default bench (its untimed count passes get shorter; the timed line must not change)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mo_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_bq.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_bq.log | tail -20; exit 1; }
tail -1 gpurun_out/pt_bq.log
SECONDS=0; timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_bq.log 2> gpurun_out/bench_bq.err || { echo "bench failed"; tail -20 gpurun_out/bench_bq.err; exit 1; }
echo "bench wall ${SECONDS} s"
grep metric gpurun_out/bench_bq.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); r=d["roofline"]; c=d["config"]; print(d["value"], r["avg_launch_ms"], c["mo_group_visits"], r["bytes_definition"])'
