# round 5: the replay generator with the camera-hit triangle cache: the C2 reference-sampler bench
# (replay ms), then the replay and C2 reference-sampler tests (sample tables bit-exact vs the oracle,
# the whole C2 frame in reference mode vs the oracle).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --sampler reference --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05i_bench_replay.log 2>&1 && \
grep '"metric"' gpurun_out/r05i_bench_replay.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])' && \
bash tools/gpu.sh r05i "tests=replay or reference_sampler"
