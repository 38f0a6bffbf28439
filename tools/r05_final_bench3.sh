# round 5, last measurements after the tightened camera-ray candidate lists: the default bench line
# (C2 hash headline, CPU baseline, reference-sampler secondary) and the reference-sampler C2 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=r05zf
bash tools/gpu.sh $T bench || exit 1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary --sampler reference > gpurun_out/${T}_bench_c2_replay.log 2>&1 || { tail -20 gpurun_out/${T}_bench_c2_replay.log; exit 1; }
grep '"metric"' gpurun_out/${T}_bench_c2_replay.log > gpurun_out/${T}_bench_c2_replay.jsonl
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])' gpurun_out/${T}_bench_c2_replay.jsonl
