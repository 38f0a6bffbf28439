# round 5, final measurements on the final tree: kernel trace and PMC passes of the C2 bench; the default bench line
# (C2, CPU baseline, reference-sampler secondary); rgbprofile, textured and reference-sampler C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=r05z
PMC_SETS="$(cat tools/pmc_sets_r05e.txt)" bash tools/gpu.sh $T kt pmc || exit 1
python3 tools/summarize_prof.py $T || exit 1  # (profiles/r05z_pmc.json on the box: the bench lines below read it)
bash tools/gpu.sh $T bench || exit 1
run() {  # name, bench args
  echo "== $1"
  timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary ${@:2} > gpurun_out/${T}_bench_$1.log 2>&1 || { echo "$1 failed"; tail -20 gpurun_out/${T}_bench_$1.log; exit 1; }
  grep '"metric"' gpurun_out/${T}_bench_$1.log > gpurun_out/${T}_bench_$1.jsonl
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])' gpurun_out/${T}_bench_$1.jsonl
}
run c2_rgb --rgb-profile && \
run c2_textured --scene scenes/skin_textured.pbrt && \
run c2_replay --sampler reference
