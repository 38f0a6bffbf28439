# GPU tests of one area (-k EXPR) and the C2 bench in its variants, one line each:
#   bash tools/gpu_variants.sh TAG "PYTEST_K_EXPR" "VARIANT_ARGS|..."
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; K=$2; VARIANTS=$3
if [ -n "$K" ]; then bash tools/gpu.sh $TAG tests="$K" || exit 1; fi
IFS='|' read -ra VS <<< "$VARIANTS"
i=0
for args in "${VS[@]}"; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $args > gpurun_out/${TAG}_v$i.log 2>&1 || { echo "bench [$args] failed"; tail -8 gpurun_out/${TAG}_v$i.log; exit 1; }
  grep '"metric"' gpurun_out/${TAG}_v$i.log > gpurun_out/${TAG}_v$i.jsonl
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_step"])' gpurun_out/${TAG}_v$i.jsonl "[$args]" | tee -a gpurun_out/${TAG}_variants.txt
done
echo ALL_OK
