# Same-box A/B of bench.py argument sets: bash tools/x_ab.sh TAG "ARGS_A" "ARGS_B" [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; A=$2; B=$3; R=${4:-2}
for r in $(seq 1 $R); do
  for v in A B; do
    args=$A; [ $v = B ] && args=$B
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $args > gpurun_out/${TAG}_$v$r.log 2>&1 || { echo "run $v$r failed"; tail -5 gpurun_out/${TAG}_$v$r.log; exit 1; }
    python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); c=d["config"]; print(sys.argv[2], d["value"], d["roofline"]["kernel_ms_per_step"]["mo_band"], c.get("mo_lane_records"))' gpurun_out/${TAG}_$v$r.log "$v$r [$args]" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
echo ALL_OK
