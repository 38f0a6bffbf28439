# Same-box A/B of an environment switch: bash tools/x_ab_env.sh TAG "ARGS" VAR [ROUNDS]  (A: VAR unset, B: VAR=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; ARGS=$2; VAR=$3; R=${4:-2}
for r in $(seq 1 $R); do
  for v in A B; do
    if [ $v = B ]; then export $VAR=1; else unset $VAR; fi
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary $ARGS > gpurun_out/${TAG}_$v$r.log 2>&1 || { echo "run $v$r failed"; tail -5 gpurun_out/${TAG}_$v$r.log; exit 1; }
    python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); c=d["config"]; print(sys.argv[2], d["value"], d["roofline"]["kernel_ms_per_step"]["mo_band"])' gpurun_out/${TAG}_$v$r.log "$v$r" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
echo ALL_OK
