#!/bin/bash
# Same-box A/B of an environment knob's values: bash tools/x_ab_val.sh TAG VAR "V1 V2 ..." [ROUNDS] ["bench args"]
# ("-" as a value: VAR unset). One line per run -> gpurun_out/TAG_ab.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; VAR=$2; VALS=$3; R=${4:-2}; ARGS=${5:-}
for r in $(seq 1 $R); do
  for v in $VALS; do
    if [ "$v" = "-" ]; then unset $VAR; else export $VAR=$v; fi
    log=gpurun_out/${TAG}_${v}_$r.log
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary $ARGS > $log 2>&1 || { echo "run $v $r failed"; tail -5 $log; exit 1; }
    python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); print(sys.argv[2], d["value"], d["roofline"]["kernel_ms_per_step"]["mo_band"], d["roofline"]["kernel_ms_per_step"].get("replay"))' $log "$VAR=$v#$r" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
unset $VAR
echo ALL_OK
