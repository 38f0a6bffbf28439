#!/bin/bash
# Same-box comparison of library builds on image parity and speed: for each V in $VARIANTS,
# ab/libmpss_V.so becomes the in-tree library, then the listed parity tests (pytest -k EXPR, their
# unfloored errors -> gpurun_out/TAG_parity_V.jsonl; $TEST_VARIANTS, if set, instead) and a quick C2
# bench (-> TAG_ab.txt) run.
#   VARIANTS="A B" bash tools/ab_parity.sh TAG "pytest -k expression" [ROUNDS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:?usage: ab_parity.sh TAG EXPR [ROUNDS]}
EXPR=${2:-}
ROUNDS=${3:-1}
mkdir -p gpurun_out
lib=pbrt-v2-skin_amd/mpss/libmpss.so
cp $lib ab/libmpss_orig.so
out=gpurun_out/${TAG}_ab.txt
: > $out
restore() { cp ab/libmpss_orig.so $lib; }
for v in ${TEST_VARIANTS:-${VARIANTS:-A B}}; do
  cp ab/libmpss_$v.so $lib
  if [ -n "$EXPR" ]; then
    log=gpurun_out/${TAG}_pytest_$v.log
    MPSS_PARITY_REPORT=gpurun_out/${TAG}_parity_$v.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$EXPR" > $log 2>&1 || { echo "tests $v failed"; tail -30 $log; restore; exit 1; }
    echo "$v tests: $(tail -1 $log)" | tee -a $out
  fi
done
for r in $(seq 1 $ROUNDS); do
  for v in ${VARIANTS:-A B}; do
    cp ab/libmpss_$v.so $lib
    log=gpurun_out/${TAG}_ab_${v}${r}.log
    timeout -k 10 600 python -u bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $log 2>&1 || { echo "bench $v$r failed"; tail -20 $log; restore; exit 1; }
    python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); print(sys.argv[2], d["value"], d["roofline"]["kernel_ms_per_step"]["mo_band"], d["config"]["mo_l2_footprint"]["per_sss_sample"]["rows"]["lines"], d["config"]["mo_l2_footprint"]["per_sss_sample"]["tables"]["lines"])' $log $v$r | tee -a $out
  done
done
restore
echo ALL_OK
