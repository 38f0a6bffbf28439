#!/bin/bash
# Same-box A/B of two builds of libmpss.so (box-to-box spread is a few per cent, more than the
# variants under test): ab/libmpss_A.so and ab/libmpss_B.so take turns as the in-tree library,
# (or ab/libmpss_V.so for each V in $VARIANTS) each running the quick bench of CFG (c4: tools/bench_mc.py), ROUNDS times; one line per run -> gpurun_out/TAG_ab.txt.
#
#   bash tools/ab.sh TAG [CFG] [ROUNDS] ["extra bench.py args"]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:?usage: ab.sh TAG [CFG] [ROUNDS]}
CFG=${2:-c2}
ROUNDS=${3:-2}
EXTRA_ARGS=${4:-}
mkdir -p gpurun_out
lib=pbrt-v2-skin_amd/mpss/libmpss.so
cp $lib ab/libmpss_orig.so
out=gpurun_out/${TAG}_ab.txt
: > $out
steps=(--steps 3 --warmup 1)
[ $CFG = c5 ] && steps=(--steps 1 --warmup 1)
for r in $(seq 1 $ROUNDS); do
  for v in ${VARIANTS:-A B}; do
    cp ab/libmpss_$v.so $lib
    log=gpurun_out/${TAG}_ab_${v}${r}.log
    if [ $CFG = c4 ]; then
      timeout -k 10 300 python -u tools/bench_mc.py --cpu-seconds 0 > $log 2>&1 || { echo "run $v$r failed"; tail -20 $log; cp ab/libmpss_orig.so $lib; exit 1; }
      python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); print(sys.argv[2], d["value"], d["seconds"], d["total_r"], d["total_t"])' $log $v$r | tee -a $out
    else
      timeout -k 10 600 python -u bench.py --config $CFG "${steps[@]}" --no-cpu-baseline --no-secondary $EXTRA_ARGS > $log 2>&1 || { echo "run $v$r failed"; tail -20 $log; cp ab/libmpss_orig.so $lib; exit 1; }
      python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); print(sys.argv[2], d["value"], d["roofline"]["kernel_ms_per_step"])' $log $v$r | tee -a $out
    fi
  done
done
cp ab/libmpss_orig.so $lib
echo ALL_OK
