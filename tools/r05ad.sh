# round 5: the spread of the final replay generator's task times (MPSS_REPLAY_TASKTIME build), C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
lib=pbrt-v2-skin_amd/mpss/libmpss.so
cp $lib ab/libmpss_keep.so && cp ab/libmpss_T.so $lib && \
timeout -k 10 300 python -u bench.py --sampler reference --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > gpurun_out/r05ad_tasktime.log 2>&1; rc=$?
cp ab/libmpss_keep.so $lib
[ $rc = 0 ] && python3 tools/replay_tasktime.py gpurun_out/r05ad_tasktime.log | tee gpurun_out/r05ad_tasktime_summary.txt
