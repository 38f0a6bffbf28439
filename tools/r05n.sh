# round 5: where the replay generator's time goes after the camera-ray bins: the launch with each
# section of the pixel loop left out (MPSS_REPLAY_SKIP bits: 1 own shuffles + partners, 2 block swaps,
# 8 light values, 16 draw copies), and the task-time diagnostic build's spread of task times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/x_ab_val.sh r05n_skip MPSS_REPLAY_SKIP "- 1 2 4 8 16" 1 "--sampler reference" || exit 1
lib=pbrt-v2-skin_amd/mpss/libmpss.so
cp $lib ab/libmpss_keep.so && cp ab/libmpss_T.so $lib && \
timeout -k 10 300 python -u bench.py --sampler reference --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > gpurun_out/r05n_tasktime.log 2>&1; rc=$?
cp ab/libmpss_keep.so $lib
[ $rc = 0 ] && python3 tools/replay_tasktime.py gpurun_out/r05n_tasktime.log
