# round 5: (1) the L2-width microbenchmark under PMC (L2 requests and TA busy per lane lookup, so the
# gather's TCP_TCC_READ_REQ can be set against the ceiling in the same unit); (2) replay generator
# variants, same box, C2 reference sampler: A the committed camera-hit cache (refilled from the walk's
# hits only), B refilled from every hit, C = B + each sample's own shuffle in registers, D = C with 8
# cached triangles; then the replay tests on C (the in-tree build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r05k_l2w
timeout -s KILL 60 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum -d gpurun_out/prof_r05k_l2w/pmc_1 -o run --output-format csv -- ./tools/microbench/l2_width 256 > gpurun_out/prof_r05k_l2w/pmc_1.log 2>&1 || { echo "l2_width pmc failed"; tail -20 gpurun_out/prof_r05k_l2w/pmc_1.log; exit 1; }
VARIANTS="A B C D" bash tools/ab.sh r05k c2 2 "--sampler reference" && \
bash tools/gpu.sh r05k "tests=replay or reference_sampler"
# (3) the task-time diagnostic build (MPSS_REPLAY_TASKTIME): one reference-sampler C2 frame
lib=pbrt-v2-skin_amd/mpss/libmpss.so
cp $lib ab/libmpss_keep.so && cp ab/libmpss_T.so $lib && \
timeout -k 10 300 python -u bench.py --sampler reference --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > gpurun_out/r05k_tasktime.log 2>&1; rc=$?
cp ab/libmpss_keep.so $lib
[ $rc = 0 ] && python3 tools/replay_tasktime.py gpurun_out/r05k_tasktime.log
