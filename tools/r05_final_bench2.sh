# round 5, final measurements (2): C3 and C5 on one GPU; the scalar-cache counters of the BVH kernels
# at C2 and C5 (the nodelet question); kernel trace of the reference-sampler C2 frame.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05z bench=c3 bench=c5 && \
PMC_SETS="SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_INSTS_SMEM" bash tools/gpu.sh r05z_sqc pmc pmc=c5 && \
BENCH_ARGS="--sampler reference" bash tools/gpu.sh r05z_ref kt && \
# and where the replay generator's time goes on the final tree (each section of the pixel loop left out)
bash tools/x_ab_val.sh r05z_skip MPSS_REPLAY_SKIP "- 1 2 4 8 16" 1 "--sampler reference"
