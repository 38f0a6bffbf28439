# round 5: the block shuffles of up to 64 samples walked forward across the lanes (R, in-tree) vs each
# on its own lane through LDS (Q): the replay tests on R, then the reference-sampler C2 frame, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05aa "tests=replay or reference_sampler" && \
VARIANTS="Q R" bash tools/ab.sh r05aa_ref c2 2 "--sampler reference"
