# round 5: the replay generator's MT19937 twist in three dependent phases (M, in-tree) vs one LDS
# round trip per 64 words (L): the replay tests on M, then the reference-sampler C2 frame, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05s "tests=replay or reference_sampler" && \
VARIANTS="L M" bash tools/ab.sh r05s_ref c2 2 "--sampler reference"
