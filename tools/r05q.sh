# round 5: reference-sampler C2 frame, same box: I vs J (in-tree: each sample's own shuffle of 4 values
# in one register); the replay tests on J first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05q "tests=replay or reference_sampler" && \
VARIANTS="I J" bash tools/ab.sh r05q_ref c2 2 "--sampler reference"
