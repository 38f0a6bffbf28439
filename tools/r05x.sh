# round 5: camera-ray candidate lists tightened to the pixels a triangle's projection meets (not its
# whole box) and ordered by projected area (Q, in-tree) vs the box lists in index order (P): the replay
# tests on Q, then the reference-sampler C2 frame, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05x "tests=replay or reference_sampler" && \
VARIANTS="P Q" bash tools/ab.sh r05x_ref c2 2 "--sampler reference"
