# round 5: the replay generator's camera rays tested against per-pixel candidate triangles (scene.h
# CameraBins) instead of the BVH walk: E (in-tree) vs B (the walk behind a 4-triangle hit cache), same
# box, C2 reference sampler; then the replay tests on E.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05l "tests=replay or reference_sampler" && \
VARIANTS="B E" bash tools/ab.sh r05l c2 2 "--sampler reference"
