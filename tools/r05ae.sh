# round 5: the camera rays' candidate records loaded two (V, in-tree) or four (W) at a time vs one by one
# (Q): the replay tests on V, then the reference-sampler C2 frame, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05ae "tests=replay_table or replay_irradiance or c2_replay_full" && \
VARIANTS="Q V W" bash tools/ab.sh r05ae_ref c2 2 "--sampler reference"
