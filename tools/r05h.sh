# round 5: the replay generator's sections, each left out in turn (MPSS_REPLAY_SKIP bits, a diagnostic:
# the values are then wrong), on the C2 reference-sampler bench: where a task's time goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/x_ab_val.sh r05h_replay_skip MPSS_REPLAY_SKIP "- 1 2 4 8 16 31" 1 "--sampler reference"
