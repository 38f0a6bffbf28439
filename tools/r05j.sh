# round 5, final gather profile: kernel trace + PMC passes (tools/pmc_sets_r05e.txt) of the gather as
# committed, the default C2 bench line (CPU baseline, reference-sampler secondary), and the replay
# generator's camera-trace cost with the hit cache (MPSS_REPLAY_SKIP=4 leaves the trace out).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_SETS="$(cat tools/pmc_sets_r05e.txt)" bash tools/gpu.sh r05j kt pmc bench && \
bash tools/x_ab_val.sh r05j_skip MPSS_REPLAY_SKIP "- 4" 1 "--sampler reference"
