# round 5: the MT19937 twist's ten 64-word blocks unrolled (S, in-tree: the wrap selects resolved at
# compile time) vs looped (Q): the replay tests on S, then the reference-sampler C2 frame, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05ac "tests=replay_table or replay_irradiance" && \
VARIANTS="Q S" bash tools/ab.sh r05ac_ref c2 2 "--sampler reference"
