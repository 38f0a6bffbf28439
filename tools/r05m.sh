# round 5: the replay generator writes the light-sample values only of samples whose camera ray hits
# (F, in-tree) vs every sample's (E); replay / reference-sampler / render-parity tests on F first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05m "tests=replay or reference_sampler" && \
VARIANTS="E F" bash tools/ab.sh r05m c2 2 "--sampler reference"
