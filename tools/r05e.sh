# round 5, fifth GPU session: the VALU-issue microbenchmark with the round-5 record mix; PMC passes of
# the current gather (tools/pmc_sets_r05e.txt); the texture / render-parity / LayeredSkin-switch tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/valu_issue 4096 > gpurun_out/micro_valu_issue_e.json 2>&1 || { echo valu_issue failed; cat gpurun_out/micro_valu_issue_e.json; exit 1; }
PMC_SETS="$(cat tools/pmc_sets_r05e.txt)" bash tools/gpu.sh r05e kt pmc && \
bash tools/gpu.sh r05e "tests=texture or render_parity or layeredskin"
