# round 5, first GPU session: the counter list, the VALU-issue and L2-width microbenchmarks, and the
# kernel trace + PMC passes (tools/pmc_sets_r05.txt) of the current C2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/r05a_counters.txt 2>&1 || echo "list failed"
timeout -k 10 120 ./tools/microbench/valu_issue 4096 > gpurun_out/micro_valu_issue.json 2>&1 || { echo valu_issue failed; cat gpurun_out/micro_valu_issue.json; exit 1; }
cat gpurun_out/micro_valu_issue.json
bash tools/gpu_micro.sh l2_width && \
PMC_SETS="$(cat tools/pmc_sets_r05.txt)" bash tools/gpu.sh r05a kt pmc
