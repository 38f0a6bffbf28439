# round 5: after the host grid builder's threading (the kernel sources' hash changed, their code did
# not): the gather / rgbprofile / full-frame tests, then kernel trace + PMC passes on the final sources
# and the default bench line that reads them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05w "tests=test_mo_ or rgb or pigment or full_frame or common_grid" || exit 1
T=r05y
PMC_SETS="$(cat tools/pmc_sets_r05e.txt)" bash tools/gpu.sh $T kt pmc || exit 1
python3 tools/summarize_prof.py $T || exit 1
bash tools/gpu.sh $T bench
