# round 5: the common-grid Mo() test with its unfloored per-query bound
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu.sh r05v "tests=test_mo_common_grid_vs_oracle"
