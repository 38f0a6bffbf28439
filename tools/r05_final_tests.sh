# round 5, final: the whole GPU suite and smoke() on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu.sh r05zz tests smoke
