# round 5: the rgbprofile grid's knot errors relative to the largest of R, G, B (L, in-tree) vs their own
# value (K): the rgb tests on L, then the rgbprofile C2 frame, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05r "tests=rgb or pigment" && \
VARIANTS="K L" bash tools/ab.sh r05r_rgb c2 2 "--rgb-profile"
