# round 5: I (in-tree) = H without FromRGB's W row held in registers (that pushed the rgbprofile
# gather's 64 VGPRs into a spill): rgbprofile C2 frame, same box, F / H / I; then the rgb tests on I.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="F I H" bash tools/ab.sh r05p_rgb c2 2 "--rgb-profile" && \
bash tools/gpu.sh r05p "tests=rgb or pigment"
