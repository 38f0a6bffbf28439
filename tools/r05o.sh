# round 5: H (in-tree) = the RGB gather without the empty fourth slot's lookups and with FromRGB's W row
# in registers, + the replay generator's block swaps in one pass with their partners read ahead;
# F = the previous build. Tests first (replay, reference sampler, rgbprofile, pigment sweep), then
# same-box A/B of the reference-sampler C2 frame and the rgbprofile C2 frame.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r05o "tests=replay or reference_sampler or rgb or pigment" && \
VARIANTS="F H" bash tools/ab.sh r05o_ref c2 2 "--sampler reference" && \
VARIANTS="F H" bash tools/ab.sh r05o_rgb c2 2 "--rgb-profile"
