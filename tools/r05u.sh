# round 5: the replay tests with the camera-ray candidate lists' edge geometry (a strip crossing the
# camera plane, a wall over kCamBinMaxArea pixels, triangles behind the camera and off the frame).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu.sh r05u "tests=replay_table"
