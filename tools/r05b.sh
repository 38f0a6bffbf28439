# round 5, second GPU session: the corrected VALU-issue microbenchmark; a same-box A/B of the
# common-grid gather's fused arithmetic (ab/libmpss_A.so: MPSS_MO_FUSED=0, B: the default); then the
# whole -m gpu suite on B (pigment sweep, end-to-end independent C2/C3/C5, reference-sampler full
# frame, LayeredSkin switches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/valu_issue 4096 > gpurun_out/micro_valu_issue_b.json 2>&1 || { echo valu_issue failed; cat gpurun_out/micro_valu_issue_b.json; exit 1; }
bash tools/ab.sh r05b_fused c2 2 && \
bash tools/gpu.sh r05b tests
