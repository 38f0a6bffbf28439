# round 5, third GPU session: the extended VALU-issue microbenchmark; a same-box A/B of the per-path
# lerp parameters (ab/libmpss_A.so: MPSS_MO_TPATH=0, B: the default; both fused); textured and
# rgbprofile quick benches; then the whole -m gpu suite on B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/valu_issue 4096 > gpurun_out/micro_valu_issue_c.json 2>&1 || { echo valu_issue failed; cat gpurun_out/micro_valu_issue_c.json; exit 1; }
bash tools/ab.sh r05c_tpath c2 2 && \
BENCH_ARGS="--scene scenes/skin_textured.pbrt" timeout -k 10 300 python -u bench.py --scene scenes/skin_textured.pbrt --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05c_bench_textured.log 2>&1 && \
timeout -k 10 300 python -u bench.py --rgb-profile --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05c_bench_rgb.log 2>&1 && \
bash tools/gpu.sh r05c tests
