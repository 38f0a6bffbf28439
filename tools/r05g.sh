# round 5: same-box A/B of the multiply-based dw test (ab/libmpss_A.so: MPSS_MO_DWMUL=0, B: default);
# the rgbprofile bench (fused FromRGB on the grid); the replay generator's section profile
# (ab/libmpss_rp.so, MPSS_REPLAY_PROFILE) on the C2 reference-sampler bench; Mo and rgbprofile tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab.sh r05g_dwmul c2 2 && \
timeout -k 10 300 python -u bench.py --rgb-profile --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05g_bench_rgb.log 2>&1 && \
bash tools/gpu.sh r05g "tests=test_mo_gpu or rgbprofile or golden" && \
cp pbrt-v2-skin_amd/mpss/libmpss.so ab/libmpss_keep.so && cp ab/libmpss_rp.so pbrt-v2-skin_amd/mpss/libmpss.so && \
{ timeout -k 10 300 python -u bench.py --sampler reference --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r05g_replay_profile.log 2>&1; rc=$?; cp ab/libmpss_keep.so pbrt-v2-skin_amd/mpss/libmpss.so; exit $rc; }
