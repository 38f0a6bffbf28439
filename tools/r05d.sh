# round 5, fourth GPU session: same-box A/B of the lazy per-band indices (ab/libmpss_A.so:
# MPSS_MO_LAZYF=0, B: the default); the textured bench (assemble's textured fast path); the texture
# and render parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab.sh r05d_lazyf c2 2 && \
timeout -k 10 300 python -u bench.py --scene scenes/skin_textured.pbrt --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05d_bench_textured.log 2>&1 && \
bash tools/gpu.sh r05d "texture or render_parity or layeredskin"
