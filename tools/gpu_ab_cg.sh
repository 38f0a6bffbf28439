# Same-box A/B of the Mo() gather's common grid (mpss_config.mo_common_grid 1 vs 0) on the C2 bench,
# after the gather and parity GPU tests (SKIP_TESTS=1 skips them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r04b}
if [ -z "$SKIP_TESTS" ]; then
  bash tools/gpu.sh $TAG tests="test_mo_gpu or test_golden_gpu or test_configs_gpu or test_c_abi_client" smoke || exit 1
fi
for cg in 1 0 1 0; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --common-grid $cg > gpurun_out/${TAG}_ab_cg$cg.log 2>&1 || { echo "bench cg=$cg failed"; tail -20 gpurun_out/${TAG}_ab_cg$cg.log; exit 1; }
  python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); c=d["config"]; print("cg", sys.argv[2], d["value"], d["roofline"]["kernel_ms_per_step"], c["mo_common_grid"], c["mo_lane_records"])' gpurun_out/${TAG}_ab_cg$cg.log $cg | tee -a gpurun_out/${TAG}_ab.txt
done
echo ALL_OK
