set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh r04b tests="test_mo_gpu or test_golden_gpu or test_configs_gpu" smoke || exit 1
for cg in 1 0 1 0; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --common-grid $cg > gpurun_out/r04b_ab_cg$cg.log 2>&1 || { echo "bench cg=$cg failed"; tail -20 gpurun_out/r04b_ab_cg$cg.log; exit 1; }
  python3 -c 'import json,sys; d=json.loads([l for l in open(sys.argv[1]) if "\"metric\"" in l][0]); c=d["config"]; print("cg", sys.argv[2], d["value"], d["roofline"]["kernel_ms_per_step"], c["mo_common_grid"], c["mo_lane_records"], c["mo_lookups_in_profile"] if "mo_lookups_in_profile" in c else "")' gpurun_out/r04b_ab_cg$cg.log $cg | tee -a gpurun_out/r04b_ab.txt
done
echo ALL_OK
