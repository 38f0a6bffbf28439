# The common grid's absolute error floor (MPSS_CG_ABS_TOL, relative to each band's peak) against
# the full-frame C2 parity and the C2 bench: one line per value.
#   bash tools/gpu_abstol.sh TAG "1e-10 1e-13 0"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
for v in $2; do
  echo "== abs tol $v"
  MPSS_CG_ABS_TOL=$v MPSS_PARITY_REPORT=gpurun_out/${TAG}_abstol_${v}_parity.jsonl timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -x -q --timeout 380 --timeout-method thread -k full_frame > gpurun_out/${TAG}_abstol_${v}_pytest.log 2>&1
  tail -1 gpurun_out/${TAG}_abstol_${v}_pytest.log
  MPSS_CG_ABS_TOL=$v timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_abstol_${v}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${TAG}_abstol_${v}_bench.log; exit 1; }
  grep '"metric"' gpurun_out/${TAG}_abstol_${v}_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["roofline"]["kernel_ms_per_step"]["mo_band"])'
done
echo ALL_OK
