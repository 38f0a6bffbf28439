#!/bin/bash
# r02aw: kernel trace of the dual-kernel gather experiment (do the no-LDS waves run beside the
# near-field workgroups?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/prof_r02aw
export TMPDIR=/tmp MPSS_MO_DUAL=32
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_r02aw/kt -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_r02aw/kt.log 2>&1 || { echo "kt failed"; tail -5 gpurun_out/prof_r02aw/kt.log; exit 1; }
python3 - <<'PY'
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/prof_r02aw/kt/run_kernel_trace.csv')) if 'wave_kernel<false' in r['Kernel_Name']]
for r in rows[-4:]:
    print(r['Kernel_Name'][:60], int(r['Start_Timestamp'])//1000, int(r['End_Timestamp'])//1000, (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6, 'ms')
PY
