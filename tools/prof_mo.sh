set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 200 python tools/bench_mo.py --iters 2 --queries 2097152 > gpurun_out/prof/packet.json
timeout -k 10 200 python tools/bench_mo.py --iters 2 --queries 2097152 --exact > gpurun_out/prof/exact.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o run --output-format csv -- python3 tools/bench_mo.py --iters 2 --queries 2097152 > gpurun_out/prof/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/prof/pmc1 -o run --output-format csv -- python3 tools/bench_mo.py --iters 1 --queries 2097152 > gpurun_out/prof/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/prof/pmc2 -o run --output-format csv -- python3 tools/bench_mo.py --iters 1 --queries 2097152 > gpurun_out/prof/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc3 -o run --output-format csv -- python3 tools/bench_mo.py --iters 1 --queries 2097152 > gpurun_out/prof/pmc3.log 2>&1
