#!/bin/bash
# One GPU session on the gpurun box, as a list of steps run in order; every GPU step has its own
# time limit and the first failure ends the session (nothing more touches the GPU after it).
#
#   bash tools/gpu.sh TAG STEP...
#
# Steps:
#   tests[=EXPR]      pytest -m gpu (optionally -k EXPR)          -> gpurun_out/TAG_pytest_gpu.log
#                     (+ the image tests' unfloored errors         -> gpurun_out/TAG_parity.jsonl)
#   smoke             __graft_entry__.smoke()                      -> gpurun_out/TAG_smoke.log
#   bench[=CFG]       bench.py --config CFG (c2 default), 5 steps  -> gpurun_out/TAG_bench_CFG.jsonl
#   quick[=CFG]       bench.py, 3 steps, no CPU baseline           -> gpurun_out/TAG_bench_CFG.jsonl
#   mc                tools/bench_mc.py (C4)                       -> gpurun_out/TAG_bench_c4_mc.jsonl
#   pmc_mc            rocprofv3 --pmc SQ_INSTS_VALU of tools/bench_mc.py -> gpurun_out/prof_TAG_c4/pmc_1
#   kt[=CFG]          rocprofv3 --kernel-trace --stats of the bench -> gpurun_out/prof_TAG[_CFG]/kt
#   pmc[=CFG]         rocprofv3 --pmc passes of the bench (one counter set per run, $PMC_SETS
#                     overrides the default sets, one per line)   -> gpurun_out/prof_TAG[_CFG]/pmc_i
# $BENCH_ARGS: extra bench.py arguments for kt and pmc (e.g. "--rgb-profile"). The gather's full counter sets:
#   PMC_SETS="$(cat tools/pmc_sets_gather.txt)" (tools/pmc_sets_replay.txt for the replay generator).
# Afterwards `python tools/summarize_prof.py TAG` writes profiles/TAG_kernel_stats.csv + TAG_pmc.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:?usage: gpu.sh TAG STEP...}
shift
mkdir -p gpurun_out
DEFAULT_PMC="FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"

fail() { echo "$1 failed"; tail -${3:-40} "$2"; exit 1; }
sfx() { [ "$1" = c2 ] && echo "" || echo "_$1"; }

for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  case $name in
    tests)
      log=gpurun_out/${TAG}_pytest_gpu.log
      k=()
      [ -n "$arg" ] && k=(-k "$arg")
      echo "== tests ${arg}"
      MPSS_PARITY_REPORT=gpurun_out/${TAG}_parity.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread "${k[@]}" > $log 2>&1 || fail tests $log 60
      tail -1 $log ;;
    smoke)
      log=gpurun_out/${TAG}_smoke.log
      echo "== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || fail smoke $log
      tail -1 $log ;;
    bench|quick)
      cfg=${arg:-c2}
      log=gpurun_out/${TAG}_bench_${cfg}.log
      extra=(--steps 5 --warmup 1)
      [ $name = quick ] && extra=(--steps 3 --warmup 1 --no-cpu-baseline --no-secondary)
      [ $cfg = c5 ] && extra=(--steps 1 --warmup 1 --no-cpu-baseline)
      echo "== $name $cfg"
      timeout -k 10 600 python -u bench.py --config $cfg "${extra[@]}" > $log 2>&1 || fail bench $log
      grep '"metric"' $log > gpurun_out/${TAG}_bench_${cfg}.jsonl
      python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).readline()); r=d["roofline"]; print(d["value"], d["unit"], d["ms_per_step"], "ms", r["kernel_ms_per_step"], "cpu", (d.get("cpu_baseline") or {}).get("value"))' gpurun_out/${TAG}_bench_${cfg}.jsonl ;;
    mc)
      log=gpurun_out/${TAG}_bench_c4_mc.log
      echo "== mc"
      timeout -k 10 300 python tools/bench_mc.py > $log 2>&1 || fail mc $log
      grep '"metric"' $log > gpurun_out/${TAG}_bench_c4_mc.jsonl; cat gpurun_out/${TAG}_bench_c4_mc.jsonl ;;
    pmc_mc)
      d=gpurun_out/prof_${TAG}_c4
      mkdir -p $d
      echo "== pmc mc"
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $d/pmc_1 -o run --output-format csv -- python3 tools/bench_mc.py --cpu-seconds 0 > $d/pmc_1.log 2>&1 || fail "pmc mc" $d/pmc_1.log 20 ;;
    kt)
      cfg=${arg:-c2}
      d=gpurun_out/prof_${TAG}$(sfx $cfg)
      mkdir -p $d
      steps=(--steps 3 --warmup 1)
      [ $cfg = c5 ] && steps=(--steps 1 --warmup 1)
      echo "== kernel trace $cfg"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $d/kt -o run --output-format csv -- python3 bench.py --config $cfg "${steps[@]}" --no-cpu-baseline --no-secondary $BENCH_ARGS > $d/kt.log 2>&1 || fail kt $d/kt.log 30
      grep '"metric"' $d/kt.log > $d/kt_bench.jsonl || true ;;
    pmc)
      cfg=${arg:-c2}
      d=gpurun_out/prof_${TAG}$(sfx $cfg)
      mkdir -p $d
      i=0
      while read -r line; do
        [ -z "$line" ] && continue
        i=$((i+1))
        echo "== pmc $cfg $i: $line"
        timeout -s KILL 300 rocprofv3 --pmc $line -d $d/pmc_$i -o run --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-secondary $BENCH_ARGS > $d/pmc_$i.log 2>&1 || fail "pmc pass $i" $d/pmc_$i.log 20
      done <<< "${PMC_SETS:-$DEFAULT_PMC}" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo ALL_OK
