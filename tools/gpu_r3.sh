#!/bin/bash
# Round-3 GPU session: STEPS is a list of tests | bench_C3 | bench_C5 | shards_C3 | shards_C4 | diag_C3 | diag_C5 |
# trace_C3 | trace_C5 | pmc_C3 | pmc_C5, run in order, each under its own time limit, chained (the first
# failure -- a crash, abort or time limit -- ends the session).  TAG names the outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
P=gpurun_out/${TAG}_progress.txt
echo "start $(date +%T)" > $P
step() { echo "$1 $(date +%T)" >> $P; }
pmc() {  # config name counters...
  local cfg=$1 name=$2; shift 2
  step "pmc $cfg $name"
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d gpurun_out/${TAG}_${cfg}_pmc_$name -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/${TAG}_${cfg}_pmc_$name.json 2> gpurun_out/${TAG}_${cfg}_pmc_$name.err
}
for s in ${STEPS:-tests}; do
  case $s in
    tests)
      step tests
      timeout -k 10 ${TESTS_LIMIT:-1200} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
        ${PYTEST_ARGS:-} > gpurun_out/${TAG}_tests.log 2>&1 || { step "tests failed"; exit 1; } ;;
    bench_*)
      cfg=${s#bench_}; st=10; wu=2; [ $cfg = C5 ] && st=3 && wu=1
      step "bench $cfg"
      timeout -k 10 600 python3 bench.py --config $cfg --steps $st --warmup $wu $([ $cfg = C3 ] || echo --no-cpu-baseline) ${BENCH_ARGS:-} \
        > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err || exit 1 ;;
    shards_*)
      cfg=${s#shards_}
      step "shards $cfg"
      timeout -k 10 600 python3 tools/shard_scaling.py --config $cfg --ns ${SHARD_NS:-1,8} --reps ${SHARD_REPS:-3} \
        > gpurun_out/${TAG}_${cfg}_shards.json 2> gpurun_out/${TAG}_${cfg}_shards.err || exit 1 ;;
    diag_*)
      cfg=${s#diag_}
      step "diag $cfg"
      RP_LIB=raytracing-potato_amd/lib/librp_diag.so timeout -k 10 300 python3 tools/diag.py --config $cfg --spp 256 \
        > gpurun_out/${TAG}_${cfg}_diag.json 2> gpurun_out/${TAG}_${cfg}_diag.err || exit 1 ;;
    trace_*)
      cfg=${s#trace_}; st=10; wu=2; [ $cfg = C5 ] && st=3 && wu=1
      step "trace $cfg"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${cfg}_trace -o run --output-format csv -- \
        python3 bench.py --config $cfg --steps $st --warmup $wu --no-cpu-baseline \
        > gpurun_out/${TAG}_${cfg}_bench_under_rocprof.json 2> gpurun_out/${TAG}_${cfg}_trace.err || exit 1 ;;
    pmc_*)
      cfg=${s#pmc_}
      pmc $cfg sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
        SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT &&
      pmc $cfg mix64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
        SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU &&
      pmc $cfg mix32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 \
        SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS &&
      pmc $cfg fetch FETCH_SIZE &&
      pmc $cfg write WRITE_SIZE &&
      pmc $cfg l2 TCC_HIT_sum TCC_MISS_sum || exit 1
      lc=$(echo $cfg | tr A-Z a-z)
      python3 tools/roofline.py --config $cfg --bench gpurun_out/${TAG}_${cfg}_pmc_sq.json \
        $([ -f gpurun_out/${TAG}_${cfg}_diag.json ] && echo --diag gpurun_out/${TAG}_${cfg}_diag.json) \
        --out gpurun_out/${TAG}_${lc}_roofline.json \
        gpurun_out/${TAG}_${cfg}_pmc_sq gpurun_out/${TAG}_${cfg}_pmc_mix64 gpurun_out/${TAG}_${cfg}_pmc_mix32 \
        gpurun_out/${TAG}_${cfg}_pmc_fetch gpurun_out/${TAG}_${cfg}_pmc_write gpurun_out/${TAG}_${cfg}_pmc_l2 \
        > gpurun_out/${TAG}_${cfg}_roofline.log 2>&1 || exit 1 ;;
    *) echo "unknown step $s" >> $P; exit 2 ;;
  esac
done
step done
