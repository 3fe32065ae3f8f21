#!/bin/bash
# One measured GPU-box session: parity tests, the bench line (with the CPU baseline), a rocprofv3
# kernel-trace summary of the bench, and the PMC passes tools/roofline.py turns into the per-ray record
# bench.py prices its roofline with.  Every GPU step has its own time limit; steps are chained with &&.
#   TAG=r2a CONFIGS="C3 C5" TESTS=1 bash tools/gpu_round.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-round}
CONFIGS=${CONFIGS:-C3}
P=gpurun_out/${TAG}_progress.txt
echo start > $P
run_tests() {
  [ "${TESTS:-1}" = 0 ] && return 0
  echo tests >> $P
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1
}
pmc() {  # config name counters...
  local cfg=$1 name=$2; shift 2
  echo "pmc $cfg $name: $*" >> $P
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d gpurun_out/${TAG}_${cfg}_pmc_$name -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/${TAG}_${cfg}_pmc_$name.json 2> gpurun_out/${TAG}_${cfg}_pmc_$name.err
}
per_config() {
  local cfg=$1 steps=10 warm=2
  [ $cfg = C5 ] && steps=3 && warm=1
  echo "bench $cfg" >> $P
  timeout -k 10 600 python3 bench.py --config $cfg --steps $steps --warmup $warm $([ $cfg = C3 ] || echo --no-cpu-baseline) \
    > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err &&
  echo "trace $cfg" >> $P &&
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${cfg}_trace -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps $steps --warmup $warm --no-cpu-baseline \
    > gpurun_out/${TAG}_${cfg}_bench_under_rocprof.json 2> gpurun_out/${TAG}_${cfg}_trace.err &&
  pmc $cfg sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT &&
  pmc $cfg mix64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
    SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU &&
  pmc $cfg mix32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 \
    SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS &&
  pmc $cfg fetch FETCH_SIZE &&
  pmc $cfg write WRITE_SIZE &&
  pmc $cfg l2 TCC_HIT_sum TCC_MISS_sum &&
  python3 tools/roofline.py --config $cfg --bench gpurun_out/${TAG}_${cfg}_pmc_sq.json \
    --out gpurun_out/${TAG}_$(echo $cfg | tr A-Z a-z)_roofline.json \
    gpurun_out/${TAG}_${cfg}_pmc_sq gpurun_out/${TAG}_${cfg}_pmc_mix64 gpurun_out/${TAG}_${cfg}_pmc_mix32 \
    gpurun_out/${TAG}_${cfg}_pmc_fetch gpurun_out/${TAG}_${cfg}_pmc_write gpurun_out/${TAG}_${cfg}_pmc_l2 \
    > gpurun_out/${TAG}_${cfg}_roofline.log 2>&1
}
ok=0
run_tests; rc=$?
echo "tests rc $rc" >> $P
# a failed assertion (pytest rc 1) still lets the measurements run; a crash, abort or time limit does not
[ $rc = 0 ] || [ $rc = 1 ] || ok=1
if [ $ok = 0 ]; then
  for cfg in $CONFIGS; do per_config $cfg || { ok=1; break; }; done
fi
echo "done $ok" >> $P
exit $ok
