#!/bin/bash
# Quick measurement loop on the GPU box: optional parity subset, then the C3 bench line (no CPU baseline)
# and, with PMC=1, the SQ cycle-budget pass.  Every GPU step has its own time limit; chained with &&.
#   TAG=x TESTS="tests/test_gpu_parity.py" PMC=1 bash tools/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
P=gpurun_out/${TAG}_progress.txt
echo start > $P
ok=0
if [ -n "$TESTS" ]; then
  echo tests >> $P
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
  echo "tests rc $rc" >> $P
  [ $rc = 0 ] || [ $rc = 1 ] || ok=1
fi
for cfg in ${CONFIGS:-C3}; do
  [ $ok = 0 ] || break
  echo "bench $cfg" >> $P
  timeout -k 10 600 python3 bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline $BENCH_ARGS \
    > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err || { ok=1; break; }
  if [ -n "$PMC" ]; then
    echo "pmc $cfg" >> $P
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/${TAG}_${cfg}_pmc_sq \
      -o run --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline $BENCH_ARGS \
      > gpurun_out/${TAG}_${cfg}_pmc_sq.json 2> gpurun_out/${TAG}_${cfg}_pmc_sq.err || { ok=1; break; }
  fi
done
echo "done $ok" >> $P
exit $ok
