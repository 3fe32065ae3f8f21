#!/bin/bash
# Exploration session on the GPU box (not a benchmark): diagnostic phase breakdown, timing A/B of
# library variants (tools/ablate.py), and PMC passes (one counter group per rocprofv3 run) over one
# C3 frame.  Every GPU step has its own time limit; steps are chained with &&.
#   VARIANTS="librp.so librp_w4.so@32" PMC="fetch:FETCH_SIZE write:WRITE_SIZE" TAG=x bash tools/gpu_explore.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-explore}
P=gpurun_out/${TAG}_progress.txt
echo start > $P
ok=0
if [ -n "${DIAG:-1}" ] && [ "${DIAG:-1}" != 0 ]; then
  echo diag >> $P
  timeout -k 10 300 python tools/diag.py --config C3 --spp ${DIAG_SPP:-32} > gpurun_out/${TAG}_diag.json 2> gpurun_out/${TAG}_diag.err || ok=1
fi
if [ $ok = 0 ] && [ -n "$VARIANTS" ]; then
  echo ablate >> $P
  timeout -k 10 900 python tools/ablate.py $VARIANTS > gpurun_out/${TAG}_ablate.json 2> gpurun_out/${TAG}_ablate.err || ok=1
fi
if [ $ok = 0 ] && [ -n "$PMC" ]; then
  for set in $PMC; do
    name=${set%%:*}; ctrs=$(echo ${set#*:} | tr ',' ' ')
    echo "pmc $name: $ctrs" >> $P
    timeout -s KILL 240 rocprofv3 --pmc $ctrs -d gpurun_out/${TAG}_pmc_$name -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_pmc_$name.json 2> gpurun_out/${TAG}_pmc_$name.err || { ok=1; break; }
  done
fi
echo "done $ok" >> $P
exit $ok
