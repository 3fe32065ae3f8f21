#!/bin/bash
# PMC passes over one bench frame, one rocprofv3 run per counter group (rocprofv3 does not split passes).
#   TAG=x CONFIG=C3 BENCH_ARGS="..." bash tools/gpu_pmc_passes.sh "name:CTR,CTR,..." ["name2:..."]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
CONFIG=${CONFIG:-C3}
P=gpurun_out/${TAG}_progress.txt
echo start > $P
for set in "$@"; do
  name=${set%%:*}; ctrs=$(echo ${set#*:} | tr ',' ' ')
  echo "pass $name: $ctrs" >> $P
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d gpurun_out/${TAG}_$name -o run --output-format csv -- \
    python3 bench.py --config $CONFIG --steps 1 --warmup 0 --no-cpu-baseline $BENCH_ARGS \
    > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "fail $name" >> $P; exit 1; }
done
echo done >> $P
