#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1
for set in "${@}"; do
  name=$(echo $set | cut -d: -f1); ctrs=$(echo $set | cut -d: -f2 | tr ',' ' ')
  echo "pass $name: $ctrs" >> gpurun_out/${TAG}_progress.txt
  timeout -k 10 240 rocprofv3 --pmc $ctrs -d gpurun_out/${TAG}_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --spp ${SPP:-0} --no-cpu-baseline > /dev/null 2> gpurun_out/${TAG}_$name.err || { echo "fail $name" >> gpurun_out/${TAG}_progress.txt; exit 1; }
done
