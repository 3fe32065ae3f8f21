#!/bin/bash
# Interleaved A/B bench runs on one GPU box: each argument is "label|CONFIG|STEPS|LIB|extra bench args"
# (LIB empty = the product librp.so; else a variant under raytracing-potato_amd/lib/).  Every run has its own
# time limit; the first failure ends the script.
#   TAG=x bash tools/gpu_abrun.sh "new|C3|5||" "old|C3|5|librp_f32node.so|" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-abrun}
P=gpurun_out/${TAG}_progress.txt
echo start > $P
for run in "$@"; do
  IFS='|' read -r label cfg steps lib extra <<< "$run"
  echo "run $label" >> $P
  if [ -n "$lib" ]; then export RP_LIB=$PWD/raytracing-potato_amd/lib/$lib; else unset RP_LIB; fi
  timeout -k 10 400 python3 bench.py --config $cfg --steps $steps --warmup 1 --no-cpu-baseline $extra \
    > gpurun_out/${TAG}_$label.json 2> gpurun_out/${TAG}_$label.err || { echo "fail $label" >> $P; exit 1; }
done
echo done >> $P
