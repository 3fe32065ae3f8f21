#!/bin/bash
# A/B timing of library variants and options on one box, interleaved (RUNS: "name:lib:opts" with lib = the
# suffix of lib/librp_<lib>.so or "main" and opts = bench.py --opt field=value,...), REPS rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-ab}
CFG=${CFG:-C3}
P=gpurun_out/${TAG}_progress.txt
echo "start $(date +%T)" > $P
for rep in $(seq 1 ${REPS:-2}); do
  for run in $RUNS; do
    name=${run%%:*}; rest=${run#*:}; lib=${rest%%:*}; opts=${rest#*:}
    args=""
    for o in $(echo $opts | tr ',' ' '); do args="$args --opt $o"; done
    libpath=raytracing-potato_amd/lib/librp.so
    [ "$lib" != main ] && libpath=raytracing-potato_amd/lib/librp_$lib.so
    echo "$rep $name $(date +%T)" >> $P
    RP_LIB=$libpath timeout -k 10 300 python3 bench.py --config $CFG --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline $args \
      > gpurun_out/${TAG}_${name}_$rep.json 2> gpurun_out/${TAG}_${name}_$rep.err || exit 1
  done
done
echo done >> $P
