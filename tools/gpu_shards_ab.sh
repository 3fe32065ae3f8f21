#!/bin/bash
# 8-way shard times (tools/shard_scaling.py, balanced plan, frames in flight) for library variants LIBS ("name:lib").
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for run in ${LIBS:-main:main}; do
  name=${run%%:*}; lib=${run#*:}
  libpath=raytracing-potato_amd/lib/librp.so; [ "$lib" != main ] && libpath=raytracing-potato_amd/lib/librp_$lib.so
  RP_LIB=$libpath timeout -k 10 300 python3 tools/shard_scaling.py --config ${CFG:-C3} --ns ${SHARD_NS:-8} --maps balanced \
    --reps ${SHARD_REPS:-3} --inflight ${INFLIGHT:-3} > gpurun_out/${TAG:-sh}_${name}.json 2> gpurun_out/${TAG:-sh}_${name}.err || exit 1
done
