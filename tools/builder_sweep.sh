#!/bin/bash
# C5 tree quality of the device builders: bvh_build_time.py under library variants (LIBS: lib suffixes, main = librp.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in ${LIBS:-main}; do
  p=raytracing-potato_amd/lib/librp.so; [ $lib != main ] && p=raytracing-potato_amd/lib/librp_$lib.so
  RP_LIB=$p timeout -k 10 600 python3 tools/bvh_build_time.py --spp ${SPP:-32} --builders ${BUILDERS:-ploc:q8} \
    > gpurun_out/${TAG:-bs}_$lib.json 2> gpurun_out/${TAG:-bs}_$lib.err || exit 1
done
