#!/bin/bash
# Timing-only library variants for ablation studies (tools/ablate.py): the render kernel rebuilt with
# extra -D flags, linked against the product objects.  Never used for parity or bench numbers.
#   tools/build_variant.sh NAME [-DFLAG ...]   ->  raytracing-potato_amd/lib/librp_NAME.so
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)/raytracing-potato_amd
NAME=$1; shift
make -s -C "$HERE" "$HERE/lib/librp.so"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -mllvm -disable-machine-licm \
  "$@" -c "$HERE/csrc/rp_kernel.hip" -o "$HERE/lib/k_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$HERE/lib/librp_$NAME.so" "$HERE/lib/k_$NAME.o" \
  "$HERE/lib/rp_wavefront.o" "$HERE/lib/rp_api.o" "$HERE/lib/rp_bvh_hip.o" "$HERE/lib/rp_bvh_gpu.o" -lrccl
rm -f "$HERE/lib/k_$NAME.o"
