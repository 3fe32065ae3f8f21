#!/bin/bash
# Timing-only library variants for A/B studies (tools/ablate.py): the render kernel rebuilt from a PATCHED COPY
# of the product sources, linked against the product objects.  Never used for parity or bench numbers.  The
# product sources carry no experiment switches (rp_device.h refuses the old ones); an experiment is a set of
# sed expressions applied to the copy, e.g.
#   tools/build_variant.sh tries3 's/TRIES = 2;/TRIES = 3;/'
#   tools/build_variant.sh prio1  's/PRIO_REFILL = 0/PRIO_REFILL = 1/'
#   tools/build_variant.sh NAME SED_EXPR... [-- EXTRA_HIPCC_FLAGS...]
#      ->  raytracing-potato_amd/lib/librp_NAME.so
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)/raytracing-potato_amd
NAME=$1; shift
SEDS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SEDS+=("-e" "$1"); shift; done
[ "$1" = "--" ] && shift
make -s -C "$HERE" "$HERE/lib/librp.so"
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
cp "$HERE"/csrc/*.h "$HERE"/csrc/rp_kernel.hip "$TMP"/
if [ ${#SEDS[@]} -gt 0 ]; then
  sed -i "${SEDS[@]}" "$TMP/rp_device.h" "$TMP/rp_kernel.hip"
  if diff -q "$HERE/csrc/rp_device.h" "$TMP/rp_device.h" >/dev/null && diff -q "$HERE/csrc/rp_kernel.hip" "$TMP/rp_kernel.hip" >/dev/null; then
    echo "build_variant: the expressions changed nothing" >&2; exit 1
  fi
fi
mkdir -p "$TMP/include" && cp "$HERE"/../include/*.h "$TMP/include/"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -mllvm -disable-machine-licm \
  "$@" -c "$TMP/rp_kernel.hip" -o "$HERE/lib/k_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$HERE/lib/librp_$NAME.so" "$HERE/lib/k_$NAME.o" \
  "$HERE/lib/rp_api.o" "$HERE/lib/rp_bvh_hip.o" "$HERE/lib/rp_bvh_gpu.o" "$HERE/lib/rp_sched.o" \
  "$HERE/lib/rp_id.o" -lrccl
rm -f "$HERE/lib/k_$NAME.o"
