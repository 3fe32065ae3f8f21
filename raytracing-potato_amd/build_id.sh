#!/bin/bash
# rp_build_id: a hash of the machine code that decides a frame's per-ray work (see the Makefile).
#
#   build_id.sh ARCH DEVICE_OBJ... -- HOST_OBJ...
#
# DEVICE_OBJ: a hipcc object whose .hip_fatbin bundle holds the ARCH code object -- its .text (instructions) and
# .rodata (kernel descriptors) are hashed.  HOST_OBJ: a host object -- its .text is hashed.  Nothing that names the
# build enters the hash: the bundle itself embeds a `__hip_cuid_<hash>` symbol derived from the object's path, so
# hashing the whole .hip_fatbin gave every checkout directory its own id.  Prints 16 hex digits.
set -e -o pipefail
ARCH=$1; shift
LLVM_BIN=${LLVM_BIN:-/opt/rocm/lib/llvm/bin}
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
n=0
parts=()
dev=1
for o in "$@"; do
  if [ "$o" = "--" ]; then dev=0; continue; fi
  n=$((n + 1))
  if [ $dev = 1 ]; then
    objcopy -O binary --only-section=.hip_fatbin "$o" "$tmp/$n.fat"
    "$LLVM_BIN/clang-offload-bundler" --unbundle --type=o --input="$tmp/$n.fat" \
      --targets="hipv4-amdgcn-amd-amdhsa--$ARCH" --output="$tmp/$n.co"
    "$LLVM_BIN/llvm-objcopy" -O binary --only-section=.text "$tmp/$n.co" "$tmp/$n.text"
    "$LLVM_BIN/llvm-objcopy" -O binary --only-section=.rodata "$tmp/$n.co" "$tmp/$n.rodata"
    parts+=("$tmp/$n.text" "$tmp/$n.rodata")
  else
    objcopy -O binary --only-section=.text "$o" "$tmp/$n.text"
    parts+=("$tmp/$n.text")
  fi
done
cat "${parts[@]}" | sha256sum | cut -c1-16
