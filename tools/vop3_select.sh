#!/bin/bash
# Compile a HIP source to a host object whose gfx950 code object has every lane select in the VOP3 encoding.
#
#   vop3_select.sh "HIPCC FLAGS..." ARCH SRC OUT
#
# Experiment only (not in the Makefile; profiles/r6/c3_c5_vop3_select_ab.json: C3 +0.1 %, C5 -0.7 %).
# Why (profiles/r6/valu_rates_gfx950.json, select_probe_gfx950.json): on gfx950 a VOP2 v_cndmask_b32 -- the mask implicit in VCC,
# the encoding LLVM's SIShrinkInstructions picks whenever the mask was allocated to VCC -- occupies the SIMD for ~23 cycles
# per wave-instruction, against ~4 for the same select in the VOP3 encoding (VCC or any SGPR pair as an explicit third
# operand).  tools/select_probe.hip times the render kernel's 4-wide sorting network at 390 SIMD cycles compiled from C
# and 105 with VOP3 selects.  LLVM has no switch to keep the VOP3 form, so the device code goes through assembly:
#   1. the device compile stops at assembly (same flags, -S --cuda-device-only);
#   2. each `v_cndmask_b32_e32 vD, src0, vS1, vcc` becomes `v_cndmask_b32_e64 vD, src0, vS1, vcc` -- the same
#      instruction (same operands, same VCC read, same hazard waits the compiler placed), another encoding; the other
#      VOP2 carry-in forms that read VCC (v_addc/v_subb/v_subbrev_co_u32) likewise; a VOP2 src0 literal would not
#      encode in VOP3 on gfx9 and the assembler would refuse it (none occurs: the compiler keeps literals in registers
#      for selects);
#   3. the assembly is assembled and linked into the code object, bundled as hipcc bundles it, and the host side is
#      compiled around it (-fcuda-include-gpubinary), so the object is a drop-in for `hipcc -c` (kernel registration,
#      the build id's .hip_fatbin section).
set -e -o pipefail
HIPCC_FLAGS=$1
ARCH=$2
SRC=$3
OUT=$4
LLVM_BIN=${LLVM_BIN:-/opt/rocm/lib/llvm/bin}
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
# shellcheck disable=SC2086
$HIPCC_FLAGS --cuda-device-only -S "$SRC" -o "$tmp/dev.s" 2> >(grep -v "hip-link" >&2)
sed -E -e 's/^(\s+)v_cndmask_b32_e32 (v[0-9]+), ([^,]+), (v[0-9]+), vcc$/\1v_cndmask_b32_e64 \2, \3, \4, vcc/' \
       -e 's/^(\s+)v_(addc|subb|subbrev)_co_u32_e32 /\1v_\2_co_u32_e64 /' "$tmp/dev.s" > "$tmp/dev3.s"
if grep -qE '^\s+v_cndmask_b32_e32' "$tmp/dev3.s"; then
  echo "vop3_select.sh: a VOP2 v_cndmask_b32 form the rewrite does not cover:" >&2
  grep -m3 -E '^\s+v_cndmask_b32_e32' "$tmp/dev3.s" >&2
  exit 1
fi
"$LLVM_BIN/clang" -x assembler -target amdgcn-amd-amdhsa -mcpu="$ARCH" -c "$tmp/dev3.s" -o "$tmp/dev.o"
"$LLVM_BIN/lld" -flavor gnu -m elf64_amdgpu --no-undefined -shared -o "$tmp/dev.co" "$tmp/dev.o"
"$LLVM_BIN/clang-offload-bundler" -type=o -bundle-align=4096 \
  -targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--"$ARCH" -input=/dev/null -input="$tmp/dev.co" \
  -output="$tmp/dev.hipfb"
# shellcheck disable=SC2086
$HIPCC_FLAGS --cuda-host-only -Xclang -fcuda-include-gpubinary -Xclang "$tmp/dev.hipfb" -c "$SRC" -o "$OUT" \
  2> >(grep -v "hip-link" >&2)
