#!/bin/bash
# Host sanitizer run: CPU only, in the build container.
#   1. make -C raytracing-potato_amd sanitize: the host library and the oracle under ASan + UBSan, and the native driver
#      tools/san_driver.cpp (host + oracle sources linked in) under TSan and under ASan + UBSan;
#   2. both drivers (threaded SAH build / collapse at 1-16 threads, traversal model, OBJ/TGA readers incl. malformed
#      files, threaded bulk StdRng, the oracle's threaded renderer);
#   3. the CPU test suite (pytest -m "not gpu") with the ASan + UBSan builds of librp_host.so and liboracle.so loaded
#      in place of the product ones (RP_HOST_LIB, OR_LIB) and the sanitizer runtimes preloaded into python.
# Logs: $OUT (default profiles/r5/sanitize_*.log).  Exit status 0 = no sanitizer report and every check passed.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-profiles/r5}
mkdir -p "$OUT"
make -s -C raytracing-potato_amd sanitize || exit 1
SAN=raytracing-potato_amd/lib/san
TMPD=$(mktemp -d)
trap 'rm -rf "$TMPD"' EXIT
rc=0
ASAN_OPTIONS=halt_on_error=1:detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  timeout 1800 $SAN/san_asan "$TMPD" > "$OUT/sanitize_driver_asan_ubsan.log" 2>&1 || rc=1
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 \
  timeout 3600 $SAN/san_tsan "$TMPD" > "$OUT/sanitize_driver_tsan.log" 2>&1 || rc=1
# python is not instrumented: the ASan runtime must be loaded first; leak checking would report python's own arenas
PRE="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
LD_PRELOAD="$PRE${LD_PRELOAD:+ $LD_PRELOAD}" ASAN_OPTIONS=halt_on_error=1:detect_leaks=0 \
  UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 RP_HOST_LIB=$SAN/librp_host.so OR_LIB=$SAN/liboracle.so \
  timeout 3600 python -m pytest tests -q -m "not gpu" -p no:cacheprovider -x \
  --deselect tests/test_abi.py::test_profile_records_are_of_this_build \
  > "$OUT/sanitize_pytest_asan_ubsan.log" 2>&1 || rc=1
grep -l "ERROR: AddressSanitizer\|runtime error:\|WARNING: ThreadSanitizer" "$OUT"/sanitize_*.log && rc=1
echo "sanitize: rc=$rc"
exit $rc
