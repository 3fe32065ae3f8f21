#!/bin/bash
# Local (CPU container) check after a kernel edit: build, register report of the render kernel, CPU tests.
#   tools/dev_check.sh [SAVE_AS]   -- SAVE_AS: copy lib/librp.so to lib/librp_SAVE_AS.so for A/B runs
set -o pipefail
cd "$(dirname "$0")/.."
make -s -C raytracing-potato_amd 2>&1 | grep -E "error|warning" && exit 1
make -s -C raytracing-potato_amd resources 2>&1 | grep -A6 "render_kernelILb0" | grep -E "VGPRs|Spill" | sed 's/.*remark: *//'
timeout 900 python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider 2>&1 | tail -1
if [ -n "$1" ]; then cp raytracing-potato_amd/lib/librp.so "raytracing-potato_amd/lib/librp_$1.so"; fi
