#!/bin/bash
# One GPU session of this round: the -m gpu suite on the current build, then interleaved A/B runs of library
# variants (tools/gpu_ab_r3.sh) for each config in AB_CFGS ("C3:reps:steps C5:reps:steps").  Chained: the first
# failure ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-s}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  TAG=$T STEPS=tests TESTS_LIMIT=${TESTS_LIMIT:-400} bash tools/gpu_r3.sh || exit 1
fi
for c in ${AB_CFGS:-C3:3:8}; do
  cfg=${c%%:*}; rest=${c#*:}; reps=${rest%%:*}; st=${rest#*:}
  TAG=${T}_${cfg} CFG=$cfg REPS=$reps STEPS=$st bash tools/gpu_ab_r3.sh || exit 1
done
