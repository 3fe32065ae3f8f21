#!/bin/bash
# Build a committed revision's librp.so as raytracing-potato_amd/lib/librp_NAME.so for A/B timing.
#   tools/build_head_variant.sh NAME [REV=HEAD]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=${2:-HEAD}
WT=$(mktemp -d /tmp/rp_wt.XXXXXX)
git -C "$ROOT" worktree add -q "$WT" "$REV"
make -s -C "$WT/raytracing-potato_amd" -j4 >/dev/null
cp "$WT/raytracing-potato_amd/lib/librp.so" "$ROOT/raytracing-potato_amd/lib/librp_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
