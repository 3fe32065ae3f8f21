#!/bin/bash
# One-off A/B: the learned per-unit order of round 5 (rp_sched.hip, removed from librp in round 6)
# with its bucket bug fixed.  Runs in a side checkout of the round-5 tree (_old/ = `git worktree add _old ce41b3f`,
# libraries built there: lib/librp.so = the round-5 product build 8bb994a1752f1509, lib/librp_uofix.so = the same with
# the unit keys' bucket widened to 8 bits -- log2(duration) * 4 + 1 clamped at 254 instead of 63, radix end bit 40), one
# lone frame per launch (the learned order applies to n_frames == 1 only), interleaved reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT/_old"
out=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-uo}
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
for rep in 1 2; do
  for run in "tiles256:librp:--samples-per-stream 256" "uo256:librp:--samples-per-stream 256 --opt unit_order=learned" \
             "uofix256:librp_uofix:--samples-per-stream 256 --opt unit_order=learned" \
             "tiles32:librp:" "uofix32:librp_uofix:--opt unit_order=learned"; do
    name=${run%%:*}; rest=${run#*:}; lib=${rest%%:*}; args=${rest#*:}
    echo "$name rep $rep $(date +%T)" >> ${out}_progress.txt
    RP_LIB=raytracing-potato_amd/lib/$lib.so timeout -k 10 300 python3 bench.py --config C3 --steps 4 --warmup 4 \
      --frames-per-launch 1 --contract-steps 0 --no-cpu-baseline $args > ${out}_${name}_$rep.json 2> ${out}_${name}_$rep.err || exit 1
  done
done
