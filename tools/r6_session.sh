#!/bin/bash
# Round 6's measurement session (one gpurun call; each part a tools/gpu_session.sh run with its own tag, stopping at the
# first failure).  PART selects a subset: all (default), final, sweep.
#   final: pytest -m gpu; the bench line (C3, one-stream contract, CPU baseline); rocprofv3 kernel traces of it and of
#          the driver's command; diag + six PMC passes for the C3 record under one stream per pixel (key C3) and under
#          32-sample streams (key C3@32, the N > 1 runs); diag + PMC for C5 in 32-sample streams (key C5@32)
#   sweep: the learned unit order on frame launches, traversal knobs and the leaf-loop break on the one-stream headline,
#          interleaved reps
#   shards: the one-stream contract's 8-way shard cost on this build, and the projected N-GPU scaling of bench.py's N > 1
#          loop (every shard of N = 1, 2, 4, 8 on one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
P=${PART:-all}
T=${TAGP:-q6}
S=tools/gpu_session.sh
if [ "$P" = all ] || [ "$P" = final ]; then
  TAG=${T}t STEPS="tests" bash $S || exit 1
  TAG=${T}b STEPS="bench_C3 trace_C3 tracedrv_C3" BENCH_ARGS="--steps 20 --warmup 5" bash $S || exit 1
  TAG=${T}p STEPS="diag_C3 pmc_C3" DIAG_ARGS="--sps 256" bash $S || exit 1
  TAG=${T}q STEPS="diag_C3 pmc_C3" DIAG_ARGS="--sps 32" PMC_LABEL=s32 PMC_DIAG=gpurun_out/${T}q_C3_diag.json \
    PMC_BENCH_ARGS="--steps 16 --warmup 0 --no-single-frame --samples-per-stream 32" bash $S || exit 1
  TAG=${T}r STEPS="diag_C5 pmc_C5" DIAG_ARGS="--sps 32" PMC_LABEL=s32 PMC_DIAG=gpurun_out/${T}r_C5_diag.json \
    PMC_BENCH_ARGS="--steps 3 --warmup 0 --no-single-frame --samples-per-stream 32" bash $S || exit 1
fi
if [ "$P" = all ] || [ "$P" = sweep ]; then
  TAG=${T}s STEPS="ab_C3" STEPS_AB=16 REPS=2 BENCH_ARGS="--no-single-frame --contract-steps 0" \
    RUNS="main:main: pix:main:--frame-order=pixel uol:main:unit_order=learned tt20:main:trav_threshold=20 tt28:main:trav_threshold=28 lb6:main:leaf_break=6 lb12:main:leaf_break=12 pb8:pb8: pb16:pb16:" \
    bash $S || exit 1
fi
if [ "$P" = all ] || [ "$P" = shards ]; then
  mkdir -p gpurun_out
  echo "shards $(date +%T)" >> gpurun_out/${T}x_progress.txt
  echo "gpurun_out/${T}x_contract_shards.json: python3 tools/shard_steady.py --per-launch 20 --cases frame_256spp:L=20,frame_256spp:sps=256:L=20,shard_balanced:L=20,shard_balanced:sps=256:L=20" > gpurun_out/${T}x_manifest.txt
  timeout -k 10 600 python3 tools/shard_steady.py --per-launch 20 \
    --cases frame_256spp:L=20,frame_256spp:sps=256:L=20,shard_balanced:L=20,shard_balanced:sps=256:L=20 \
    > gpurun_out/${T}x_contract_shards.json 2> gpurun_out/${T}x_contract_shards.err || exit 1
  TAG=${T}y STEPS="shards_C3" SHARD_NS=1,2,4,8 SHARD_REPS=1 \
    SHARD_ARGS="--maps balanced --inflight 3 --per-launch 20 --frames 20" bash $S || exit 1
fi
if [ "$P" = s2 ]; then
  # the PIXEL frame order confirmed on the whole frame and on an 8-way shard (3 reps), then the records and the bench line
  # under it (bench.py's default since v58); the diag records of session q6 (lone frames: no frame order) are reused
  TAG=${T}u STEPS="ab_C3" STEPS_AB=16 REPS=3 BENCH_ARGS="--no-single-frame --contract-steps 0" \
    RUNS="inter:main:--frame-order=interleaved pix:main:" bash $S || exit 1
  TAG=${T}v STEPS="ab_C3" STEPS_AB=40 REPS=3 BENCH_ARGS="--no-single-frame --contract-steps 0 --frames-per-launch 20" \
    RUNS="sinter:main:--shard-of=8,--shard=3,--frame-order=interleaved spix:main:--shard-of=8,--shard=3" bash $S || exit 1
  TAG=${T}w STEPS="bench_C3 tracedrv_C3" BENCH_ARGS="--steps 20 --warmup 5" bash $S || exit 1
  TAG=${T}w STEPS="pmc_C3" PMC_DIAG=profiles/r6/c3_v58_diag.json bash $S || exit 1
  TAG=${T}w STEPS="pmc_C3" PMC_LABEL=s32 PMC_DIAG=profiles/r6/c3_v58_s32_diag.json \
    PMC_BENCH_ARGS="--steps 16 --warmup 0 --no-single-frame --samples-per-stream 32" bash $S || exit 1
  TAG=${T}w STEPS="pmc_C5" PMC_LABEL=s32 PMC_DIAG=profiles/r6/c5_v58_s32_diag.json \
    PMC_BENCH_ARGS="--steps 3 --warmup 0 --no-single-frame --samples-per-stream 32" bash $S || exit 1
fi
if [ "$P" = s3 ]; then
  # the final tree's GPU suite, and the projected N-GPU scaling of bench.py's N > 1 loop in its PIXEL frame order
  TAG=${T}t STEPS="tests" bash $S || exit 1
  TAG=${T}y STEPS="shards_C3" SHARD_NS=1,2,4,8 SHARD_REPS=1 \
    SHARD_ARGS="--maps balanced --inflight 3 --per-launch 20 --frames 20 --frame-order pixel" bash $S || exit 1
fi
echo "r6_session done $(date +%T)" >> gpurun_out/${T}_done.txt
