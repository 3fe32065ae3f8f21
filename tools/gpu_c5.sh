#!/bin/bash
# C5 (10M-triangle random mesh, 4096x4096) on one GPU at reduced spp: host scene generation + BVH build,
# then one timed frame; and the PMC traffic passes over the same frame.  Not part of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPP=${SPP:-16}
echo "bench" > gpurun_out/c5_progress.txt
timeout -k 10 900 python -u bench.py --config C5 --spp $SPP --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
