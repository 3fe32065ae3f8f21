#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel-trace summary.  Each GPU step has its
# own time limit and the steps are chained with && (nothing runs on the GPU after a failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1}
echo tests > gpurun_out/progress_$TAG.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 &&
echo bench >> gpurun_out/progress_$TAG.txt &&
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
echo prof >> gpurun_out/progress_$TAG.txt &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/prof_$TAG.err
