#!/bin/bash
# Iteration loop on the GPU box: parity tests, a short bench line, the diagnostic phase breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-iter}
echo "tests" > gpurun_out/${TAG}_progress.txt
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 &&
echo "bench" >> gpurun_out/${TAG}_progress.txt &&
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
echo "diag" >> gpurun_out/${TAG}_progress.txt &&
timeout -k 10 300 python tools/diag.py --config C3 --spp 32 > gpurun_out/${TAG}_diag.json 2> gpurun_out/${TAG}_diag.err
