#!/bin/bash
# C5 (10M-triangle random mesh, 4096x4096) on one GPU: scene generation + device BVH build, then timed
# frames (SPP=0: the config's 256 spp); then the PMC traffic passes (FETCH_SIZE, WRITE_SIZE) over one frame.
# Not part of the default bench.  Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
SPP=${SPP:-0}
TAG=${TAG:-c5}
echo "bench" > gpurun_out/${TAG}_progress.txt
timeout -k 10 600 python -u bench.py --config C5 --spp $SPP --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
echo "pmc fetch" >> gpurun_out/${TAG}_progress.txt &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_pmc_fetch -o run --output-format csv -- \
  python3 bench.py --config C5 --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_pmc_fetch.json 2> gpurun_out/${TAG}_pmc_fetch.err &&
echo "pmc write" >> gpurun_out/${TAG}_progress.txt &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_pmc_write -o run --output-format csv -- \
  python3 bench.py --config C5 --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_pmc_write.json 2> gpurun_out/${TAG}_pmc_write.err &&
echo "done" >> gpurun_out/${TAG}_progress.txt
