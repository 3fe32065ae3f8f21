# Kernel timeline of one 8-way shard rendered frame after frame (bench.py --shard-of 8, no gather), with 1 and 3
# frames in flight: where the per-shard time above 1/8 of the frame goes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for f in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/st_f$f -o run --output-format csv -- \
    python3 bench.py --config C3 --shard-of 8 --shard 0 --steps 12 --warmup 3 --inflight $f --no-cpu-baseline \
    > gpurun_out/st_f$f.json 2> gpurun_out/st_f$f.err || exit 1
done
