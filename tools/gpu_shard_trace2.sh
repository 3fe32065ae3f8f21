# Kernel timeline of the 8-way shards with the learned cost table installed (tools/shard_scaling.py: what every rank
# holds after its first gathered frame), 3 frames in flight.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/st2 -o run --output-format csv -- \
  python3 tools/shard_scaling.py --config C3 --ns 8 --maps balanced --inflight 3 --frames 9 \
  > gpurun_out/st2.json 2> gpurun_out/st2.err
