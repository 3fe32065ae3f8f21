# Strong-scaling projection on one GPU for every N of the driver's SCALE run (1, 2, 4, 8): each rank's shard
# rendered with F frames in flight, balanced plan from the learned table (tools/shard_scaling.py).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for f in 3 4; do
  timeout -k 10 400 python3 -u tools/shard_scaling.py --config C3 --ns 1,2,4,8 --maps balanced --inflight $f \
    --frames 9 > gpurun_out/proj_C3_f$f.json 2> gpurun_out/proj_C3_f$f.err || exit 1
done
