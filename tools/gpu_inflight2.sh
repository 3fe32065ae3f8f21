# One GPU, frames in flight after the LDS-free tile sorts (v47): bench.py --inflight 1 / 2 / 3, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2 3; do for f in 1 3 2; do
  timeout -k 10 300 python3 bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline --inflight $f > gpurun_out/if2_C3_f${f}_$rep.json 2> gpurun_out/if2_C3_f${f}_$rep.err || exit 1
done; done
for f in 1 3; do timeout -k 10 300 python3 bench.py --config C5 --steps 4 --warmup 3 --no-cpu-baseline --inflight $f > gpurun_out/if2_C5_f${f}_1.json 2> gpurun_out/if2_C5_f${f}_1.err || exit 1; done
