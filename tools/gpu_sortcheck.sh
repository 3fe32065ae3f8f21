set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "plan or tile or balanced or gather or shard or multi" > gpurun_out/sc_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/st3 -o run --output-format csv -- \
  python3 tools/shard_scaling.py --config C3 --ns 8 --maps balanced --inflight 3 --frames 9 > gpurun_out/st3.json 2> gpurun_out/st3.err &&
timeout -k 10 300 python3 tools/shard_scaling.py --config C3 --ns 1,2,4,8 --maps balanced --inflight 3 --frames 9 > gpurun_out/proj3.json 2> gpurun_out/proj3.err &&
timeout -k 10 300 python3 bench.py --config C3 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/sc_bench.json 2> gpurun_out/sc_bench.err
