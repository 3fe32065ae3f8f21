# Round-3 closing checks: frames in flight 3 vs 4 (C3), the default bench line (with the CPU baseline), smoke, and the
# bench-refusal / multi-entry tests.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do for f in 3 4; do
  timeout -k 10 300 python3 bench.py --config C3 --steps 10 --warmup 4 --no-cpu-baseline --inflight $f > gpurun_out/if3_C3_f${f}_$rep.json 2> gpurun_out/if3_C3_f${f}_$rep.err || exit 1
done; done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_output_stage.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fin_tests.log 2>&1
