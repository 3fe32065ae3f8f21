set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m "gpu and not slow" -x -q -p no:cacheprovider > gpurun_out/t1.log 2>&1
