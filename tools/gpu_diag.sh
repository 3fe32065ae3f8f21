#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-diag}
timeout -k 10 300 python tools/diag.py --config C3 --spp 32 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}.err &&
timeout -k 10 300 python tools/diag.py --config C2 --spp 16 > gpurun_out/${TAG}_c2.json 2>> gpurun_out/${TAG}.err &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d gpurun_out/pmc1_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --spp 16 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc1_$TAG.err &&
timeout -k 10 600 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD -d gpurun_out/pmc2_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --spp 16 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc2_$TAG.err &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc3_$TAG -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --spp 16 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc3_$TAG.err
