#!/bin/bash
# Round-2 baseline probe on the GPU box: counter list, cycle-budget PMC pass (SQ wait/active/issue +
# GRBM clock), the diagnostic region breakdown, and a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2probe}
timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/${TAG}_pmcA -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_pmcA.out 2> gpurun_out/${TAG}_pmcA.err &&
timeout -k 10 300 python3 tools/diag.py --config C3 --spp 32 > gpurun_out/${TAG}_diag_c3.json 2> gpurun_out/${TAG}_diag.err
