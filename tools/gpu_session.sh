#!/bin/bash
# The one GPU session script (run on the box through gpurun; every profiles/rN record names the step that made it).
#
#   TAG=r4a STEPS="tests bench_C3 trace_C3 pmc_C3" tools/gpu_session.sh
#
# STEPS, run in order, each under its own time limit; the first failure (a crash, abort or time limit) ends the session:
#   tests              pytest -m gpu (TESTS_K: a -k expression, may hold spaces; PYTEST_ARGS: more words)
#   bench_<CFG>        bench.py --config CFG (BENCH_ARGS appended; the CPU baseline only for C3 unless NO_CPU=1)
#   shards_<CFG>[.<L>] tools/shard_scaling.py: every shard of SHARD_NS (default 1,8) on one GPU, SHARD_REPS reps,
#                      SHARD_ARGS (or SHARD_ARGS_<L> for a labelled run), library SHARD_LIB_<L> (default main)
#   shardtrace_<CFG>   rocprofv3 --kernel-trace around one tools/shard_scaling.py run (SHARD_NS, SHARD_ARGS)
#   diag_<CFG>         tools/diag.py with the diagnostic build (phase shares, node visits, lane utilisation)
#   trace_<CFG>        rocprofv3 --kernel-trace --stats around bench.py (the kernel's average launch duration: every launch
#                      of the run renders the bench's frames per launch, no lone-frame or contract launches)
#   tracedrv_<CFG>     rocprofv3 --kernel-trace --stats around the driver's command (--steps 20 --warmup 5)
#   pmc_<CFG>          six rocprofv3 --pmc passes over one bench launch -> tools/roofline.py record (+ the diag record
#                      PMC_DIAG, default gpurun_out/${TAG}_<CFG>_diag.json, if present; PMC_LABEL names a labelled run)
#   units_<CFG>        tools/unit_times.py: the longest measured unit per tile of a whole frame (UNITS_ARGS)
#   lat_<CFG>          two --pmc passes: L1 TLB hits/misses, L2 read latency seen by the vector L1, DRAM share of L2 fills
#   pmcx_<CFG>         one --pmc pass of the counters in PMCX (output name PMCX_NAME)
#   ab[_<CFG>]         interleaved A/B timing: RUNS (or RUNS_<CFG>) = "name:lib:opts ..." (lib = suffix of lib/librp_<lib>.so or main,
#                      opts = bench.py --opt field=value,... or --flag=value or --flag), REPS rounds, config CFG, STEPS_AB frames each
#   abpmc[_<CFG>]      per run of RUNS one FETCH_SIZE and one WRITE_SIZE pass over one CFG frame (traffic A/B)
# Outputs: gpurun_out/${TAG}_*; gpurun_out/${TAG}_manifest.txt lists every output file with the command that made it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-s}
CFG=${CFG:-C3}
P=gpurun_out/${TAG}_progress.txt
M=gpurun_out/${TAG}_manifest.txt
echo "start $(date +%T)" > $P
: > $M
step() { echo "$1 $(date +%T)" >> $P; }
made() { echo "$1: $2" >> $M; }  # output file: command
frames() { case $1 in C5) echo "3 3" ;; C4) echo "4 4" ;; *) echo "32 16" ;; esac; }
# one launch of the bench's frames per launch (C3: 16 frames; C5: 3), the default PMC pass workload
pmcframes() { case $1 in C5) echo "--steps 3 --warmup 0 --no-single-frame" ;; C4) echo "--steps 8 --warmup 0 --no-single-frame" ;; *) echo "--steps 16 --warmup 0 --no-single-frame" ;; esac; }
pmc() {  # lib cfg name counters...   (PMC_BENCH_ARGS: the bench frames, default one frame; PMC_LABEL: output suffix)
  local lib=$1 cfg=$2 name=$3; shift 3
  local out=gpurun_out/${TAG}_${cfg}${PMC_LABEL:+_$PMC_LABEL}_pmc_$name cmd
  local ba=${PMC_BENCH_ARGS:-$(pmcframes $cfg)}
  cmd="rocprofv3 --pmc $* -- python3 bench.py --config $cfg $ba --no-cpu-baseline --contract-steps 0"
  step "pmc $cfg $name"
  made "$out" "RP_LIB=$lib $cmd"
  RP_LIB=$lib timeout -s KILL 300 rocprofv3 --pmc "$@" -d $out -o run --output-format csv -- \
    python3 bench.py --config $cfg $ba --no-cpu-baseline --contract-steps 0 > $out.json 2> $out.err
}
LIB=raytracing-potato_amd/lib/librp.so
libpath() { [ "$1" = main ] && echo $LIB || echo raytracing-potato_amd/lib/librp_$1.so; }
for s in ${STEPS:-tests}; do
  case $s in
    tests)
      step tests
      made gpurun_out/${TAG}_tests.log "pytest tests -m gpu ${PYTEST_ARGS:-}"
      timeout -k 10 ${TESTS_LIMIT:-1200} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
        -p no:cacheprovider ${TESTS_K:+-k "$TESTS_K"} ${PYTEST_ARGS:-} > gpurun_out/${TAG}_tests.log 2>&1 || { step "tests failed"; exit 1; } ;;
    bench_*)
      cfg=${s#bench_}; read st wu <<< "$(frames $cfg)"
      cpu=""; { [ $cfg != C3 ] || [ -n "${NO_CPU:-}" ]; } && cpu=--no-cpu-baseline
      step "bench $cfg"
      made gpurun_out/${TAG}_${cfg}_bench.json "python3 bench.py --config $cfg --steps $st --warmup $wu $cpu ${BENCH_ARGS:-}"
      timeout -k 10 600 python3 bench.py --config $cfg --steps $st --warmup $wu $cpu ${BENCH_ARGS:-} \
        > gpurun_out/${TAG}_${cfg}_bench.json 2> gpurun_out/${TAG}_${cfg}_bench.err || exit 1 ;;
    shards_*)  # shards_<CFG>[.<label>]: SHARD_ARGS, or SHARD_ARGS_<label> for a labelled run
      cfg=${s#shards_}; label=""; [[ $cfg == *.* ]] && label=${cfg#*.} && cfg=${cfg%%.*}
      sa=SHARD_ARGS${label:+_$label}; sargs=${!sa:-${SHARD_ARGS:-}}
      sl=SHARD_LIB${label:+_$label}; slib=$(libpath ${!sl:-main})  # SHARD_LIB_<label>: a lib/librp_<name>.so variant
      out=gpurun_out/${TAG}_${cfg}${label:+_$label}_shards
      step "shards $cfg $label"
      made $out.json "RP_LIB=$slib python3 tools/shard_scaling.py --config $cfg --ns ${SHARD_NS:-1,8} --reps ${SHARD_REPS:-3} $sargs"
      RP_LIB=$slib timeout -k 10 900 python3 tools/shard_scaling.py --config $cfg --ns ${SHARD_NS:-1,8} --reps ${SHARD_REPS:-3} $sargs \
        > $out.json 2> $out.err || exit 1 ;;
    shardtrace_*)  # rocprofv3 kernel trace of one shards run (SHARD_ARGS, SHARD_NS): overlap of in-flight frames
      cfg=${s#shardtrace_}
      out=gpurun_out/${TAG}_${cfg}_shardtrace
      step "shardtrace $cfg"
      made $out "rocprofv3 --kernel-trace -- python3 tools/shard_scaling.py --config $cfg --ns ${SHARD_NS:-8} --reps 1 ${SHARD_ARGS:-}"
      timeout -k 10 600 rocprofv3 --kernel-trace -d $out -o run --output-format csv -- \
        python3 tools/shard_scaling.py --config $cfg --ns ${SHARD_NS:-8} --reps 1 ${SHARD_ARGS:-} > $out.json 2> $out.err || exit 1 ;;
    diag_*)
      cfg=${s#diag_}
      step "diag $cfg"
      made gpurun_out/${TAG}_${cfg}_diag.json "RP_LIB=raytracing-potato_amd/lib/librp_diag.so python3 tools/diag.py --config $cfg --spp 256 ${DIAG_ARGS:-}"
      RP_LIB=raytracing-potato_amd/lib/librp_diag.so timeout -k 10 300 python3 tools/diag.py --config $cfg --spp 256 ${DIAG_ARGS:-} \
        > gpurun_out/${TAG}_${cfg}_diag.json 2> gpurun_out/${TAG}_${cfg}_diag.err || exit 1 ;;
    trace_*)
      cfg=${s#trace_}; read st wu <<< "$(frames $cfg)"
      step "trace $cfg"
      made gpurun_out/${TAG}_${cfg}_trace "rocprofv3 --kernel-trace --stats -- python3 bench.py --config $cfg --steps $st --warmup $wu --no-cpu-baseline --contract-steps 0 --no-single-frame ${BENCH_ARGS:-}"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${cfg}_trace -o run --output-format csv -- \
        python3 bench.py --config $cfg --steps $st --warmup $wu --no-cpu-baseline --contract-steps 0 --no-single-frame ${BENCH_ARGS:-} \
        > gpurun_out/${TAG}_${cfg}_bench_under_rocprof.json 2> gpurun_out/${TAG}_${cfg}_trace.err || exit 1 ;;
    tracedrv_*)  # rocprofv3 --kernel-trace --stats around the driver's own command (--steps 20 --warmup 5): compare its
      # average with the line's roofline.kernel_ms_all_launches (every launch of the process, side runs included)
      cfg=${s#tracedrv_}
      step "tracedrv $cfg"
      made gpurun_out/${TAG}_${cfg}_tracedrv "rocprofv3 --kernel-trace --stats -- python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${cfg}_tracedrv -o run --output-format csv -- \
        python3 bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/${TAG}_${cfg}_bench_drv_under_rocprof.json 2> gpurun_out/${TAG}_${cfg}_tracedrv.err || exit 1 ;;
    pmc_*)
      cfg=${s#pmc_}
      pmc $LIB $cfg sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
        SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT &&
      pmc $LIB $cfg mix64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
        SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_THREAD_CYCLES_VALU &&
      pmc $LIB $cfg mix32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 \
        SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS &&
      pmc $LIB $cfg fetch FETCH_SIZE &&
      pmc $LIB $cfg write WRITE_SIZE &&
      pmc $LIB $cfg l2 TCC_HIT_sum TCC_MISS_sum || exit 1
      lc=$(echo $cfg | tr A-Z a-z)${PMC_LABEL:+_$PMC_LABEL}
      pre=gpurun_out/${TAG}_${cfg}${PMC_LABEL:+_$PMC_LABEL}_pmc
      made gpurun_out/${TAG}_${lc}_roofline.json "python3 tools/roofline.py --config $cfg over the six pmc passes above"
      python3 tools/roofline.py --config $cfg --bench ${pre}_sq.json ${PMC_BENCH_ARGS:+--all-dispatches} \
        $(d=${PMC_DIAG:-gpurun_out/${TAG}_${cfg}_diag.json}; [ -f $d ] && echo --diag $d) \
        --out gpurun_out/${TAG}_${lc}_roofline.json \
        ${pre}_sq ${pre}_mix64 ${pre}_mix32 ${pre}_fetch ${pre}_write ${pre}_l2 \
        > gpurun_out/${TAG}_${cfg}${PMC_LABEL:+_$PMC_LABEL}_roofline.log 2>&1 || exit 1 ;;
    units_*)  # the longest measured unit per tile (product build): tools/unit_times.py
      cfg=${s#units_}
      step "units $cfg"
      made gpurun_out/${TAG}_${cfg}_units.json "python3 tools/unit_times.py --config $cfg ${UNITS_ARGS:-}"
      timeout -k 10 300 python3 tools/unit_times.py --config $cfg ${UNITS_ARGS:-} \
        > gpurun_out/${TAG}_${cfg}_units.json 2> gpurun_out/${TAG}_${cfg}_units.err || exit 1 ;;
    lat_*)  # memory-latency picture: L1 TLB hits/misses, L2 read latency seen by the vector L1, DRAM share of fills
      cfg=${s#lat_}
      pmc $LIB $cfg lat_tcp TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum \
        TCP_TCC_READ_REQ_sum &&
      pmc $LIB $cfg lat_tcc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum || exit 1 ;;
    pmcx_*)  # one extra --pmc pass: PMCX="<counters>" (within one pass's per-block limits), named PMCX_NAME
      cfg=${s#pmcx_}
      pmc $LIB $cfg ${PMCX_NAME:-x} $PMCX || exit 1 ;;
    ab|ab_*)
      [ "$s" != ab ] && CFG=${s#ab_}
      read st wu <<< "$(frames $CFG)"
      runs_var=RUNS_$CFG; runs=${!runs_var:-$RUNS}  # RUNS_<CFG> overrides RUNS for that config
      for rep in $(seq 1 ${REPS:-2}); do
        for run in $runs; do
          name=${run%%:*}; rest=${run#*:}; lib=${rest%%:*}; opts=${rest#*:}
          args=""
          for o in $(echo $opts | tr ',' ' '); do  # field=value: --opt; --flag=value: a bench.py flag
            if [[ $o == --*=* ]]; then args="$args ${o%%=*} ${o#*=}"; elif [[ $o == --* ]]; then args="$args $o"; else args="$args --opt $o"; fi
          done
          out=gpurun_out/${TAG}_${CFG}_${name}_$rep.json
          step "ab $rep $name"
          made $out "RP_LIB=$(libpath $lib) python3 bench.py --config $CFG --steps ${STEPS_AB:-$st} --warmup $wu --no-cpu-baseline $args ${BENCH_ARGS:-}"
          RP_LIB=$(libpath $lib) timeout -k 10 300 python3 bench.py --config $CFG --steps ${STEPS_AB:-$st} --warmup $wu \
            --no-cpu-baseline $args ${BENCH_ARGS:-} > $out 2> ${out%.json}.err || exit 1
        done
      done ;;
    abpmc|abpmc_*)
      [ "$s" != abpmc ] && CFG=${s#abpmc_}
      runs_var=RUNS_$CFG; runs=${!runs_var:-$RUNS}
      for run in $runs; do
        name=${run%%:*}; rest=${run#*:}; lib=${rest%%:*}
        pmc $(libpath $lib) $CFG ${name}_fetch FETCH_SIZE && pmc $(libpath $lib) $CFG ${name}_write WRITE_SIZE || exit 1
      done ;;
    ldswait_*)  # tools/gather_lds_wait.py: a kernel of RCCL's all-gather footprint behind frames in flight (LDSW_ARGS)
      cfg=${s#ldswait_}
      out=gpurun_out/${TAG}_${cfg}_ldswait${LDSW_LABEL:+_$LDSW_LABEL}
      step "ldswait $cfg $LDSW_LABEL"
      made $out.json "python3 tools/gather_lds_wait.py --config $cfg ${LDSW_ARGS:-}"
      timeout -k 10 600 python3 tools/gather_lds_wait.py --config $cfg ${LDSW_ARGS:-} > $out.json 2> $out.err || exit 1 ;;
    *) echo "unknown step $s" >> $P; exit 2 ;;
  esac
done
step done
