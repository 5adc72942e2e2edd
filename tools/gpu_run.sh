#!/bin/bash
# GPU-box steps, run in order; the first failing step ends the call.
#   tools/gpu_run.sh STEP [STEP ...]      (TAG=name labels the outputs)
#   tests            pytest -m gpu (TESTS="-k expr" or a file list narrows it)
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (BENCH_ARGS adds flags)
#   prof             rocprofv3 --kernel-trace --stats of a short bench
#   pmc              FETCH_SIZE / WRITE_SIZE passes (+ calibration) of the same bench
#   lines            the C5 / C3 / C4 config lines
#   lineprof         rocprofv3 --kernel-trace --stats of short C4 / C3 / C5 runs (LINEPROF="c4 c3 ...")
#   gramprof         Gram-solver wave profile (diag build, tools/prof_gram.py)
#   ab               the short bench on each library in VARIANTS (names of build/v_NAME; "base" = in-tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-now}
O=gpurun_out
SHORT="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap ${BENCH_ARGS}"
# the prof step profiles the bench's own window (20 warmup + 50 timed rounds), so the
# kernels' averages over launches 21.. are the timed window bench.py's HIP events see
PROFRUN="python3 bench.py --steps 50 --warmup 20 --no-cpu-baseline --no-gap ${BENCH_ARGS}"

line() {  # name, args...
  local n=$1; shift
  timeout -k 10 600 python3 bench.py "$@" > $O/line_${n}_$TAG.json 2> $O/line_${n}_$TAG.err || return $?
  python3 -c "import json;d=json.loads(open('$O/line_${n}_$TAG.json').readlines()[-1]);print('$n', round(d['ms_per_step'],3), '%.4g'%d['value'], d['plan']['solver'], d.get('time_to_gap_s'), d.get('rounds_to_gap'), d['kernel_ms'], 'frac', round(d['roofline']['frac'],3), round(d['roofline_eval']['frac'],3))"
}

for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 1500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        > $O/gpu_tests_$TAG.log 2>&1; rc=$?
      grep -E "passed|failed|error" $O/gpu_tests_$TAG.log | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || exit $?
      tail -1 $O/smoke_$TAG.log ;;
    bench)
      timeout -k 10 600 python3 bench.py ${BENCH_ARGS} > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit $?
      tail -1 $O/bench_$TAG.json ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_$TAG -o run --output-format csv -- $PROFRUN \
        > $O/rocprof_$TAG.log 2>&1 || exit $?
      python3 tools/rocprof_stats.py $O/rocprof_$TAG 20 | tee $O/rocprof_window_$TAG.txt ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc_${c}_$TAG -o run --output-format csv -- $SHORT \
          > $O/pmc_${c}_$TAG.log 2>&1 || exit $?
        timeout -s KILL 60 rocprofv3 --pmc $c -d $O/calib_${c}_$TAG -o run --output-format csv -- tools/ubench/calib \
          > $O/calib_${c}_$TAG.log 2>&1 || exit $?
      done ;;
    lines)
      line c5_cocoa --method cocoa --steps 10 --warmup 2 --cpu-seconds 8 || exit $?
      line c5_mbcd --method mbcd --steps 10 --warmup 2 --cpu-seconds 8 || exit $?
      line c5_mbsgd --method mbsgd --steps 10 --warmup 2 --cpu-seconds 8 || exit $?
      line c5_localsgd --method localsgd --steps 10 --warmup 2 --cpu-seconds 8 || exit $?
      line c3 --config c3 --steps 10 --warmup 2 --cpu-seconds 8 || exit $?
      line c4 --config c4 --steps 10 --warmup 2 --gap-max-rounds 1500 --cpu-seconds 20 || exit $? ;;
    linec4)  # the C4 line alone (gap run to 1e-4, bounded CPU baseline)
      line c4 --config c4 --steps 10 --warmup 2 --gap-max-rounds 1500 --cpu-seconds 20 || exit $? ;;
    c4pmc)  # HBM bytes and L2 hits of the C4 kernels (one counter group per pass)
      C4SHORT="python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-gap"
      for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_BUSY_max"; do
        n=$(echo $grp | cut -d' ' -f1)
        timeout -s KILL 300 rocprofv3 --pmc $grp -d $O/c4pmc_${n}_$TAG -o run --output-format csv -- $C4SHORT \
          > $O/c4pmc_${n}_$TAG.log 2>&1 || exit $?
      done
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 60 rocprofv3 --pmc $c -d $O/calib_${c}_$TAG -o run --output-format csv -- tools/ubench/calib \
          > $O/calib_${c}_$TAG.log 2>&1 || exit $?
      done ;;
    lineprof)  # rocprofv3 kernel stats of the C3 / C4 / C5 lines (short runs)
      for cfg in ${LINEPROF:-c4 c3 c5_cocoa}; do
        case $cfg in
          c5_*) args="--method ${cfg#c5_}" ;;
          *) args="--config $cfg" ;;
        esac
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_${cfg}_$TAG -o run --output-format csv -- \
          python3 bench.py $args --steps 5 --warmup 1 --no-cpu-baseline --no-gap > $O/rocprof_${cfg}_$TAG.log 2>&1 || exit $?
        python3 tools/rocprof_stats.py $O/rocprof_${cfg}_$TAG
      done ;;
    evalab)  # eval kernel variants (COCOA_EVAL_VARIANT) on the C2 bench
      for v in ${EVAL_VARIANTS:-0 1 2}; do
        COCOA_EVAL_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gap ${BENCH_ARGS} \
          > $O/evalab_${v}_$TAG.json 2> $O/evalab_${v}_$TAG.err || exit $?
        python3 -c "import json;d=json.loads(open('$O/evalab_${v}_$TAG.json').readlines()[-1]);print('eval variant $v', round(d['roofline_eval']['avg_launch_ms'],4), 'ms', round(d['roofline_eval']['frac'],3), 'step', round(d['ms_per_step'],3), 'gap[-1]', repr(d['gap_trajectory_timed'][-1]))"
      done ;;
    evalpmc)  # PMC counters of the eval kernel (one pass per counter group)
      for grp in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"; do
        n=$(echo $grp | cut -d' ' -f1)
        COCOA_EVAL_VARIANT=${EV:-0} timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/evalpmc_${n}_$TAG -o run --output-format csv -- $SHORT \
          > $O/evalpmc_${n}_$TAG.log 2>&1 || exit $?
      done ;;
    solverpmc)  # PMC groups of the solver / gram kernels (one pass per group; PMC_LIB selects a variant)
      for grp in "TA_BUSY_avr TA_BUSY_max" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAVES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
        n=$(echo $grp | cut -d' ' -f1)
        COCOA_LIB=${PMC_LIB:-cocoa_amd/libcocoa_hip.so} timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/spmc_${n}_$TAG -o run --output-format csv -- $SHORT \
          > $O/spmc_${n}_$TAG.log 2>&1 || exit $?
      done
      python3 tools/pmc_kernels.py $O $TAG ;;
    gramprof)
      COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py cocoa+ \
        > $O/prof_gram_$TAG.json 2> $O/prof_gram_$TAG.err || exit $? ;;
    ab)
      for v in ${VARIANTS:-base}; do
        # NAME or NAME+ENVVAR=VALUE (an env setting for that run, e.g. diag+COCOA_GRAM_HOTLDS=1)
        name=${v%%+*}; envset=""; [ "$name" = "$v" ] || envset=${v#*+}
        lib=cocoa_amd/libcocoa_hip.so; [ "$name" = base ] || lib=build/v_$name/libcocoa_hip.so
        [ "$name" = diag ] && lib=build/diag/libcocoa_hip.so
        v=${v//=/_}
        env $envset COCOA_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-gap ${BENCH_ARGS} \
          > $O/ab_${v}_$TAG.json 2> $O/ab_${v}_$TAG.err || exit $?
        python3 -c "import json;d=json.loads(open('$O/ab_${v}_$TAG.json').readlines()[-1]);k=d['kernel_ms'];print('$v', 'step', round(d['ms_per_step'],4), 'solver', round(k['solver'],4), 'gram', round(k.get('gram',0),4), 'eval', round(d['roofline_eval']['avg_launch_ms'],4), 'gap[-1]', repr(d['gap_trajectory_timed'][-1]))"
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
