#!/bin/bash
# Eval-pass study on the C2 shape with tools/ubench/evalspmv (no bench data
# generation in the loop): the shipped kernel under each COCOA_EVAL_VARIANT
# of the library, the eval_wave_kernel variants, and PMC passes of the
# shipped kernel (variant 0) against the single-address no-gather diagnostic
# (variant 4).  Outputs under gpurun_out/ (TAG labels them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-now}
B=tools/ubench/evalspmv
for v in ${EVAL_VARIANTS:-0 3 4 5 6 7}; do
  COCOA_EVAL_VARIANT=$v timeout -k 10 120 $B 20 shipped >> $O/evalvar_$TAG.txt 2>&1 || exit $?
done
timeout -k 10 180 $B 20 all >> $O/evalvar_$TAG.txt 2>&1 || exit $?
cat $O/evalvar_$TAG.txt
i=0
for grp in "TA_BUSY_avr TA_BUSY_max" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"; do
  i=$((i + 1))
  for v in ${PMC_VARIANTS:-0 4}; do
    COCOA_EVAL_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/epmc_${TAG}_v${v}_g$i -o run --output-format csv \
      -- $B 3 shipped > $O/epmc_${TAG}_v${v}_g$i.log 2>&1 || exit $?
  done
done
echo pmc done
