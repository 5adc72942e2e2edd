#!/bin/bash
# Eval-pass study on the C2 shape with tools/ubench/evalspmv (no bench data
# generation in the loop): the shipped kernel under each COCOA_EVAL_VARIANT
# of the library, the eval_wave_kernel variants, and PMC passes of the
# shipped kernel (variant 0) against the single-address no-gather diagnostic
# (variant 4).  Outputs under gpurun_out/ (TAG labels them).  The variants live
# in the diagnostic build only (make diag): the harness loads build/diag's
# library through LD_LIBRARY_PATH (its RUNPATH names the in-tree one).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-now}
B=tools/ubench/evalspmv
for v in ${EVAL_VARIANTS:-0 3 4 5 6 7}; do
  LD_LIBRARY_PATH=build/diag COCOA_EVAL_VARIANT=$v timeout -k 10 120 $B 20 shipped >> $O/evalvar_$TAG.txt 2>&1 || exit $?
done
[ -n "$NO_ALL" ] || timeout -k 10 180 $B 20 all >> $O/evalvar_$TAG.txt 2>&1 || exit $?
cat $O/evalvar_$TAG.txt
# counter groups, ';'-separated (one rocprofv3 pass each)
PMCG=${PMC_GROUPS:-"TA_BUSY_avr TA_BUSY_max;TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"}
i=0
IFS=';' read -ra GARR <<< "$PMCG"
for grp in "${GARR[@]}"; do
  i=$((i + 1))
  for v in ${PMC_VARIANTS:-0 4}; do
    LD_LIBRARY_PATH=build/diag COCOA_EVAL_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/epmc_${TAG}_v${v}_g$i -o run --output-format csv \
      -- $B 3 shipped > $O/epmc_${TAG}_v${v}_g$i.log 2>&1 || exit $?
  done
done
echo pmc done
