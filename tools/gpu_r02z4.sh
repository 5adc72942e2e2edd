#!/bin/bash
# r02 session 3: Gram-solver phase profile (diag build) of the current tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for dg in ${DIAGS:-0}; do
  COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_DIAG=$dg timeout -k 10 200 python3 tools/prof_gram.py cocoa+ > gpurun_out/prof_now$dg.json 2> gpurun_out/prof_now$dg.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/prof_now$dg.json'));print($dg, {k:round(v,3) for k,v in d['kernel_ms'].items()}, round(d['cyc_per_step_chain'],1), {k:round(v['wait_frac'],3) for k,v in d['waves'].items()}, {k:round(v) for k,v in d['memory_phases_cyc_per_batch'].items()}, {k:round(v) for k,v in d['gram_phase_cyc_per_wg'].items()})"
done
