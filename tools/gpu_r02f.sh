#!/bin/bash
# Gram solver diagnostics: memory-wave costs with scatter atomics / gathers switched off (timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for dg in 0 1 2 3; do
  for m in cocoa+ mbcd; do
    COCOA_GRAM_DIAG=$dg timeout -k 10 120 python -u tools/prof_gram.py $m > gpurun_out/prof_diag${dg}_$m.json 2> gpurun_out/prof_diag${dg}_$m.err || exit 1
    echo "diag=$dg $m"; python -c "import json;d=json.load(open('gpurun_out/prof_diag${dg}_$m.json'));print(round(d['kernel_ms']['solver'],3), {k:round(v) for k,v in d['memory_phases_cyc_per_batch'].items()}, {k:round(v['wait_frac'],3) for k,v in d['waves'].items()})"
  done
done
