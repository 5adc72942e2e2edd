#!/bin/bash
# memory-wave atomics/products phase split (diag build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r09e}
for dg in 0 4; do
COCOA_GRAM_DIAG=$dg COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py cocoa+ --eval > $O/profsolver_${T}_d$dg.json 2> $O/profsolver_${T}_d$dg.err || exit $?
python3 -c "import json;d=json.load(open('$O/profsolver_${T}_d$dg.json'));print('diag $dg', round(d['kernel_ms']['solver'],4), {k: round(v) for k, v in d['memory_phases_cyc_per_batch']['memory0'].items()}, {k: round(v) for k, v in d['memory_split_cyc_per_batch']['memory0'].items()})"
done
