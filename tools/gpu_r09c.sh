#!/bin/bash
# chain phase breakdown (diag build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r09c}
for m in cocoa+ cocoa; do
COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py $m --eval > $O/profsolver_${T}_$m.json 2> $O/profsolver_${T}_$m.err || exit $?
python3 -c "import json;d=json.load(open('$O/profsolver_${T}_$m.json'));[print(k, d[k]) for k in ['kernel_ms','cyc_per_step_chain','chain_base_wait_frac','chain_wait_frac','chain_phase_cyc_per_batch','memory_phases_cyc_per_batch','loader_cyc_per_batch']]"
done
