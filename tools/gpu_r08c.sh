#!/bin/bash
# the loader's phases (diag build), mirror on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
for m in ${MIRRORS:-1}; do
  COCOA_GRAM_MIRROR=$m COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py cocoa+ --eval \
    > $O/profsolver_${TAG:-r08c}_m$m.json 2> $O/profsolver_${TAG:-r08c}_m$m.err || exit $?
  python3 -c "import json;d=json.load(open('$O/profsolver_${TAG:-r08c}_m$m.json'));print('mirror $m', d['kernel_ms']['solver'], d['loader_cyc_per_batch'], d['loader_phase_cyc_per_batch'], d['chain_wait_frac'])"
done
