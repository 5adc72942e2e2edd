#!/bin/bash
# round 6: who bounds the solver -- per-wave waits with the loader's vm_drain
# cycles (diag build, the bench's eval-every-round flow), mirror on / off; then
# the mirror / gram_seq tests on the tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for m in ${MIRRORS:-1 0}; do
  COCOA_GRAM_MIRROR=$m COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py cocoa+ --eval \
    > $O/profsolver_r08b_m$m.json 2> $O/profsolver_r08b_m$m.err || exit $?
  python3 -c "import json;d=json.load(open('$O/profsolver_r08b_m$m.json'));print('mirror $m', {k:v for k,v in d.items() if k not in ('gram_phase_cyc_per_wg','plan')})"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_gram_seq.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/gpu_tests_r08b.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_r08b.log | tail -3; exit $rc
