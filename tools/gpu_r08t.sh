#!/bin/bash
# eight column runs (four memory waves per mirrored half): tests, then A/B against four runs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_gram.py tests/test_gpu_gram_seq.py \
  tests/test_gpu_configs.py -k "mirror or gram or c2 or c5" -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_r08t.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_r08t.log | tail -3; [ $rc -eq 0 ] || exit $rc
STEPS=50 REPS=2 TAG=ab8t tools/benchab.sh " --" "COCOA_LIB=build/v_runs4/libcocoa_hip.so --" || exit $?
COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py cocoa+ --eval > $O/profsolver_r08t.json 2> $O/profsolver_r08t.err || exit $?
python3 -c "import json;d=json.load(open('$O/profsolver_r08t.json'));print({k:v for k,v in d.items() if k not in ('gram_phase_cyc_per_wg','plan')})"
