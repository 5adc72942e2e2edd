#!/bin/bash
# DPP wave scan, gram_seq walk off the MFMA waves: tests, Gram phases, A/B vs build/v_old
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r09b}
timeout -k 10 900 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_mirror.py tests/test_gpu_gram_seq.py \
  tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_$T.log | tail -3; [ $rc -eq 0 ] || exit $rc
COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py cocoa+ --eval > $O/profsolver_$T.json 2> $O/profsolver_$T.err || exit $?
python3 -c "import json;d=json.load(open('$O/profsolver_$T.json'));print(d['kernel_ms']);print(d['gram_phase_cyc_per_wg'])"
STEPS=100 REPS=2 TAG=ab_$T tools/benchab.sh " --" "COCOA_LIB=build/v_old/libcocoa_hip.so --" || exit $?
