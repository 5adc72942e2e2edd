#!/bin/bash
# memory waves read batch b+3's ring entries before b's atomics: tests, profile, A/B vs build/v_old
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r09f}
timeout -k 10 900 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_mirror.py tests/test_gpu_gram_seq.py \
  tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_driver.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_$T.log | tail -3; [ $rc -eq 0 ] || exit $rc
COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 200 python3 tools/prof_gram.py cocoa+ --eval > $O/profsolver_$T.json 2> $O/profsolver_$T.err || exit $?
python3 -c "import json;d=json.load(open('$O/profsolver_$T.json'));print(round(d['kernel_ms']['solver'],4), {k: round(v) for k, v in d['chain_phase_cyc_per_batch'].items()}, {k: round(v) for k, v in d['memory_phases_cyc_per_batch']['memory0'].items()}, {k: round(v) for k, v in d['memory_split_cyc_per_batch']['memory0'].items()})"
STEPS=100 REPS=2 TAG=ab_$T tools/benchab.sh " --" "COCOA_LIB=build/v_old/libcocoa_hip.so --" || exit $?
STEPS=20 REPS=1 TAG=ab_${T}c5 tools/benchab.sh "-- --config c5" "COCOA_LIB=build/v_old/libcocoa_hip.so -- --config c5" || exit $?
