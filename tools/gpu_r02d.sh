#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_gram.log 2>&1
rc=$?; echo "gram tests rc=$rc"; tail -2 gpurun_out/gpu_gram.log; [ $rc -ne 0 ] && exit $rc
for m in cocoa+ mbcd; do timeout -k 10 200 python3 tools/prof_gram.py $m > gpurun_out/prof_gram_$m.json 2> gpurun_out/prof_gram_$m.err || exit $?; cat gpurun_out/prof_gram_$m.json; done
