#!/bin/bash
# r02 session 2: GPU ingest tests + ingest timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_ingest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/gpu_ingest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 tools/bench_ingest.py 200000 /tmp/ingest_rcv1.txt > gpurun_out/bench_ingest.json 2> gpurun_out/bench_ingest.err || exit $?
cat gpurun_out/bench_ingest.json
