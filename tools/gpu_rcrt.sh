#!/bin/bash
# Runtime register-chunk selection: GPU tests under both settings, then the
# C2 headline, C5 MbCD and C4 lines with the default selection.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T > gpurun_out/rcrt_tests.log 2>&1 || { tail -20 gpurun_out/rcrt_tests.log; exit 1; }
tail -1 gpurun_out/rcrt_tests.log
timeout -k 10 300 env COCOA_REG_CHUNKS_RT=short $T > gpurun_out/rcrt_tests4.log 2>&1 || { tail -20 gpurun_out/rcrt_tests4.log; exit 1; }
tail -1 gpurun_out/rcrt_tests4.log
for args in "--steps 20 --warmup 3" "--method mbcd --steps 5 --warmup 2" "--config c4 --steps 5 --warmup 2"; do
  tag=$(echo $args | cut -d' ' -f1-2 | tr -d ' -')
  timeout -k 10 300 python3 -u bench.py $args --no-cpu-baseline --no-gap > gpurun_out/rcrt_$tag.json 2> gpurun_out/rcrt_$tag.err || exit $?
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], '%.3f' % j['ms_per_step'], '%.3f' % j['kernel_ms']['solver'])" gpurun_out/rcrt_$tag.json
done
