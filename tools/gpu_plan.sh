#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 env COCOA_PLAN=1 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_plan.log 2>&1
rc=$?; echo "plan tests rc=$rc"; grep -E "passed|failed|error|FAIL" gpurun_out/gpu_tests_plan.log | tail -8; [ $rc -ne 0 ] && exit $rc
for P in 0 1; do
  timeout -k 10 300 env COCOA_PLAN=$P python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap > gpurun_out/b_c2_p$P.json 2> gpurun_out/b_c2_p$P.err || exit $?
  python3 -c "import json; j=json.loads(open('gpurun_out/b_c2_p$P.json').read().strip().splitlines()[-1]); print('c2 plan=$P', j['ms_per_step'], j['kernel_ms'])"
  timeout -k 10 300 env COCOA_PLAN=$P python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-gap > gpurun_out/b_c3_p$P.json 2> gpurun_out/b_c3_p$P.err || exit $?
  python3 -c "import json; j=json.loads(open('gpurun_out/b_c3_p$P.json').read().strip().splitlines()[-1]); print('c3 plan=$P', j['ms_per_step'], j['kernel_ms'])"
done
