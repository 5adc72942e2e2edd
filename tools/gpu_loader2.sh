#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
CHAINS=v3 bash tools/gpu_chain.sh || exit $?
timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-gap > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || exit $?
python3 -c "import json; j=json.loads(open('gpurun_out/b_c3.json').read().strip().splitlines()[-1]); print('c3', j['ms_per_step'], j['kernel_ms'])"
