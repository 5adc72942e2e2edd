#!/bin/bash
# r02 session 2: Gram-solver products by LDS adds: gram tests, C2 configs, bench x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_y.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_y.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/bench_y$i.json 2> gpurun_out/bench_y$i.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_y$i.json').readlines()[-1]);print(round(d['ms_per_step'],4), '%.4g'%d['value'], round(d['time_to_gap_s'],4), {k:round(v,4) for k,v in d['kernel_ms'].items()})"
done
