#!/bin/bash
# r02: Gram-window solver parity + first timing against the chain solver.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_gram.log 2>&1
rc=$?; echo "gram tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_gram.log | tail -5; [ $rc -ne 0 ] && exit $rc
for sv in gram chain; do
  timeout -k 10 300 python3 bench.py --solver $sv --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$sv.json 2> gpurun_out/bench_$sv.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_$sv.json').readlines()[-1]);print('$sv', round(d['ms_per_step'],3), {k:round(v,4) for k,v in d['kernel_ms'].items()}, d['rounds_to_gap'], d['time_to_gap_s'])"
done
