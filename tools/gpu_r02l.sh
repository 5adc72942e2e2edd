#!/bin/bash
# r02 session 2: Gram-kernel phase profile (diag build), C5 method lines on the current tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 300 python3 tools/prof_gram.py cocoa+ > gpurun_out/prof_gram.json 2> gpurun_out/prof_gram.err || exit $?
cat gpurun_out/prof_gram.json
for m in cocoa mbcd mbsgd localsgd; do
  timeout -k 10 300 python3 bench.py --method $m --steps 10 --warmup 2 > gpurun_out/bench_c5_$m.json 2> gpurun_out/bench_c5_$m.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_c5_$m.json').readlines()[-1]);print('$m', round(d['ms_per_step'],3), d['value'], d['plan']['solver'], d['cpu_baseline']['value'])"
done
