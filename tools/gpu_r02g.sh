#!/bin/bash
# r02: bench gram vs chain (C2 cocoa+, mbcd), no profiling counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in cocoa+ mbcd; do
for sv in gram chain; do
  timeout -k 10 300 python3 bench.py --method $m --solver $sv --steps 10 --warmup 2 --no-cpu-baseline --no-gap > gpurun_out/bench_${m}_$sv.json 2> gpurun_out/bench_${m}_$sv.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${m}_$sv.json').readlines()[-1]);print('$m $sv', round(d['ms_per_step'],3), {k:round(v,4) for k,v in d['kernel_ms'].items()})"
done
done
