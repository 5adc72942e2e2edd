#!/bin/bash
# r02 session 2: config lines on the current tree (C5 methods, C3, C4 one GPU, C4 one GPU's 8-way strong share)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lines
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 600 python3 bench.py "$@" > gpurun_out/lines/$n.json 2> gpurun_out/lines/$n.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/lines/$n.json').readlines()[-1]);print('$n', round(d['ms_per_step'],3), '%.4g'%d['value'], d['plan']['solver'], d.get('time_to_gap_s'), d.get('rounds_to_gap'), (d.get('cpu_baseline') or {}).get('value'))"
}
run c5_cocoa --method cocoa --steps 10 --warmup 2
run c5_mbcd --method mbcd --steps 10 --warmup 2
run c5_mbsgd --method mbsgd --steps 10 --warmup 2
run c5_localsgd --method localsgd --steps 10 --warmup 2
run c3 --config c3 --steps 10 --warmup 2 --cpu-seconds 10
run c4 --config c4 --steps 10 --warmup 2 --no-cpu-baseline
