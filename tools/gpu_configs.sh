#!/bin/bash
# Extra measurement lines: C5 (five methods on the C2 shape), C3 (epsilon-shaped dense), C4 (url-shaped, K=1024).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 -u bench.py "$@" > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err || { echo "$name failed rc=$?"; tail -5 gpurun_out/cfg_$name.err; return 1; }
  tail -1 gpurun_out/cfg_$name.json >> gpurun_out/configs.jsonl
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/cfg_$name.json').read().strip().splitlines()[-1]); print('$name', '%.4g upd/s' % j['value'], '%.3f ms/step' % j['ms_per_step'], 'ttg', j['time_to_gap_s'], j['rounds_to_gap'], 'solver ms %.3f' % j['kernel_ms'].get('solver', 0), 'eval ms %.3f' % j['kernel_ms'].get('eval', 0), 'cpu', (j['cpu_baseline'] or {}).get('value'))"
}
for m in ${METHODS:-cocoa mbcd mbsgd localsgd}; do
  [ "$m" = none ] && continue
  run c5_$m 240 --config c2 --method $m --steps 5 --warmup 1 --gap-max-rounds 150 --cpu-seconds 5 || exit 1
done
run c3 400 --config c3 --steps 3 --warmup 1 --gap-max-rounds 60 --cpu-seconds 5 || exit 1
run c4 400 --config c4 --steps 3 --warmup 1 --gap-max-rounds 60 --no-cpu-baseline || exit 1
