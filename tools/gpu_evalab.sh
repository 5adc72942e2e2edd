#!/bin/bash
# Same-box A/B of the eval stream's cache policy on the full C2 step (variant 3 = nontemporal, 18 = plain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-gap"
for i in 1 2; do
  for v in 3 18; do
    timeout -k 10 300 env COCOA_EVAL4=$v $B > gpurun_out/evab_${v}_$i.json 2> gpurun_out/evab.err || exit $?
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=j['kernel_ms']; print(sys.argv[1], '%.4f' % j['ms_per_step'], 'solver %.4f eval %.4f plan %.4f' % (k['solver'], k['eval'], k['plan']))" gpurun_out/evab_${v}_$i.json
  done
done
