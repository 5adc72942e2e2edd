#!/bin/bash
# Same-box A/B of chain v3 register chunks on C2 (runtime selection 3 vs forced 4), alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-gap"
for i in 1 2; do
  for rc in 3 4; do
    timeout -k 10 300 env COCOA_REG_CHUNKS_RT=$rc $B > gpurun_out/rcab_${rc}_$i.json 2> gpurun_out/rcab.err || exit $?
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], '%.4f' % j['ms_per_step'], '%.4f' % j['kernel_ms']['solver'])" gpurun_out/rcab_${rc}_$i.json
  done
done
