#!/bin/bash
# Repeat of the C2 loader-policy A/B, three alternations, with the per-kernel breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for lib in cocoa_amd build/ntl1; do
    n=$(basename $lib)
    timeout -k 10 300 env COCOA_LIB=$lib/libcocoa_hip.so python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-gap > gpurun_out/ntab3_${n}_$i.json 2> gpurun_out/ntab.err || exit $?
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=j['kernel_ms']; print(sys.argv[1], '%.4f' % j['ms_per_step'], 'solver %.4f plan %.4f eval %.4f' % (k['solver'], k['plan'], k['eval']))" gpurun_out/ntab3_${n}_$i.json
  done
done
