#!/bin/bash
# Same-box A/B: solver loader stream loads nontemporal (default build) vs plain (build/ntl0), C2 and MbCD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ntab_tests.log 2>&1 || { tail -20 gpurun_out/ntab_tests.log; exit 1; }
tail -1 gpurun_out/ntab_tests.log
for args in "--steps 20 --warmup 3" "--method mbcd --steps 5 --warmup 2"; do
  tag=$(echo $args | cut -d' ' -f1-2 | tr -d ' -')
  for i in 1 2; do
    for lib in cocoa_amd build/ntl0; do
      n=$(basename $lib)
      timeout -k 10 300 env COCOA_LIB=$lib/libcocoa_hip.so python3 -u bench.py $args --no-cpu-baseline --no-gap > gpurun_out/ntab_${tag}_${n}_$i.json 2> gpurun_out/ntab.err || exit $?
      python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=j['kernel_ms']; print(sys.argv[1], '%.4f' % j['ms_per_step'], 'solver %.4f' % k['solver'])" gpurun_out/ntab_${tag}_${n}_$i.json
    done
  done
done
