#!/bin/bash
# Register-chunk count 4 (shipped) vs 3 on the other measured lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for args in "--method cocoa" "--method mbcd" "--config c4"; do
  tag=$(echo $args | tr -d ' -')
  for rc in 4 3; do
    lib=cocoa_amd/libcocoa_hip.so; [ $rc = 3 ] && lib=build/rc3/libcocoa_hip.so
    timeout -k 10 300 env COCOA_LIB=$lib python3 -u bench.py $args --steps 5 --warmup 2 --no-cpu-baseline --no-gap > gpurun_out/rcx_${tag}_$rc.json 2> gpurun_out/rcx_${tag}_$rc.err || exit $?
    python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], '%.3f' % j['ms_per_step'], '%.3f' % j['kernel_ms']['solver'])" gpurun_out/rcx_${tag}_$rc.json
  done
done
