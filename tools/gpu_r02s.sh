#!/bin/bash
# r02 session 2: PMC traffic passes (FETCH_SIZE, WRITE_SIZE; separate runs) of the C2 bench + calibration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- $B > gpurun_out/pmc_$c.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/calib_$c -o run --output-format csv -- tools/ubench/calib > gpurun_out/calib_$c.log 2>&1 || exit $?
done
find gpurun_out/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -3
echo pmc done
