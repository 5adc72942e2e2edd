#!/bin/bash
# round 6, first lease: the final tree four ways (mirror / gram_seq on and off)
# and the 64-step window (build/v_gw64, per-window Gram rows), interleaved, with
# the bench's clock telemetry; then the headline bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=100 REPS=3 TAG=ab4 tools/benchab.sh " --" "COCOA_GRAM_MIRROR=0 --" "COCOA_GRAM_SEQ=0 --" \
  "COCOA_GRAM_MIRROR=0 COCOA_GRAM_SEQ=0 --" "COCOA_LIB=build/v_gw64/libcocoa_hip.so --" \
  "COCOA_LIB=build/v_gw64/libcocoa_hip.so COCOA_GRAM_MIRROR=0 --" || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/bench_r08a.json 2> gpurun_out/bench_r08a.err || exit $?
tail -1 gpurun_out/bench_r08a.json | cut -c1-400
