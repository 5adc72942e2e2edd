#!/bin/bash
# r02: multi-rank tests through the C ABI exchange, full GPU suite, and a
# 2-rank bench rehearsal on the box's one GPU (HOST transport).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_multirank.log 2>&1
rc=$?; echo "multirank rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_multirank.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --transport host --steps 5 --warmup 1 --no-gap > gpurun_out/bench_2rank_host.json 2> gpurun_out/bench_2rank_host.err || exit $?
tail -1 gpurun_out/bench_2rank_host.json | cut -c1-400
