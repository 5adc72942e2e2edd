#!/bin/bash
# Round-4 measurement lines: C5 / C3 / C4 bench lines, their rocprofv3 kernel
# stats, the C4 PMC traffic passes, and a 2-rank bench rehearsal (HOST
# transport: two ranks share the one GPU of the box; RCCL needs distinct GPUs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04g}
O=gpurun_out
TAG=$TAG tools/gpu_run.sh lines || exit $?
TAG=$TAG LINEPROF="c4 c3 c5_cocoa c5_localsgd" tools/gpu_run.sh lineprof || exit $?
TAG=${TAG}_c4 BENCH_ARGS="--config c4" tools/gpu_run.sh pmc || exit $?
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --no-cpu-baseline --no-gap \
  > $O/bench2_$TAG.json 2> $O/bench2_$TAG.err || exit $?
tail -1 $O/bench2_$TAG.json
