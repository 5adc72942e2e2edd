#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CHAINS=v3 bash tools/gpu_chain.sh || exit $?
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || exit $?
python3 -c "import json; j=json.loads(open('gpurun_out/b_c2.json').read().strip().splitlines()[-1]); print('c2', j['ms_per_step'], j['kernel_ms'])"
METHODS=none bash tools/gpu_configs.sh
