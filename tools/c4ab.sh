#!/bin/bash
# Same-box C4 A/B over environment settings: tools/c4ab.sh "A=1" "A=0 B=2" ...
# (each setting runs twice, interleaved; default: COCOA_DW_PRIVATE=0 / 1)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
[ $# -gt 0 ] || set -- "COCOA_DW_PRIVATE=0" "COCOA_DW_PRIVATE=1"
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 300 python3 bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline --no-gap \
      > $O/c4ab_${i}_${rep}.json 2> $O/c4ab_${i}_${rep}.err
    python3 -c "import json;d=json.loads(open('$O/c4ab_${i}_${rep}.json').readlines()[-1]);print('$v', round(d['ms_per_step'],3), {k: round(x, 3) for k, x in d['kernel_ms'].items()}, 'hot', d['plan']['chain_hot'])"
  done
done
