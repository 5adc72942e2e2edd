#!/bin/bash
# Same-box A/B of bench.py settings, interleaved, two rounds:
#   tools/benchab.sh "ENV=1 -- --flag" "ENV=0 --" ...   (env assignments, "--", bench flags)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
STEPS=${STEPS:-20}
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    envs="${v%%--*}"; flags="${v#*--}"
    env X=0 $envs timeout -k 10 300 python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-gap $flags \
      > $O/ab_${i}_${rep}.json 2> $O/ab_${i}_${rep}.err || exit $?
    python3 -c "import json;d=json.loads(open('$O/ab_${i}_${rep}.json').readlines()[-1]);print('[$v]', round(d['ms_per_step'],3), {k: round(x, 3) for k, x in d['kernel_ms'].items()})"
  done
done
