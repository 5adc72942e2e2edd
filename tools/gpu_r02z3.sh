#!/bin/bash
# r02 session 3: is the Gram solver slowed by the Gram kernel running beside it?
# (1) bench with the Gram rows in line (COCOA_GRAM_SERIAL=1) vs overlapped;
# (2) SQ instruction-fetch / issue counters of the overlapped bench (one PMC pass)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for sr in 1 0; do
  COCOA_GRAM_SERIAL=$sr timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-gap --steps 10 > gpurun_out/bench_serial$sr.json 2> gpurun_out/bench_serial$sr.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_serial$sr.json').readlines()[-1]);print('serial=$sr', round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['kernel_ms'].items()})"
done
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
want=""
for c in SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_IFETCH SQ_ACTIVE_INST_ANY; do
  grep -qw "$c" gpurun_out/pmc_list.txt && want="$want $c"
done
echo "SQ counters:$want"
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap"
[ -n "$want" ] && { timeout -s KILL 180 rocprofv3 --pmc $want -d gpurun_out/pmc_sq -o run --output-format csv -- $B > gpurun_out/pmc_sq.log 2>&1 || exit $?; }
want2=""
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE; do
  grep -qw "$c" gpurun_out/pmc_list.txt && want2="$want2 $c"
done
echo "SQC counters:$want2"
[ -n "$want2" ] && { timeout -s KILL 180 rocprofv3 --pmc $want2 -d gpurun_out/pmc_sqc -o run --output-format csv -- $B > gpurun_out/pmc_sqc.log 2>&1 || exit $?; }
echo done
