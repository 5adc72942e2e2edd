#!/bin/bash
# SQ instruction / wait counters of the solver (chain v1 vs v3), one pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gap"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
grep -o "SQ_[A-Z_0-9]*" gpurun_out/counters_list.txt | sort -u | tr '\n' ' ' > gpurun_out/sq_names.txt
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES"
for ch in v1 v3; do
  for p in 1 2; do
    eval C=\$C$p
    timeout -s KILL 90 env COCOA_CHAIN=$ch rocprofv3 --pmc $C -d gpurun_out/sq_${ch}_$p -o run --output-format csv -- $B > gpurun_out/sq_${ch}_$p.log 2>&1 || { echo "pass $ch $p failed"; tail -5 gpurun_out/sq_${ch}_$p.log; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/sq_v*_*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "solver_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: "%.4g" % (sum(v) / len(v)) for k, v in agg.items()})
PY
