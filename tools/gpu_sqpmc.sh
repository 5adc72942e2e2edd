#!/bin/bash
# SQ instruction-mix counters for the solver kernel (C2), one rocprofv3 pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1 || true
grep -o "SQ_INSTS_[A-Z_]*\|SQ_WAIT_[A-Z_]*\|SQ_WAVE_CYCLES\|SQ_WAVES\|SQ_BUSY_CYCLES\|SQ_ACTIVE_INST_[A-Z_]*\|SQ_INST_CYCLES_[A-Z_]*" gpurun_out/counters_avail.txt | sort -u | tr '\n' ' '; echo
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/sq1 -o run --output-format csv -- python3 tools/prof_solver.py --rounds 1 > gpurun_out/sq1.log 2>&1 || exit $?
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/sq2 -o run --output-format csv -- python3 tools/prof_solver.py --rounds 1 > gpurun_out/sq2.log 2>&1 || echo "pass2 rc=$?"
python3 - <<'PY'
import csv, collections, glob
for d in ("gpurun_out/sq1", "gpurun_out/sq2"):
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True) + glob.glob(d + "/run_counter_collection.csv"):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "solver_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f, {k: sum(v) / len(v) for k, v in agg.items()})
PY
