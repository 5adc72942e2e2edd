#!/usr/bin/env python3
"""Per-launch HBM traffic of the solver and eval kernels from rocprofv3 PMC passes.

Inputs (written by tools/gpu_pmc.sh on the GPU box):
  gpurun_out/pmc_FETCH_SIZE, gpurun_out/pmc_WRITE_SIZE   -- the bench command, one counter per pass
  gpurun_out/calib_FETCH_SIZE, gpurun_out/calib_WRITE_SIZE -- tools/ubench/calib (1 GiB per kernel)
FETCH_SIZE / WRITE_SIZE are in KiB.  The calibration kernels stream exactly 1 GiB with this code's
access widths (4 B and 8 B per lane); their ratio (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of
wide streaming reads on gfx950) converts the counters to bytes.
Output: profiles/traffic.json (read by bench.py for roofline.traffic).
"""
import csv
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(d):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def pick(agg, needle, counter):
    vals = [v for (k, c), vs in agg.items() if needle in k and c == counter for v in vs]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    # tools/pmc_summary.py [SRC_DIR [TAG [OUT]]]: TAG = the tools/gpu_run.sh TAG of the passes
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
    sfx = "_" + sys.argv[2] if len(sys.argv) > 2 else ""
    pre = os.environ.get("PMC_PREFIX", "pmc_")  # (c4pmc_: tools/gpu_run.sh c4pmc)
    f, w = load(os.path.join(src, pre + "FETCH_SIZE" + sfx)), load(os.path.join(src, pre + "WRITE_SIZE" + sfx))
    cf, cw = load(os.path.join(src, "calib_FETCH_SIZE" + sfx)), load(os.path.join(src, "calib_WRITE_SIZE" + sfx))
    gib = float(1 << 30)
    k_f64 = gib / (pick(cf, "read_f64", "FETCH_SIZE")[0] * 1024)
    k_i32 = gib / (pick(cf, "read_i32", "FETCH_SIZE")[0] * 1024)
    k_w = gib / (pick(cw, "write_f64", "WRITE_SIZE")[0] * 1024)
    k_fetch = 0.5 * (k_f64 + k_i32)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of "
                     "`bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap`, calibrated by tools/ubench/calib",
           "calibration": {"fetch_bytes_per_reported_byte_f64": k_f64, "fetch_bytes_per_reported_byte_i32": k_i32,
                           "write_bytes_per_reported_byte_f64": k_w},
           "kernels": {}}
    # tag -> (substring the kernel name must hold, substrings it must not hold)
    tags = (("solver_chain", "solver_kernel<", ()), ("solver_gram", "solver_gram_kernel", ()),
            ("solver_dense", "dense_solver_kernel", ()), ("gram", "gram_kernel", ("solver_gram",)),
            ("gram_seq", "gram_seq_kernel", ()), ("gram_list", "gram_list_kernel", ()),
            ("eval", "eval_stream_kernel", ()), ("eval_hot", "eval_hot_kernel", ()),
            ("eval_dense", "eval_dense_kernel", ()),
            ("plan", "plan_kernel", ()), ("fold", "fold_kernel", ("compact",)),
            ("fold_compact", "fold_compact_kernel", ()), ("fold_blocks", "fold_blocks_kernel", ()),
            ("apply", "apply_kernel", ()))
    for tag, needle, bad in tags:
        names = sorted({k for (k, c) in f if needle in k and not any(b in k for b in bad)})
        if not names:
            continue
        # the instantiation launched most (round 1's x.w-producer form runs once)
        names.sort(key=lambda k: -pick(f, k, "FETCH_SIZE")[1])
        fe, n = pick(f, names[0], "FETCH_SIZE")
        wr, _ = pick(w, names[0], "WRITE_SIZE")
        if fe is None or wr is None:
            continue
        out["kernels"][tag] = {"kernel": names[0], "launches": n, "fetch_bytes": fe * 1024 * k_fetch,
                               "write_bytes": wr * 1024 * k_w,
                               "hbm_bytes_per_launch": fe * 1024 * k_fetch + wr * 1024 * k_w}
    # tools/pmc_summary.py SRC TAG [OUT]: another workload's passes (e.g. C4) to their own file
    dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "traffic.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
