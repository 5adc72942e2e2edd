#!/usr/bin/env python3
"""Diagnostics for the local-solver kernel on the C2 workload: per-wave busy /
barrier-wait cycles (any build) and, with COCOA_LIB=build/diag/libcocoa_hip.so,
per-step phase shares.  Prints a JSON summary."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cocoa_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=677399)
    ap.add_argument("--d", type=int, default=47236)
    ap.add_argument("--parts", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--strict", action="store_true")
    ap.add_argument("--method", default="cocoa+")
    ap.add_argument("--kind", default="rcv1")
    ap.add_argument("--nnz", type=float, default=75.6)
    args = ap.parse_args()
    d = cocoa_amd.gen_synthetic(args.kind, args.n, args.d, args.nnz, args.parts, 12345)
    H = args.n // args.parts
    e = cocoa_amd.Engine(strict=args.strict)
    e.set_train(d)
    e.init(args.method, d.n, 100, H, 1e-4)
    e.round(1)
    e.solver_profile(True)
    e.stats_enable(True)
    out = []
    for t in range(2, 2 + args.rounds):
        e.round(t)
        p = e.solver_profile_read().astype(np.float64)
        st = e.kernel_stats()
        comp, load = p[:, 0, :], p[:, 1, :]
        e.stats_reset()
        rec = {"t": t, "solver_ms_total": st["solver"]["total_ms"],
               "compute_busy_cyc_mean": comp[:, 0].mean(), "compute_wait_cyc_mean": comp[:, 1].mean(),
               "loader_busy_cyc_mean": load[:, 0].mean(), "loader_wait_cyc_mean": load[:, 1].mean(),
               "batches_mean": comp[:, 2].mean(),
               "cyc_per_step_compute": comp[:, 0].mean() / H, "cyc_per_step_total": (comp[:, 0] + comp[:, 1]).mean() / H,
               "step_phase_cyc_per_step": (comp[:, 3:9].mean(axis=0) / H).tolist()}
        out.append(rec)
    print(json.dumps({"lib": os.environ.get("COCOA_LIB", "default"), "tag": "serial" if os.environ.get("COCOA_DBG_SERIAL") else "overlap", "plan": e.plan(), "H": H, "records": out}))


if __name__ == "__main__":
    main()
