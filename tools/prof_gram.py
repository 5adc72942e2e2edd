"""Diagnostics for the Gram-window solver on the C2 shape: per-wave hand-off
wait cycles vs total cycles (chain, scatter, base, loader) and kernel times."""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from cocoa_amd import Engine, configs  # noqa: E402


EVAL_FLOW = "--eval" in sys.argv


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    method = args[0] if args else "cocoa+"
    sh = configs.share("c2")
    e = Engine(strict=False)
    e.set_train(sh.train, part_begin=sh.part_begin, num_parts_global=sh.k_glob)
    e.set_solver("gram")
    e.init(method, sh.n_glob, 100, sh.H, sh.lam)
    e.solver_profile(True)
    for t in (1, 2):
        e.round(t)
        if EVAL_FLOW:
            e.eval()
    e.sync()
    e.stats_reset()
    e.stats_enable(True)
    for t in (3, 4, 5):
        e.round(t)
        if EVAL_FLOW:  # the bench's flow: an evaluation behind every round (x.w of the plan from its row cache)
            e.eval()
    e.sync()
    st = e.kernel_stats()
    S = 128  # kProfStride (kernels.h)
    allp = e.solver_profile_read(e.K_loc * S + 8).astype(np.float64)
    full = allp[:e.K_loc * S].reshape(e.K_loc, S)
    nwg = e.K_loc * ((sh.H + 15) // 16)
    seq = e.plan().get("gram_chunks", 0) > 0
    names = (["B1_hot_counts(+E wait)", "bar1", "B3_insert+issue", "bar2", "C_mfma_walk", "bar3", "D_store_meta", "-"]
             if seq else ["meta_zero", "load_hot_image", "-", "hot_product", "store", "cold_insert", "cold_probe", "-"])
    gram_phases = dict(zip(names, (allp[e.K_loc * S:e.K_loc * S + 8] / nwg).tolist()))  # per batch (seq: per batch and run)
    # solver_gram.h: [k][64] = wave w at 4 w (wait cycles, total cycles), memory
    # wave c's phase cycles at 48 + 4 c; roles in the default layout (COCOA_GLAYOUT)
    nc = 4 if e.plan().get("gram_mirror") else 2  # column classes (kernels.h kGramRuns / 2 mirrored)
    roles = ["chain", "loader"] + sum([[f"memory{2*g}", f"memory{2*g+1}", f"fetch{2*g}", f"fetch{2*g+1}"]
                                        for g in range(nc // 2)], [])
    raw = full[:, :4 * len(roles)].reshape(e.K_loc, len(roles), 4)
    nb = (sh.H + 15) // 16
    out = {"method": method, "eval_flow": EVAL_FLOW, "plan": e.plan(), "kernel_ms": {k: v["total_ms"] / max(v["launches"], 1) for k, v in st.items()},
           "waves": {r: {"wait_cyc_mean": float(raw[:, i, 0].mean()), "total_cyc_mean": float(raw[:, i, 1].mean()),
                         "wait_frac": float(raw[:, i, 0].sum() / max(raw[:, i, 1].sum(), 1))}
                     for i, r in enumerate(roles)},
           "cyc_per_step_chain": float(raw[:, 0, 1].mean() / sh.H),
           "chain_base_wait_frac": {"local": float(raw[:, 0, 2].sum() / max(raw[:, 0, 1].sum(), 1)),
                                    "remote": float(raw[:, 0, 3].sum() / max(raw[:, 0, 1].sum(), 1))},
           "chain_wait_frac": {"loader": float(full[:, 48].sum() / max(raw[:, 0, 1].sum(), 1)),
                               "scatter_ring": float(full[:, 49].sum() / max(raw[:, 0, 1].sum(), 1))},
           "chain_phase_cyc_per_batch": dict(zip(["waits", "head_loads", "steps", "tail"],
                                                 (full[:, 50:54].mean(axis=0) / nb).tolist())),
           "loader_drain_frac": float(raw[:, 1, 2].sum() / max(raw[:, 1, 1].sum(), 1)),
           "loader_cyc_per_batch": float(raw[:, 1, 1].mean() / nb),
           "loader_phase_cyc_per_batch": dict(zip(["wait_drain", "load_issue", "scans", "forward_search", "records",
                                                   "layouts_marks", "gram_dma_release"],
                                                  (full[:, 56:63].mean(axis=0) / nb).tolist())),
           "memory_phases_cyc_per_batch": {
               "memory%d" % c: dict(zip(["drain", "atomics_products", "gather_issue", "scatter_prep"],
                                        (full[:, 64 + 4 * c:68 + 4 * c].mean(axis=0) / nb).tolist()))
               for c in range(nc)},
           "memory_split_cyc_per_batch": {
               "memory%d" % c: dict(zip(["scatter_atomics", "part_zero", "part_adds", "gather_fetch_wait"],
                                        (full[:, 96 + 4 * c:100 + 4 * c].mean(axis=0) / nb).tolist()))
               for c in range(2)},
           "gram_phase_cyc_per_wg": gram_phases}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
