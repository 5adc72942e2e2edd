#!/usr/bin/env python3
"""Column-frequency profile of C4 partitions (private
columns): per partition its entries, distinct columns, the entry share of its
most frequent columns and of columns it holds once / twice / ...; the first
three partitions of the seeded url-shaped stream (cocoa_amd/configs.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cocoa_amd import configs
from cocoa_amd.data import gen_synthetic


def main():
    cfg = configs.CONFIGS["c4"]
    rows = cfg["n"] // cfg["parts"]
    allr = gen_synthetic("url", 4 * 4096, cfg["d"], cfg["nnz"], 1, configs.SEED, first_row=0, threads=8)
    for k in range(3):
        a = allr.row_range(k * rows, (k + 1) * rows)
        u, inv, cnt = np.unique(a.col, return_inverse=True, return_counts=True)
        order = np.argsort(-cnt, kind="stable")
        rank = np.empty_like(order)
        rank[order] = np.arange(len(u))
        er, ec = rank[inv], cnt[inv]
        print(f"partition {k}: {len(a.col)} entries, {len(u)} distinct columns, "
              f"{int(np.sum(cnt == 1))} held once ({np.mean(ec == 1):.3f} of the entries), "
              f"{int(np.sum(cnt >= 2))} held by >= 2 entries")
        print("  entry share of the top 832 / 2048 / 4096 / 16384 columns:",
              " ".join(f"{np.mean(er < m):.3f}" for m in (832, 2048, 4096, 16384)))
        print("  entry share of columns held 2 / 3 / 4 times:", " ".join(f"{np.mean(ec == f):.3f}" for f in (2, 3, 4)))


if __name__ == "__main__":
    main()
