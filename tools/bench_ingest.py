#!/usr/bin/env python3
"""Ingest timing: the host loader (16 threads) vs the GPU loader on an
rcv1-shaped LIBSVM text file (values printed with 7 significant digits, the
form of the public rcv1 files).  Prints one JSON line.

usage: python3 tools/bench_ingest.py [rows] [path]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cocoa_amd import gen_synthetic, load_libsvm  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    path = sys.argv[2] if len(sys.argv) > 2 else "/tmp/ingest_rcv1.txt"
    ds = gen_synthetic("rcv1", rows, 47236, 75.6, 1, 12345)
    t = time.time()
    with open(path, "w") as f:
        for r in range(ds.n):
            b, e = ds.row_ptr[r], ds.row_ptr[r + 1]
            f.write(("+1" if ds.y[r] > 0 else "-1") + "".join(" %d:%.7g" % (c + 1, v) for c, v in
                                                             zip(ds.col[b:e].tolist(), ds.val[b:e].tolist())) + "\n")
    gen_s = time.time() - t
    size = os.path.getsize(path)
    load_libsvm(path, 64, 47236, device=0)  # warm the device context
    res = {}
    for name, dev in (("host_16_threads", None), ("gpu", 0)):
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            d = load_libsvm(path, 64, 47236, device=dev)
            best = min(best, time.perf_counter() - t)
        res[name] = {"s": best, "MB_per_s": size / best / 1e6, "nnz": int(d.nnz)}
    a, b = load_libsvm(path, 64, 47236, device=0), load_libsvm(path, 64, 47236)
    same = bool(np.array_equal(a.row_ptr, b.row_ptr) and np.array_equal(a.col, b.col)
                and a.val.tobytes() == b.val.tobytes() and np.array_equal(a.part_ptr, b.part_ptr))
    print(json.dumps({"rows": rows, "bytes": size, "text_gen_s": gen_s, "identical": same, **res}))


if __name__ == "__main__":
    main()
