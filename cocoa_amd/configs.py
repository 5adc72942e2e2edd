"""The BASELINE.json workloads as seeded synthetic problems (SURVEY.md section 8
table and 8(d)), and one rank's share of them.

C1 is the reference demo (data/small_*.dat via run-demo-local.sh); C2-C4 are
the synthetic shapes below; C5 is C2 with each of the five methods.  There is
no dataset download: every config is generated from its seed, and a rank
generates only its own rows.

Scaling modes (BASELINE.json names both kinds of config):
  weak   -- every rank holds its own n-row shard of one seeded problem with
            `parts` partitions, so K = parts * world and n = n * world globally
            (H = n/K is unchanged);
  strong -- one fixed problem (n rows, K = parts partitions) whose partitions
            are split into contiguous blocks: rank r owns partitions
            [r K / N, (r+1) K / N) (CoCoA.scala:28: K is data.partitions.size,
            hingeDriver.scala:70-71: H = n / K), test rows split by row range.
"""
from dataclasses import dataclass

import numpy as np

from .data import LabeledData, gen_synthetic

SEED = 12345
_SYN = "synthetic: seeded {} generator ({}); no dataset download"
CONFIGS = {
    "c2": dict(kind="rcv1", n=677399, d=47236, nnz=75.6, parts=64, lam=1e-4, n_test=50000, shape="rcv1-shaped",
               data=_SYN.format("rcv1-shaped", "Zipf columns, unit-norm tf-idf-like rows, planted separator + 10% noise")),
    "c3": dict(kind="epsilon", n=400000, d=2000, nnz=2000.0, parts=64, lam=1e-4, n_test=10000,
               shape="epsilon-shaped dense",
               data=_SYN.format("epsilon-shaped", "dense N(0,1) rows, L2-normalised, planted separator")),
    "c4": dict(kind="url", n=2396130, d=3231961, nnz=116.0, parts=1024, lam=1e-4, n_test=20000,
               shape="url-shaped very sparse",
               data=_SYN.format("url-shaped", "heavy-Zipf columns, ~116 nnz/row, planted separator")),
}


def balanced(n, K):
    """Contiguous balanced row blocks: partition k = rows [n k / K, n (k+1) / K)."""
    return np.array([(n * k) // K for k in range(K + 1)], np.int64)


def shard_bounds(K, world, rank):
    """Contiguous partition block [k0, k1) of rank `rank`."""
    return (K * rank) // world, (K * (rank + 1)) // world


@dataclass
class Share:
    train: LabeledData       # this rank's partitions (part_ptr local)
    test: LabeledData        # this rank's test rows
    n_glob: int              # Params.n
    k_glob: int              # data.partitions.size
    part_begin: int          # global index of this rank's first partition
    H: int                   # localIters = max(1, floor(localIterFrac * n / K))
    lam: float


def _rows(kind, r0, r1, d, nnz, seed, threads):
    """Rows [r0, r1) of the seeded stream (the generator starts at multiples of 4096)."""
    g0 = (r0 // 4096) * 4096
    allr = gen_synthetic(kind, r1 - g0, d, nnz, 1, seed, first_row=g0, threads=threads)
    return allr.row_range(r0 - g0, r1 - g0)


def share(config, rank=0, world=1, scaling="weak", n=None, d=None, nnz=None, parts=None, lam=None, n_test=None,
          threads=0, local_iter_frac=1.0):
    cfg = dict(CONFIGS[config])
    for k, v in (("n", n), ("d", d), ("nnz", nnz), ("parts", parts), ("lam", lam), ("n_test", n_test)):
        if v is not None:
            cfg[k] = v
    n, d, nnz, parts, n_test, kind = cfg["n"], cfg["d"], cfg["nnz"], cfg["parts"], cfg["n_test"], cfg["kind"]
    if scaling == "weak":
        rows = n + n_test
        stride = ((rows + 4095) // 4096) * 4096
        allr = gen_synthetic(kind, rows, d, nnz, 1, SEED, first_row=rank * stride, threads=threads)
        tr = allr.row_range(0, n)
        tr.part_ptr = balanced(n, parts)
        te = allr.row_range(n, rows)
        n_glob, k_glob, part_begin = n * world, parts * world, rank * parts
    elif scaling == "strong":
        if parts % world:
            raise ValueError("strong scaling needs K divisible by the number of ranks")
        k0, k1 = shard_bounds(parts, world, rank)
        pp = balanced(n, parts)
        r0, r1 = int(pp[k0]), int(pp[k1])
        tr = _rows(kind, r0, r1, d, nnz, SEED, threads)
        tr.part_ptr = (pp[k0:k1 + 1] - r0).astype(np.int64)
        t0, t1 = shard_bounds(n_test, world, rank)
        te = _rows(kind, n + t0, n + t1, d, nnz, SEED, threads)
        n_glob, k_glob, part_begin = n, parts, k0
    else:
        raise ValueError("scaling must be 'weak' or 'strong'")
    H = max(int(local_iter_frac * n_glob / k_glob), 1)  # hingeDriver.scala:70-71
    return Share(tr, te, n_glob, k_glob, part_begin, H, cfg["lam"])
