"""How many entries of one column class a Gram-solver batch stages (C2 shape,
CPU only): 16 sampled rows, about half of each row's entries per class.  The
LDS ring stages up to kGMaxU = 16 units (1,024 entries) per class and batch;
larger batches take the slow direct path."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cocoa_amd import configs  # noqa: E402

sh = configs.share("c2", n=200000, n_test=0, threads=8)
z = np.diff(sh.train.row_ptr)
print("row length: mean %.1f, p99 %d, max %d" % (z.mean(), np.percentile(z, 99), z.max()))
rng = np.random.default_rng(1)
per_class = rng.choice(z, size=(200000, 16)).sum(1) / 2.0
for th in (512, 640, 768, 896, 1024):
    print("P(class run of a batch > %4d entries) = %.4f" % (th, (per_class > th).mean()))
