"""Column-list lengths of C4's compact deltaW slices: for every device column, how many of the
1,024 partitions hold it (the fold's access pattern).  CPU only."""
import numpy as np, time, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from cocoa_amd import configs
t=time.time()
sh = configs.share("c4", n_test=1000, threads=8)
tr = sh.train
print('gen', time.time()-t, tr.n, tr.nnz, flush=True)
d = tr.num_features
cnt = np.zeros(d, np.int64)
freq = np.bincount(tr.col, minlength=d)
for k in range(tr.num_parts):
    r0, r1 = tr.part_ptr[k], tr.part_ptr[k+1]
    e0, e1 = tr.row_ptr[r0], tr.row_ptr[r1]
    u = np.unique(tr.col[e0:e1])
    cnt[u] += 1
order = np.argsort(-freq, kind='stable')
L = cnt[order]
tot = L.sum()
print('sum_u', tot, 'max len', L.max())
for th in (1024, 512, 256, 128, 64, 32, 16, 8, 4, 2, 1):
    m = L >= th
    print(f'len>={th}: cols {m.sum()} entries {L[m].sum()} ({100*L[m].sum()/tot:.1f}%)')
# position of last column with len>=64 in device order
for th in (64, 256):
    idx = np.nonzero(L >= th)[0]
    print(th, 'last idx', idx.max() if len(idx) else None, 'count', len(idx))
