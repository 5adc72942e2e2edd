"""Gram rows by runs of batches (gram_seq_kernel, solver_gram.h) against the
per-window kernel (gram_kernel, COCOA_GRAM_SEQ=0) and the oracle: the Gram
entries G(s, j) = x_s . x_j of every window feed the chain's corrections
(CoCoA.scala:157-163 through x . deltaW), so a wrong or missing entry moves
w and alpha.  Cases: C2-shaped rows with several chunk counts (chunk borders
inside a partition), windows whose cold entries overflow the LDS pool (the
fallback list, recomputed by gram_list_kernel), batches longer than the
register chunk, and the edge rows of test_gpu_gram.py."""
import numpy as np
import pytest

from cocoa_amd import Engine, configs
from cocoa_amd.data import LabeledData
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def _run(monkeypatch, tr, method, H, T, seq, chunks=None, lam=2e-3):
    monkeypatch.setenv("COCOA_GRAM_SEQ", "1" if seq else "0")
    if chunks is not None:
        monkeypatch.setenv("COCOA_GRAM_CHUNKS", str(chunks))
    else:
        monkeypatch.delenv("COCOA_GRAM_CHUNKS", raising=False)
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_solver("gram")
    e.init(method, tr.n, T, H, lam, 1.0, 1.0, 1, 3)
    for t in range(1, T + 1):
        e.round(t)
    plan = dict(e.plan(), gram_fallback_last=e.gram_fallback_count())
    monkeypatch.delenv("COCOA_GRAM_SEQ")
    monkeypatch.delenv("COCOA_GRAM_CHUNKS", raising=False)
    return e, plan


def _oracle(tr, method, H, T, lam=2e-3):
    run = oracle.Run(odata(tr), method, tr.n, H, lam, 1.0, 1.0, seed=3, nthreads=8)
    for t in range(1, T + 1):
        run.round(t)
    return run


def _check(e, run, ref=None):
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL
    if ref is not None:  # the per-window kernel's run: the same rounds far inside the tolerance
        assert np.max(np.abs(e.w() - ref.w())) <= 1e-12 * np.max(np.abs(wr))


def _c2_small():
    return configs.share("c2", n=48000, parts=16, n_test=100).train


@pytest.mark.parametrize("method", ["cocoa+", "cocoa"])
def test_gram_seq_c2_rows_match_per_window_kernel_and_oracle(method, monkeypatch):
    tr = _c2_small()
    H, T = tr.n // 16, 3
    ref, rp = _run(monkeypatch, tr, method, H, T, False)
    assert rp["gram_chunks"] == 0
    run = _oracle(tr, method, H, T, 2e-3)
    for chunks in (1, 2, 5):
        e, plan = _run(monkeypatch, tr, method, H, T, True, chunks)
        # (C2 batches rarely pass the 3,072-entry register chunk: a handful of windows on the list)
        assert plan["gram_chunks"] == chunks and 0 <= plan["gram_fallback_last"] <= 12, plan
        _check(e, run, ref)


def _cold_rows(seed, n, d, zlo, zhi):
    """Rows of uniform columns over a wide range: every entry is cold (device
    column >= 48 for nearly all), so the window's cold entries outgrow the pool."""
    rng = np.random.default_rng(seed)
    z = rng.integers(zlo, zhi + 1, size=n)
    row_ptr = np.concatenate([[0], np.cumsum(z)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(d, size=k, replace=False)) for k in z]).astype(np.int32)
    val = rng.random(row_ptr[-1]) + 0.1
    for i in range(n):  # unit-norm rows, as the demo data
        a, b = row_ptr[i], row_ptr[i + 1]
        val[a:b] /= np.linalg.norm(val[a:b])
    y = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    return row_ptr, col, val, y


@pytest.mark.parametrize("zlo,zhi", [(150, 170), (40, 220)])
def test_gram_seq_pool_overflow_goes_to_the_list_kernel(zlo, zhi, monkeypatch):
    """(150, 170): every window holds ~7,700 cold entries (pool 5,632): every
    third batch fails to fit beside the two before it; (40, 220): some windows
    fit, some do not."""
    n, d = 8000, 400000
    row_ptr, col, val, y = _cold_rows(7, n, d, zlo, zhi)
    tr = LabeledData(row_ptr, col, val, y, configs.balanced(n, 4), d)
    H, T = 1500, 3
    ref, _ = _run(monkeypatch, tr, "cocoa+", H, T, False)
    e, plan = _run(monkeypatch, tr, "cocoa+", H, T, True, 3)
    assert plan["gram_fallback_last"] > 0, plan
    if zlo == 150:  # (every third batch fails to fit beside the two before it)
        assert plan["gram_fallback_last"] >= 2 * ((H + 15) // 16), plan
    _check(e, _oracle(tr, "cocoa+", H, T), ref)


def test_gram_seq_long_batches_and_edge_rows(monkeypatch):
    """Rows of 5,000 entries (a batch past the 3,072-entry register chunk is
    never inserted: its windows go to the list), empty rows, duplicate columns,
    a one-row partition, H not a multiple of 16."""
    from tests.test_gpu_gram import _edge
    tr = _edge()
    for H in (20, 150, 601):
        ref, _ = _run(monkeypatch, tr, "cocoa+", H, 4, False)
        e, plan = _run(monkeypatch, tr, "cocoa+", H, 4, True, 2)
        _check(e, _oracle(tr, "cocoa+", H, 4), ref)


def _gram_ref(tr, samples_k, p0, H):
    """Gram rows of one partition in numpy: row j, slot s % 48 = x_s . x_j for s
    in (j, 16 floor(j / 16) + 48) within the round."""
    import scipy.sparse as sp
    X = sp.csr_matrix((tr.val, tr.col, tr.row_ptr), shape=(tr.n, tr.num_features))
    Xs = X[p0 + samples_k]
    nb = (H + 15) // 16
    G = np.zeros((nb * 16, 48))
    for g in range(nb):
        j0 = 16 * g
        blk = Xs[j0:min(j0 + 48, H)]
        D = (blk[:min(16, H - j0)] @ blk.T).toarray()
        for u in range(D.shape[0]):
            for p in range(u + 1, D.shape[1]):
                G[j0 + u, (j0 + p) % 48] = D[u, p]
    return G


def _rows_both(monkeypatch, tr, H, chunks=2):
    out = []
    for seq in (True, False):
        monkeypatch.setenv("COCOA_GRAM_SEQ", "1" if seq else "0")
        monkeypatch.setenv("COCOA_GRAM_CHUNKS", str(chunks))
        e = Engine(strict=False)
        e.set_train(tr)
        e.set_solver("gram")
        e.init("cocoa+", tr.n, 2, H, 2e-3, 1.0, 1.0, 1, 3)
        out.append((e.gram_rows(1), e.plan()))
    monkeypatch.delenv("COCOA_GRAM_SEQ")
    monkeypatch.delenv("COCOA_GRAM_CHUNKS")
    return out


@pytest.mark.parametrize("case", ["c2", "edge", "cold"])
def test_gram_rows_seq_equal_per_window_kernel_and_numpy(case, monkeypatch):
    """The Gram rows themselves (cocoa_debug_gram_rows, no solver): the
    sequential kernel's equal the per-window kernel's within summation-order
    rounding, and a numpy restatement for two partitions."""
    import cocoa_amd
    if case == "c2":
        tr, H = _c2_small(), 3000
    elif case == "edge":
        from tests.test_gpu_gram import _edge
        tr, H = _edge(), 150
    else:
        n, d = 8000, 400000
        row_ptr, col, val, y = _cold_rows(7, n, d, 40, 220)
        tr, H = LabeledData(row_ptr, col, val, y, configs.balanced(n, 4), d), 1500
    (a, pa), (b, pb) = _rows_both(monkeypatch, tr, H)
    assert pa["gram_chunks"] == 2 and pb["gram_chunks"] == 0
    assert np.max(np.abs(a - b)) <= 1e-12 * max(1.0, np.max(np.abs(b))), np.argwhere(np.abs(a - b) > 1e-12)[:8]
    for k in (0, tr.num_parts - 1):
        p0, p1 = int(tr.part_ptr[k]), int(tr.part_ptr[k + 1])
        smp = cocoa_amd.jrandom_ints(3 + 1, p1 - p0, H)
        G = _gram_ref(tr, smp, p0, H)
        assert np.max(np.abs(a[k] - G)) <= 1e-12 * max(1.0, np.max(np.abs(G)))
