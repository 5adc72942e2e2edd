"""Fast mini-batch SGD in its pull form (kernels_fast.hip, mbsgd_pull_kernel):
within a round the driver's w is fixed (SGD.scala:48-58), so the round's
deltaW = sum over sampled steps of [1 - y x.w > 0] x y (SGD.scala:108-129) =
X^T c with c_r = (samples of r) y_r for the violating rows, summed column by
column over a CSC copy instead of scattered with atomics.  Same terms, another
order (fast mode): w within 1e-9 of the oracle, error counts exact, with the
rows' x.w from the last evaluation's cache (an evaluation after every round, the
bench's flow) or formed in the round, on C2 and on edge rows (empty rows,
5,000-entry rows, duplicate columns, a one-row partition)."""
import numpy as np
import pytest

from cocoa_amd import Engine, configs
from oracle import oracle
from tests.test_gpu_gram import _edge

pytestmark = pytest.mark.gpu
REL = 1e-9


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def _pair(monkeypatch, tr, H, lam, pull):
    monkeypatch.setenv("COCOA_MBSGD_PULL", "1" if pull else "0")
    e = Engine(strict=False)
    e.set_train(tr)
    e.init("mbsgd", tr.n, 10, H, lam, 1.0, 1.0, 1, 3)
    assert e.plan()["mbsgd_pull"] == (1 if pull else 0)
    monkeypatch.delenv("COCOA_MBSGD_PULL")
    return e


@pytest.mark.parametrize("evals", [True, False])
def test_mbsgd_pull_c2_vs_oracle(evals, monkeypatch):
    sh = configs.share("c2", n_test=2000)
    tr, te = sh.train, sh.test
    e = _pair(monkeypatch, tr, sh.H, sh.lam, True)
    e.set_test(te)
    run = oracle.Run(odata(tr), "mbsgd", sh.n_glob, sh.H, sh.lam, 1.0, 1.0, seed=3, nthreads=16)
    ot = odata(te)
    for t in range(1, 5):
        e.round(t)
        run.round(t)
        if evals or t == 4:
            ev, rv = e.eval(), run.eval(ot)
            assert abs(ev["primal"] - rv["primal"]) <= REL * abs(rv["primal"]), t
            assert ev["test_err_count"] == rv["test_err"], t
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))


def test_mbsgd_pull_edge_rows_vs_scatter_and_oracle(monkeypatch):
    tr = _edge()
    H, lam = 300, 2e-3
    pull = _pair(monkeypatch, tr, H, lam, True)
    scat = _pair(monkeypatch, tr, H, lam, False)
    run = oracle.Run(odata(tr), "mbsgd", tr.n, H, lam, 1.0, 1.0, seed=3)
    for t in range(1, 6):
        pull.round(t)
        scat.round(t)
        run.round(t)
        if t % 2 == 0:
            pull.eval()  # (the next round's x.w from the cache)
    wr = run.w()
    for e in (pull, scat):
        assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
