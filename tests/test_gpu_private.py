"""Private columns (fast CoCoA+ on the chain solver over compact slices,
cocoa_ctx::priv_ready): a column held by one entry of a partition has no deltaW
slot.  Its deltaW is x_rc y_r (alpha_r - alpha_r^0) / (lambda n) -- the sum of
the row's updates (CoCoA.scala:181-184) -- so the chain adds the row's private
share y_r qp_r (alpha_r - alpha_r^0) / (lambda n) to its dot, its epilogue
writes each private entry's deltaW and the fold adds them.  Same arithmetic up to reassociation: the
runs agree with the oracle within 1e-9 and with COCOA_DW_PRIVATE=0 (the slot
per distinct column) far inside that.  COCOA_DW_PRIVATE is read by
cocoa_set_train.
"""
import numpy as np
import pytest

from cocoa_amd import Engine, configs
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def _run(tr, te, n_glob, H, lam, private, monkeypatch, rounds=4, seed=3, gamma=1.0):
    monkeypatch.setenv("COCOA_DW_COMPACT", "1")
    monkeypatch.setenv("COCOA_DW_PRIVATE", "1" if private else "0")
    e = Engine(strict=False)
    e.set_train(tr)
    if te is not None:
        e.set_test(te)
    e.set_solver("chain")
    e.init("cocoa+", n_glob, rounds, H, lam, 1.0, gamma, 1, seed)
    p = e.plan()
    assert p["dw_compact"] == 1 and p["dw_private"] == (1 if private else 0), p
    evs = []
    for t in range(1, rounds + 1):
        e.round(t)
        if te is not None:
            evs.append(e.eval())
    monkeypatch.delenv("COCOA_DW_PRIVATE")
    monkeypatch.delenv("COCOA_DW_COMPACT")
    return e, evs


def test_private_columns_c4_shape_vs_oracle_and_slot_layout(monkeypatch):
    sh = configs.share("c4", n=40000, d=400000, parts=32, n_test=2000)
    a, ea = _run(sh.train, sh.test, sh.n_glob, sh.H, sh.lam, True, monkeypatch)
    p = a.plan()
    assert p["fold"] == "blocks" and p["n_tail"] > 0 and p["max_uh"] * 2 < p["max_u"], p
    b, eb = _run(sh.train, sh.test, sh.n_glob, sh.H, sh.lam, False, monkeypatch)
    wb = b.w()
    assert np.max(np.abs(a.w() - wb)) <= 1e-11 * np.max(np.abs(wb))
    assert np.max(np.abs(a.alpha() - b.alpha())) <= 1e-11
    r = oracle.Run(odata(sh.train), "cocoa+", sh.n_glob, sh.H, sh.lam, seed=3, nthreads=16)
    for t in range(1, 5):
        r.round(t)
    wr = r.w()
    assert np.max(np.abs(a.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(a.alpha() - r.alpha())) <= REL
    rv = r.eval(odata(sh.test))
    ev = ea[-1]
    assert abs(ev["primal"] - rv["primal"]) <= REL * abs(rv["primal"])
    assert abs(ev["gap"] - rv["gap"]) <= REL * abs(rv["primal"])
    assert ev["test_err_count"] == rv["test_err"]
    for x, y in zip(ea, eb):
        assert abs(x["gap"] - y["gap"]) <= 1e-11 * abs(y["primal"]) and x["test_err_count"] == y["test_err_count"]


@pytest.mark.parametrize("H,gamma", [(150, 1.0), (1400, 1.0), (600, 0.5)])
def test_private_columns_edge_rows_vs_oracle(H, gamma, monkeypatch):
    """Empty rows, 5,000-entry rows (read from HBM past the stream buffer),
    duplicate columns (never private: two entries), a one-row partition (every
    column of it private), rows sampled many times per round, and gamma < 1
    (sigma' = K gamma in the private share, the fold's scaling on the tail)."""
    from tests.test_gpu_gram import _edge
    tr = _edge()
    e, _ = _run(tr, None, tr.n, H, 2e-3, True, monkeypatch, rounds=4, seed=7, gamma=gamma)
    run = oracle.Run(odata(tr), "cocoa+", tr.n, H, 2e-3, 1.0, gamma, seed=7, nthreads=8)
    for t in range(1, 5):
        run.round(t)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL
