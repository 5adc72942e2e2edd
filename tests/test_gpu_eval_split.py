"""The split evaluation (kernels_fast.hip eval_hot_kernel + eval_stream_kernel
BASE; cocoa_ctx::split_ready): the train rows' entries in the 4,096 most
frequent device columns are summed by a hot pass with w in LDS and no global
gather, the rest by the cold pass, which adds the hot dots and forms the
hinge / alpha / ||w|| / test-error sums (OptUtils.scala:57-98).  Checked
against the oracle and the one-pass evaluation (COCOA_EVAL_SPLIT=0) on the same
(w, alpha): C2 and C4-shaped rows (16-bit and 32-bit cold columns), rows longer
than a tile in either part (a 5,000-entry row of duplicate hot columns), empty
rows, and the next round's plan reading the x.w it stored.  Wide d (C4) adds
the warm tier (COCOA_EVAL_WARM=1, measured and not the default): columns
[4,096, 69,632) in a CSR of their own, summed into the row dots by a pass
whose w gathers stay in L2."""
import numpy as np
import pytest

from cocoa_amd import Engine, LabeledData, configs
from oracle import oracle
from tests.test_gpu_parity import _eval_edge_data

pytestmark = pytest.mark.gpu


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def _state(tr, H, lam, rounds=3):
    run = oracle.Run(odata(tr), "cocoa+", tr.n, H, lam, seed=3, nthreads=16)
    for t in range(1, rounds + 1):
        run.round(t)
    return run


def _eval(monkeypatch, tr, te, run, H, lam, split, warm=False, test_split=True):
    monkeypatch.setenv("COCOA_EVAL_SPLIT", "1" if split else "0")
    monkeypatch.setenv("COCOA_EVAL_WARM", "1" if warm else "0")
    e = Engine(strict=False)
    e.set_train(tr)
    monkeypatch.delenv("COCOA_EVAL_SPLIT")
    monkeypatch.delenv("COCOA_EVAL_WARM")
    monkeypatch.setenv("COCOA_EVAL_TEST_SPLIT", "1" if test_split else "0")
    e.set_test(te)
    monkeypatch.delenv("COCOA_EVAL_TEST_SPLIT")
    e.init("cocoa+", tr.n, 0, H, lam)
    e.set_w(run.w())
    e.set_alpha(run.alpha())
    return e, e.eval()


def _check(ev, rv, tol):
    for k in ("primal", "dual", "gap"):
        assert abs(ev[k] - rv[k]) <= tol * abs(rv["primal"]), (k, ev[k], rv[k])
    assert ev["test_err_count"] == rv["test_err"]


def _dup_rows():
    """Edge rows plus a 5,000-entry row over 60 hot columns (duplicates): its hot
    part alone passes the 4,096-entry tile."""
    tr = _eval_edge_data()
    rng = np.random.default_rng(4)
    cols = rng.integers(0, 60, size=5000).astype(np.int32)
    vals = rng.standard_normal(5000) / 70.0
    row_ptr = np.concatenate([tr.row_ptr, [tr.row_ptr[-1] + 5000]]).astype(np.int64)
    part = tr.part_ptr.copy()
    part[-1] += 1
    return LabeledData(row_ptr, np.concatenate([tr.col, cols]), np.concatenate([tr.val, vals]),
                       np.concatenate([tr.y, [1.0]]), part, tr.num_features)


@pytest.mark.parametrize("data", ["c2", "c4", "edge"])
def test_split_eval_matches_oracle_and_one_pass(data, monkeypatch):
    if data == "edge":
        tr = _dup_rows()
        te = tr.row_range(200, 1300)
        H, lam = 200, 2e-3
    else:
        sh = configs.share(data, n=60000 if data == "c2" else 40000, parts=16, n_test=3000)
        tr, te = sh.train, sh.test
        H, lam = sh.H, 1e-4
    run = _state(tr, H, lam)
    rv = run.eval(odata(te))
    e1, ev1 = _eval(monkeypatch, tr, te, run, H, lam, True)
    e0, ev0 = _eval(monkeypatch, tr, te, run, H, lam, False)
    assert e1.plan()["eval_warm"] == 0
    assert e1.plan()["eval_test_split"] == 1 and e0.plan()["eval_test_split"] == 0
    _check(ev1, rv, 1e-12)
    _check(ev0, rv, 1e-12)
    for k in ("primal", "dual", "gap"):
        assert abs(ev1[k] - ev0[k]) <= 1e-13 * abs(rv["primal"])
    if data == "c4":  # three tiers (COCOA_EVAL_WARM=1) on the same data
        e2, ev2 = _eval(monkeypatch, tr, te, run, H, lam, True, warm=True)
        assert e2.plan()["eval_warm"] == 1
        _check(ev2, rv, 1e-12)


@pytest.mark.parametrize("data", ["c2", "long_test_row", "empty_test_rows"])
def test_test_rows_split_matches_oracle_and_whole(data, monkeypatch):
    """The test rows split like the train rows (EvalArgs::th_*, on by default;
    COCOA_EVAL_TEST_SPLIT=0 keeps them whole in the cold pass): their hot
    entries summed by the hot pass into row_base[n + r], the cold pass adding
    them before the sign test.  Error counts exact against the oracle with the
    split on and off: C2-shaped rows, a test row whose hot part alone passes a
    tile (5,000 hot entries), and test rows with no entries or (mostly) cold ones."""
    if data == "c2":
        sh = configs.share("c2", n=60000, parts=16, n_test=5000)
        tr, te = sh.train, sh.test
        H, lam = sh.H, 1e-4
    else:
        tr = _dup_rows()
        H, lam = 200, 2e-3
        if data == "long_test_row":
            te = tr.row_range(tr.n - 300, tr.n)
        else:
            base = tr.row_range(0, 400)
            rp = base.row_ptr.copy()
            keep = np.ones(len(base.col), bool)
            for r in range(0, 400, 3):  # every third row empty; every third one cold-only
                keep[rp[r]:rp[r + 1]] = False
            dev_order = np.argsort(-np.bincount(tr.col, minlength=tr.num_features), kind="stable")
            hot = np.zeros(tr.num_features, bool)
            hot[dev_order[:4096]] = True
            for r in range(1, 400, 3):
                seg = slice(rp[r], rp[r + 1])
                keep[seg] &= ~hot[base.col[seg]]
            cnt = np.array([keep[rp[r]:rp[r + 1]].sum() for r in range(400)])
            row_ptr = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
            te = LabeledData(row_ptr, base.col[keep], base.val[keep], base.y, np.array([0, 400], np.int64),
                             tr.num_features)
    run = _state(tr, H, lam)
    rv = run.eval(odata(te))
    e1, ev1 = _eval(monkeypatch, tr, te, run, H, lam, True)
    e0, ev0 = _eval(monkeypatch, tr, te, run, H, lam, True, test_split=False)
    assert e1.plan()["eval_test_split"] == 1 and e0.plan()["eval_test_split"] == 0
    _check(ev1, rv, 1e-12)
    _check(ev0, rv, 1e-12)
    assert ev1["test_err_count"] == ev0["test_err_count"]


def _warm_rows():
    """Rows whose device columns fill all three tiers: 4,096 frequent columns
    (hot), 5,000 of medium frequency (warm) and ~70 k singletons (warm up to
    device column 69,632, cold past it); a row with all 5,000 medium columns
    (its warm part alone passes the 4,096-entry tile), rows with no medium
    columns, and an empty row."""
    rng = np.random.default_rng(11)
    d = 300000
    rows = []
    for i in range(1500):
        parts = [rng.integers(0, 4096, size=20), rng.integers(9096, d, size=55)]
        if i % 7:
            parts.append(rng.integers(4096, 9096, size=12))
        if i == 5:
            parts.append(np.arange(4096, 9096))
        cols = np.unique(np.concatenate(parts)) if i != 3 else np.zeros(0, np.int64)
        rows.append(cols)
    row_ptr = np.zeros(len(rows) + 1, np.int64)
    row_ptr[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.standard_normal(len(col)) / 10.0
    y = np.where(rng.random(len(rows)) < 0.5, -1.0, 1.0)
    part = np.array([0, 375, 750, 1125, 1500], np.int64)
    return LabeledData(row_ptr, col, val, y, part, d)


def test_warm_tier_edges_match_oracle(monkeypatch):
    tr = _warm_rows()
    te = tr.row_range(100, 900)
    run = _state(tr, 150, 2e-3)
    rv = run.eval(odata(te))
    e1, ev1 = _eval(monkeypatch, tr, te, run, 150, 2e-3, True, warm=True)
    assert e1.plan()["eval_warm"] == 1
    e2, ev2 = _eval(monkeypatch, tr, te, run, 150, 2e-3, True)
    assert e2.plan()["eval_warm"] == 0
    _check(ev1, rv, 1e-12)
    _check(ev2, rv, 1e-12)


def test_split_eval_xw_feeds_the_next_round(monkeypatch):
    """The cold pass stores each row's full x.w (hot + cold); the next round's
    plan takes x.w from it: CoCoA+ rounds with an evaluation after each stay
    within 1e-9 of the oracle."""
    sh = configs.share("c2", n=48000, parts=16, n_test=2000)
    tr, te = sh.train, sh.test
    H = sh.H
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_test(te)
    e.init("cocoa+", tr.n, 6, H, 1e-4, 1.0, 1.0, 1, 5)
    run = oracle.Run(odata(tr), "cocoa+", tr.n, H, 1e-4, 1.0, 1.0, seed=5, nthreads=16)
    ot = odata(te)
    for t in range(1, 7):
        e.round(t)
        run.round(t)
        _check(e.eval(), run.eval(ot), 1e-9)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= 1e-9 * np.max(np.abs(wr))
