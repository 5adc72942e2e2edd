"""The fast-mode local solvers -- the Gram-window solver (solver_gram.h) and the
chain solver -- against the oracle (CoCoA.scala:148-188, MinibatchCD.scala:
95-125) within the north_star tolerance, on data that stresses the Gram
window: empty rows, rows longer than the staging passes (5,000 entries),
duplicate column indices, a one-row partition, H below one batch (32), H not
a multiple of the batch, and the same row sampled twice inside one window."""
import numpy as np
import pytest

import cocoa_amd
from cocoa_amd import Engine
from cocoa_amd.data import LabeledData
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def _rows(seed, n, d, lens, dup_every=0):
    rng = np.random.default_rng(seed)
    rows = []
    for r in range(n):
        z = lens(r, rng)
        # Zipf-like columns so the hot (dense) and cold (hashed) Gram paths both fire
        cols = np.unique(np.minimum((rng.pareto(0.8, size=3 * z + 8) * 3).astype(np.int64), d - 1))
        if len(cols) < z:
            cols = np.unique(np.concatenate([cols, rng.choice(d, size=z, replace=False)]))
        cols = np.sort(rng.choice(cols, size=z, replace=False)).astype(np.int32) if z else np.zeros(0, np.int32)
        if dup_every and r % dup_every == 3 and z > 4:
            cols[3] = cols[2]                      # duplicate column index inside the row
        v = rng.standard_normal(z)
        rows.append((cols, v / max(np.linalg.norm(v), 1e-300)))
    row_ptr = np.concatenate([[0], np.cumsum([len(c) for c, _ in rows])]).astype(np.int64)
    y = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    return row_ptr, np.concatenate([c for c, _ in rows]).astype(np.int32), np.concatenate([v for _, v in rows]), y


def _edge(seed=21):
    n, d = 1400, 7000

    def lens(r, rng):
        if r % 97 == 5:
            return 0
        if r % 233 == 11:
            return 5000
        if r % 61 == 7:
            return 700
        return int(rng.integers(1, 140))
    row_ptr, col, val, y = _rows(seed, n, d, lens, dup_every=37)
    part = np.array([0, 600, 601, 1000, 1400], np.int64)  # includes a one-row partition
    return LabeledData(row_ptr, col, val, y, part, d)


def _small_parts(seed=5):
    # 20-row partitions: with H = 100 every window holds the same rows many times
    n, d = 80, 500
    row_ptr, col, val, y = _rows(seed, n, d, lambda r, rng: int(rng.integers(5, 60)))
    return LabeledData(row_ptr, col, val, y, np.array([0, 20, 40, 60, 80], np.int64), d)


def _run(tr, method, solver, H, T, lam=2e-3, beta=1.0, gamma=1.0):
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_solver(solver)
    e.init(method, tr.n, T, H, lam, beta, gamma, 1, 7)
    assert e.plan()["solver"] == solver
    run = oracle.Run(odata(tr), method, tr.n, H, lam, beta, gamma, seed=7)
    for t in range(1, T + 1):
        e.round(t)
        run.round(t)
    return e, run


@pytest.mark.parametrize("solver", ["gram", "chain"])
@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd"])
@pytest.mark.parametrize("H", [20, 150])
def test_fast_solver_edge_rows_within_tolerance(method, solver, H):
    tr = _edge()
    e, run = _run(tr, method, solver, H, 5, gamma=0.5 if method == "cocoa+" else 1.0)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL
    ev = e.eval()
    assert abs(ev["primal"] - run.eval()["primal"]) <= REL * run.eval()["primal"]


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd"])
def test_gram_solver_repeated_rows_in_window(method):
    """Partitions of 20 rows and H = 100: every row recurs inside one Gram
    window, so the alpha forwarding between slots is exercised constantly."""
    tr = _small_parts()
    e, run = _run(tr, method, "gram", 100, 6)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


def test_gram_is_the_default_on_sparse_rows_dense_on_dense_rows_chain_on_long_rows():
    sp = _small_parts()
    e = Engine(strict=False)
    e.set_train(sp)
    e.init("cocoa+", sp.n, 1, 10, 1e-3)
    assert e.plan()["solver"] == "gram"
    s = Engine(strict=True)
    s.set_train(sp)
    s.init("cocoa+", sp.n, 1, 10, 1e-3)
    assert s.plan()["solver"] == "chain"        # strict: the reference's summation order
    rng = np.random.default_rng(1)
    n, d = 64, 1200
    dense = LabeledData(np.arange(0, n * d + 1, d, dtype=np.int64), np.tile(np.arange(d, dtype=np.int32), n),
                        rng.standard_normal(n * d) / np.sqrt(d), np.where(rng.random(n) < .5, 1., -1.),
                        np.array([0, 32, 64], np.int64), d)
    f = Engine(strict=False)
    f.set_train(dense)
    f.init("cocoa+", n, 1, 10, 1e-3)
    assert f.plan()["solver"] == "dense"        # every row stores columns 0..d-1
    # long rows that are not dense (1,200 of 5,000 columns): the chain solver
    cols = np.concatenate([np.sort(rng.choice(5000, d, replace=False)) for _ in range(n)]).astype(np.int32)
    longr = LabeledData(dense.row_ptr, cols, dense.val, dense.y, dense.part_ptr, 5000)
    g = Engine(strict=False)
    g.set_train(longr)
    g.init("cocoa+", n, 1, 10, 1e-3)
    assert g.plan()["solver"] == "chain"
    with pytest.raises(cocoa_amd.IllegalArgumentError):
        cocoa_amd._capi.check(cocoa_amd._capi.lib().cocoa_set_solver(f.h, 9), f.h)


def _run_env(monkeypatch, env, tr, method, H, T):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_solver("gram")
    e.init(method, tr.n, T, H, 2e-3, 1.0, 0.5 if method == "cocoa+" else 1.0, 1, 7)
    for t in range(1, T + 1):
        e.round(t)
    for k in env:
        monkeypatch.delenv(k)
    return e


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "localsgd"])
def test_xw_producer_matches_the_inline_plan_and_the_oracle(method, monkeypatch):
    """Rounds with no evaluation before them take x.w from xw_produce_kernel
    beside the solver (flags polled by the loader) instead of the in-line plan:
    the same 16-lane sums, so both runs agree with each other far inside the
    tolerance and with the oracle within it (CoCoA.scala:159, SGD.scala:113)."""
    tr = _edge()
    H, T = 150, 5
    a = _run_env(monkeypatch, {}, tr, method, H, T)
    b = _run_env(monkeypatch, {"COCOA_XW_PRODUCER": "0"}, tr, method, H, T)
    assert a.plan()["xw_producer"] == 1 and b.plan()["xw_producer"] == 0
    run = oracle.Run(odata(tr), method, tr.n, H, 2e-3, 1.0, 0.5 if method == "cocoa+" else 1.0, seed=7)
    for t in range(1, T + 1):
        run.round(t)
    wr = run.w()
    for e in (a, b):
        assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
        if method != "localsgd":
            assert np.max(np.abs(e.alpha() - run.alpha())) <= REL
    assert np.max(np.abs(a.w() - b.w())) <= 1e-12 * np.max(np.abs(wr))


def test_cu_masked_side_streams_pipelined_eval(monkeypatch):
    """COCOA_CU_MASK=1: the Gram rows, x.w and pipelined-evaluation streams keep
    off 8 ceil(K/8) CUs; results are the unmasked ones (oracle tolerance), the
    pipelined evaluation (cocoa_eval_async) included."""
    tr = _edge()
    H, T = 150, 4
    monkeypatch.setenv("COCOA_CU_MASK", "1")
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_solver("gram")
    e.init("cocoa+", tr.n, T, H, 2e-3, 1.0, 0.5, 1, 7)
    assert e.plan()["side_cus_reserved"] == 8 and e.plan()["xw_producer"] == 1
    run = oracle.Run(odata(tr), "cocoa+", tr.n, H, 2e-3, 1.0, 0.5, seed=7)
    gaps, want = [], []
    for t in range(1, T + 1):
        e.round(t)
        run.round(t)
        if t > 1:
            gaps.append(e.eval_wait()["gap"])
        e.eval_async()
        want.append(run.eval())
    gaps.append(e.eval_wait()["gap"])
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert len(gaps) == T
    for g, rv in zip(gaps, want):
        assert abs(g - rv["gap"]) <= REL * abs(rv["primal"])
