"""Dense rows (config C3 shape): cocoa_set_train_dense / cocoa_set_test_dense and
the fast-mode dense local solver and evaluation (solver_dense.h).

- the dense API and the CSR API give bitwise identical strict runs (the CSR
  view of a dense matrix is what the reference's LIBSVM rows would be);
- fast mode on dense rows runs the dense solver and agrees with the CPU oracle
  within the north_star tolerance (1e-9 relative), error counts exact, for the
  three SDCA methods, H not a multiple of the kernel's step group, d in each
  of the kernel's column-chunk classes, partitions with repeated samples, and
  all-zero rows (qii = 0: alpha -> 1, CoCoA.scala:175-178).
Reference: CoCoA.scala:148-188, MinibatchCD.scala:95-125, OptUtils.scala:57-98.
"""
import numpy as np
import pytest

from cocoa_amd import Engine, LabeledData
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9


def dense_problem(n, d, K, seed, n_test=64, zero_rows=()):
    g = np.random.default_rng(seed)
    X = g.standard_normal((n, d))
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    for r in zero_rows:
        X[r] = 0.0
    ws = g.standard_normal(d)
    y = np.where(X @ ws + 0.3 * g.standard_normal(n) > 0, 1.0, -1.0)
    Xt = g.standard_normal((n_test, d))
    yt = np.where(Xt @ ws > 0, 1.0, -1.0)
    pp = np.array([(n * k) // K for k in range(K + 1)], np.int64)
    return X, y, Xt, yt, pp


def csr(X, y, pp=None):
    n, d = X.shape
    return LabeledData(np.arange(n + 1, dtype=np.int64) * d, np.tile(np.arange(d, dtype=np.int32), n),
                       X.reshape(-1).copy(), y.copy(), pp if pp is not None else np.array([0, n], np.int64), d)


def dense_engine(X, y, Xt, yt, pp, strict, solver="auto"):
    e = Engine(strict=strict)
    e.set_train_dense(X, y, pp)
    e.set_test_dense(Xt, yt)
    e.set_solver(solver)
    return e


def oracle_run(X, y, pp, method, H, lam):
    tr = csr(X, y, pp)
    od = oracle.Data(tr.row_ptr, tr.col, tr.val, tr.y, tr.part_ptr, tr.num_features)
    return oracle.Run(od, method, X.shape[0], H, lam, nthreads=8)


def oracle_test(Xt, yt):
    te = csr(Xt, yt)
    return oracle.Data(te.row_ptr, te.col, te.val, te.y, te.part_ptr, te.num_features)


@pytest.mark.parametrize("method", ["cocoa+", "cocoa"])
def test_dense_api_strict_equals_csr_api(method):
    X, y, Xt, yt, pp = dense_problem(600, 130, 4, 1)
    a = dense_engine(X, y, Xt, yt, pp, strict=True)
    b = Engine(strict=True)
    b.set_train(csr(X, y, pp))
    b.set_test(csr(Xt, yt))
    for e in (a, b):
        e.init(method, 600, 4, 150, 1e-3)
        for t in range(1, 5):
            e.round(t)
    assert np.array_equal(a.w(), b.w())
    assert np.array_equal(a.alpha(), b.alpha())
    ea, eb = a.eval(), b.eval()
    assert ea["gap"].hex() == eb["gap"].hex() and ea["test_err_count"] == eb["test_err_count"]


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd"])
@pytest.mark.parametrize("d,H", [(2000, 401), (1000, 157), (3000, 90), (64, 1000)])
def test_dense_fast_vs_oracle(method, d, H):
    n, K, lam = 2048, 8, 1e-4
    X, y, Xt, yt, pp = dense_problem(n, d, K, d + H, zero_rows=(5, 700))
    e = dense_engine(X, y, Xt, yt, pp, strict=False)
    e.init(method, n, 6, H, lam)
    assert e.plan()["solver"] == "dense"
    run = oracle_run(X, y, pp, method, H, lam)
    ot = oracle_test(Xt, yt)
    for t in range(1, 7):
        e.round(t)
        run.round(t)
        if t % 3 == 0:
            ev, rv = e.eval(), run.eval(ot)
            P = rv["primal"]
            assert abs(ev["primal"] - P) <= REL * abs(P), (t, ev["primal"], P)
            assert abs(ev["dual"] - rv["dual"]) <= REL * abs(rv["dual"])
            assert abs(ev["gap"] - rv["gap"]) <= REL * abs(P)
            assert ev["test_err_count"] == rv["test_err"]
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL
    # the all-zero rows were sampled at some point and sit at alpha = 1 (scaled)
    assert np.all(e.alpha() >= 0) and np.all(e.alpha() <= 1 + 1e-12)


def test_dense_fast_tiny_partitions_repeat_samples():
    """H >> n_k: every row is sampled many times inside one round (alpha in LDS
    is read back by later steps of the chain)."""
    X, y, Xt, yt, pp = dense_problem(96, 256, 3, 7)
    e = dense_engine(X, y, Xt, yt, pp, strict=False)
    e.init("cocoa+", 96, 5, 500, 1e-3)
    run = oracle_run(X, y, pp, "cocoa+", 500, 1e-3)
    for t in range(1, 6):
        e.round(t)
        run.round(t)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


def test_dense_solver_matches_chain_solver():
    X, y, Xt, yt, pp = dense_problem(1024, 2000, 4, 3)
    res = []
    for solver in ("dense", "chain"):
        e = dense_engine(X, y, Xt, yt, pp, strict=False, solver=solver)
        e.init("cocoa+", 1024, 3, 256, 1e-4)
        assert e.plan()["solver"] == solver
        for t in (1, 2, 3):
            e.round(t)
        res.append((e.w(), e.alpha(), e.eval()))
    (w0, a0, e0), (w1, a1, e1) = res
    assert np.max(np.abs(w0 - w1)) <= REL * np.max(np.abs(w1))
    assert np.max(np.abs(a0 - a1)) <= REL
    assert abs(e0["gap"] - e1["gap"]) <= REL * abs(e1["primal"])


def test_dense_solver_request_needs_dense_rows():
    from cocoa_amd import configs
    sh = configs.share("c2", n=4096, d=3000, nnz=20.0, parts=4, n_test=100)
    e = Engine(strict=False)
    e.set_train(sh.train)
    e.set_solver("dense")
    with pytest.raises(Exception):
        e.init("cocoa+", sh.n_glob, 2, sh.H, sh.lam)
