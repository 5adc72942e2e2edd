"""The projected-gradient skip of CoCoA.scala:166-172 (MinibatchCD.scala:107-112)
on the fast solvers when alpha can leave [0, 1].

While every alpha lies in [0, 1] the clamp alone reproduces the reference's
rule (a vanishing projected gradient returns aa).  A scaling above 1 -- CoCoA+
with gamma > 1, CoCoA with beta > K -- moves alpha outside [0, 1]
(alphaOld + dAlpha * scaling, CoCoA.scala:101), and so does an alpha set from
outside (cocoa_set_alpha, a checkpoint).  The reference then skips the step
(aa <= 0 with grad >= 0, aa >= 1 with grad <= 0) where the clamp alone would
move alpha to 0 or 1; the engine switches the Gram-window and dense solvers to
their PROJ variants.  Checked against the oracle within the north_star
tolerance (1e-9 relative, error counts exact), strict bitwise.
"""
import os

import numpy as np
import pytest

import cocoa_amd
from cocoa_amd import Engine, configs
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


@pytest.fixture(scope="module")
def c1():
    tr = cocoa_amd.load_libsvm(os.path.join(G, "small_train.dat"), 4, 9947)
    te = cocoa_amd.load_libsvm(os.path.join(G, "small_test.dat"), 4, 9947)
    return tr, te, odata(tr), odata(te)


@pytest.fixture(scope="module")
def dense():
    sh = configs.share("c3", n=6400, n_test=640, parts=16)
    return sh, odata(sh.train), odata(sh.test)


def _close(e, run, ot, t, sdca=True):
    ev, rv = e.eval(), run.eval(ot)
    P = rv["primal"]
    assert abs(ev["primal"] - P) <= REL * abs(P), (t, ev["primal"], P)
    if sdca:
        assert abs(ev["gap"] - rv["gap"]) <= REL * abs(P), (t, ev["gap"], rv["gap"])
    assert ev["test_err_count"] == rv["test_err"], t
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * max(np.max(np.abs(wr)), 1e-300), t
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL * 2, t


@pytest.mark.parametrize("method,beta,gamma", [("cocoa+", 1.0, 1.5), ("cocoa", 8.0, 1.0), ("mbcd", 800.0, 1.0)])
def test_scaling_above_one_gram_vs_oracle(c1, method, beta, gamma):
    tr, te, od, ot = c1
    H = 50
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_test(te)
    e.init(method, tr.n, 12, H, 1e-3, beta=beta, gamma=gamma)
    assert e.plan()["solver"] == "gram"
    run = oracle.Run(od, method, tr.n, H, 1e-3, beta=beta, gamma=gamma)
    left = False
    for t in range(1, 13):
        e.round(t)
        run.round(t)
        a = run.alpha()
        left = left or bool(np.any((a < 0) | (a > 1)))
        if t % 4 == 0:
            _close(e, run, ot, t)
    assert left, "the scaling should have moved some alpha outside [0, 1]"


@pytest.mark.parametrize("method,beta,gamma", [("cocoa+", 1.0, 1.5), ("cocoa", 40.0, 1.0)])
def test_scaling_above_one_dense_vs_oracle(dense, method, beta, gamma):
    sh, od, ot = dense
    e = Engine(strict=False)
    e.set_train(sh.train)
    e.set_test(sh.test)
    e.init(method, sh.n_glob, 6, sh.H, sh.lam, beta=beta, gamma=gamma)
    assert e.plan()["solver"] == "dense"
    run = oracle.Run(od, method, sh.n_glob, sh.H, sh.lam, beta=beta, gamma=gamma, nthreads=8)
    for t in range(1, 7):
        e.round(t)
        run.round(t)
    assert np.any((run.alpha() < 0) | (run.alpha() > 1))
    _close(e, run, ot, 6)


@pytest.mark.parametrize("solver", ["gram", "chain"])
def test_alpha_set_outside_unit_interval(c1, solver):
    """cocoa_set_alpha with alpha in [-0.5, 1.5] (and gamma = 1): the next
    rounds follow the reference's skip rule."""
    tr, te, od, ot = c1
    H = 50
    rng = np.random.default_rng(3)
    a0 = rng.uniform(-0.5, 1.5, tr.n)
    a0[::7] = 0.0
    a0[3::7] = 1.0
    w0 = rng.standard_normal(tr.num_features) * 1e-2
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_test(te)
    e.set_solver(solver)
    e.init("cocoa+", tr.n, 4, H, 1e-3)
    e.set_w(w0)
    e.set_alpha(a0)
    run = oracle.Run(od, "cocoa+", tr.n, H, 1e-3)
    run.set_state(w0, a0)
    for t in range(1, 5):
        e.round(t)
        run.round(t)
    _close(e, run, ot, 4)


def test_scaling_above_one_strict_bitwise(c1):
    tr, te, od, ot = c1
    e = Engine(strict=True)
    e.set_train(tr)
    e.set_test(te)
    e.init("cocoa+", tr.n, 6, 50, 1e-3, gamma=1.5)
    run = oracle.Run(od, "cocoa+", tr.n, 50, 1e-3, gamma=1.5)
    for t in range(1, 7):
        e.round(t)
        run.round(t)
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())
    assert e.eval()["gap"].hex() == run.eval(ot)["gap"].hex()
