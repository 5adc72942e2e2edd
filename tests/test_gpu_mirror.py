"""The mirrored Gram-window solver (solver_gram.h, MIRROR; COCOA_GRAM_MIRROR=1):
two workgroups per partition, each running the chain on the same inputs and
the scatters / gathers of the deltaW columns of one parity, exchanging partial
bases through tagged granules every batch.  Both chains must form the same
coefficients, so the result is the one-workgroup solver's within summation
rounding, and the oracle's within the north_star tolerance
(CoCoA.scala:148-188), for CoCoA+ and CoCoA, on C2-shaped rows and on the
edge rows (empty rows, 5,000-entry rows past the staging ring, duplicates)."""
import numpy as np
import pytest

from cocoa_amd import Engine, configs
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def _run(monkeypatch, tr, method, H, T, mirror, lam=2e-3, gamma=1.0, evals=False):
    monkeypatch.setenv("COCOA_GRAM_MIRROR", "1" if mirror else "0")
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_solver("gram")
    e.init(method, tr.n, T, H, lam, 1.0, gamma, 1, 5)
    evs = []
    for t in range(1, T + 1):
        e.round(t)
        if evals:
            evs.append(e.eval())
    plan = e.plan()
    monkeypatch.delenv("COCOA_GRAM_MIRROR")
    return e, plan, evs


def _oracle(tr, method, H, T, lam=2e-3, gamma=1.0):
    run = oracle.Run(odata(tr), method, tr.n, H, lam, 1.0, gamma, seed=5, nthreads=8)
    for t in range(1, T + 1):
        run.round(t)
    return run


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "localsgd"])
def test_mirror_c2_rows_match_one_workgroup_and_oracle(method, monkeypatch):
    """(round 6: MbCD -- no bases, the halves tied by an alphaOld flag -- and
    local SGD -- MODE_LSGD's epilogue per parity -- mirrored too)"""
    tr = configs.share("c2", n=48000, parts=16, n_test=100).train
    H, T = tr.n // 16, 3
    one, p1, _ = _run(monkeypatch, tr, method, H, T, False)
    two, p2, _ = _run(monkeypatch, tr, method, H, T, True)
    assert p1["gram_mirror"] == 0 and p2["gram_mirror"] == 1 and p2["solver"] == "gram"
    run = _oracle(tr, method, H, T)
    wr = run.w()
    for e in (one, two):
        assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
        if method != "localsgd":
            assert np.max(np.abs(e.alpha() - run.alpha())) <= REL
    assert np.max(np.abs(two.w() - one.w())) <= 1e-12 * np.max(np.abs(wr))


def test_mirror_edge_rows(monkeypatch):
    from tests.test_gpu_gram import _edge
    tr = _edge()
    for H in (20, 150):
        two, p2, _ = _run(monkeypatch, tr, "cocoa+", H, 4, True, gamma=0.5)
        assert p2["gram_mirror"] == (1 if H > 48 else 0)  # (test_mirror_only_past_the_window)
        run = _oracle(tr, "cocoa+", H, 4, gamma=0.5)
        wr = run.w()
        assert np.max(np.abs(two.w() - wr)) <= REL * np.max(np.abs(wr))
        assert np.max(np.abs(two.alpha() - run.alpha())) <= REL


def test_mirror_deferred_eval_trajectory(monkeypatch):
    """Rounds with the evaluation after each (the bench's flow): gap and test
    errors per round as the oracle's."""
    tr = configs.share("c2", n=48000, parts=16, n_test=100).train
    te = configs.share("c2", n=48000, parts=16, n_test=2000).test
    H, T = tr.n // 16, 4
    monkeypatch.setenv("COCOA_GRAM_MIRROR", "1")
    e = Engine(strict=False)
    e.set_train(tr)
    e.set_test(te)
    e.init("cocoa+", tr.n, T, H, 1e-4, 1.0, 1.0, 1, 5)
    assert e.plan()["gram_mirror"] == 1
    run = oracle.Run(odata(tr), "cocoa+", tr.n, H, 1e-4, 1.0, 1.0, seed=5, nthreads=8)
    ot = odata(te)
    for t in range(1, T + 1):
        e.round(t)
        run.round(t)
        ev, rv = e.eval(), run.eval(ot)
        assert abs(ev["primal"] - rv["primal"]) <= REL * abs(rv["primal"])
        assert abs(ev["gap"] - rv["gap"]) <= REL * abs(rv["primal"])
        assert ev["test_err_count"] == rv["test_err"]


@pytest.mark.parametrize("H,on", [(10, 0), (48, 0), (49, 1)])
def test_mirror_only_past_the_window(H, on, monkeypatch):
    """The halves first trade partial bases at batch kGNB = 3 (48 steps).  With
    H <= 48 nothing ties them together, and a half that finished before the
    other started would overwrite the alphaOld that one still copies in (seen
    as an intermittent wrong w at H = 10, four members sharing one GPU), so the
    mirror takes only H > 48; the results match the oracle either way."""
    tr = configs.share("c2", n=12000, parts=16, n_test=100).train
    e, plan, _ = _run(monkeypatch, tr, "cocoa+", H, 3, True)
    assert plan["gram_mirror"] == on, plan
    run = _oracle(tr, "cocoa+", H, 3)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


def test_two_c2_contexts_on_one_gpu_mirrored(monkeypatch):
    """two C2-sized fast contexts sharing the one GPU, both
    mirrored (each 2 x 64 workgroups), their rounds enqueued back to back so
    they run concurrently: no hand-off abort, and each matches the oracle.  The
    halves of a pair are dispatched next to one another (solver_gram.h block
    numbering), so one context's lone halves cannot hold the CUs its partners
    (or the other context's) need."""
    monkeypatch.setenv("COCOA_GRAM_MIRROR", "1")
    sh = configs.share("c2", n_test=100)
    tr = sh.train
    H, T = sh.H, 2
    engs = []
    for seed in (5, 6):
        e = Engine(strict=False)
        e.set_train(tr)
        e.set_solver("gram")
        e.init("cocoa+", tr.n, T, H, 1e-4, 1.0, 1.0, 1, seed)
        assert e.plan()["gram_mirror"] == 1
        engs.append(e)
    for t in range(1, T + 1):
        for e in engs:
            e.round(t)  # (enqueued on each context's own stream; nothing waits in between)
    for e in engs:
        e.sync()
    for e, seed in zip(engs, (5, 6)):
        run = oracle.Run(odata(tr), "cocoa+", tr.n, H, 1e-4, 1.0, 1.0, seed=seed, nthreads=8)
        for t in range(1, T + 1):
            run.round(t)
        wr = run.w()
        assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
        assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


def test_mirror_off_when_members_share_a_device(monkeypatch):
    """a group whose members repeat an ordinal shares the device, so
    the mirrored solver (which needs both halves of every pair resident) is not
    used there; the result is the oracle's either way."""
    monkeypatch.setenv("COCOA_GRAM_MIRROR", "1")
    tr = configs.share("c2", n=48000, parts=16, n_test=100).train
    H, T = tr.n // 16, 2
    e = Engine(strict=False, devices=[0, 0])
    e.set_train(tr)
    e.set_solver("gram")
    e.init("cocoa+", tr.n, T, H, 2e-3, 1.0, 1.0, 1, 5)
    assert e.plan()["gram_mirror"] == 0
    for t in range(1, T + 1):
        e.round(t)
    run = _oracle(tr, "cocoa+", H, T)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
