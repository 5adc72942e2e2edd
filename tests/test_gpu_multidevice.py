"""One context over several devices (cocoa_create_multi): the single-driver
shape of the reference (hingeDriver.scala:84 -> CoCoA.runCoCoA, whose deltaW
reduce and `w +=` run inside the call, CoCoA.scala:45-48).

The test box has one GPU, so the "devices" are sub-contexts on device 0 (an
ordinal may repeat); the exchange is the same peer-copy code path that runs
over xGMI between distinct GPUs.  Strict mode must stay bitwise equal to the
oracle's single-process partition-order fold for all five methods; fast mode
within the north_star tolerance (1e-9 relative, error counts exact).
"""
import os

import numpy as np
import pytest

import cocoa_amd
from cocoa_amd import Engine, configs
from cocoa_amd._capi import CocoaError
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


def group(tr, te, n_dev, strict):
    e = Engine(devices=[0] * n_dev, strict=strict)
    e.set_train(tr)
    e.set_test(te)
    return e


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
@pytest.mark.parametrize("n_dev", [2, 3])
def test_strict_bitwise_vs_oracle(c1, method, n_dev):
    tr, te, od, ot = c1
    H = 50
    e = group(tr, te, n_dev, strict=True)
    assert e.devices() == [0] * n_dev
    assert e.comm_info() == {"transport": "local", "rank": 0, "world": n_dev}
    e.init(method, tr.n, 6, H, 1e-3)
    run = oracle.Run(od, method, tr.n, H, 1e-3)
    for t in range(1, 7):
        e.round(t)
        run.round(t)
    assert np.array_equal(e.w(), run.w())
    ev, rv = e.eval(), run.eval(ot)
    assert ev["primal"].hex() == rv["primal"].hex()
    assert ev["test_err_count"] == rv["test_err"]
    if method in ("cocoa+", "cocoa", "mbcd"):
        assert np.array_equal(e.alpha(), run.alpha())
        assert ev["gap"].hex() == rv["gap"].hex()


def test_fast_gram_vs_oracle(c1):
    tr, te, od, ot = c1
    e = group(tr, te, 2, strict=False)
    e.init("cocoa+", tr.n, 20, 50, 1e-3)
    assert e.plan()["solver"] == "gram" and e.plan()["n_devices"] == 2
    run = oracle.Run(od, "cocoa+", tr.n, 50, 1e-3)
    for t in range(1, 21):
        e.round(t)
        run.round(t)
    ev, rv = e.eval(), run.eval(ot)
    assert abs(ev["gap"] - rv["gap"]) <= REL * abs(rv["primal"])
    assert ev["test_err_count"] == rv["test_err"]
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


@pytest.fixture(scope="module")
def c2_small():
    sh = configs.share("c2", n=64 * 1500, n_test=4000)
    return sh, odata(sh.train), odata(sh.test)


@pytest.mark.parametrize("n_dev", [2, 4])
def test_fast_c2_shape_vs_oracle(c2_small, n_dev):
    """rcv1-shaped rows, K = 64 split over the devices (Gram-window solvers,
    device-local feature orders, the ordered sum on device 0)."""
    sh, od, ot = c2_small
    e = Engine(devices=[0] * n_dev, strict=False)
    e.set_train(sh.train)
    e.set_test(sh.test)
    e.init("cocoa+", sh.n_glob, 8, sh.H, sh.lam)
    run = oracle.Run(od, "cocoa+", sh.n_glob, sh.H, sh.lam, nthreads=8)
    for t in range(1, 9):
        e.round(t)
        run.round(t)
        if t % 4 == 0:
            ev, rv = e.eval(), run.eval(ot)
            assert abs(ev["primal"] - rv["primal"]) <= REL * abs(rv["primal"]), t
            assert abs(ev["gap"] - rv["gap"]) <= REL * abs(rv["primal"]), t
            assert ev["test_err_count"] == rv["test_err"], t
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))


def test_dense_rows_fast_vs_oracle():
    sh = configs.share("c3", n=6400, n_test=640, parts=16)
    od, ot = odata(sh.train), odata(sh.test)
    e = Engine(devices=[0, 0], strict=False)
    e.set_train(sh.train)
    e.set_test(sh.test)
    e.init("cocoa+", sh.n_glob, 5, sh.H, sh.lam)
    assert e.plan()["solver"] == "dense"
    run = oracle.Run(od, "cocoa+", sh.n_glob, sh.H, sh.lam, nthreads=8)
    for t in range(1, 6):
        e.round(t)
        run.round(t)
    ev, rv = e.eval(), run.eval(ot)
    assert abs(ev["gap"] - rv["gap"]) <= REL * abs(rv["primal"])
    assert ev["test_err_count"] == rv["test_err"]


def test_run_callback_and_checkpoint_interchange(c1, tmp_path):
    """cocoa_run on the group reports the single-device trajectory; a group
    checkpoint resumes on a one-device context (and back) bitwise."""
    tr, te, od, ot = c1
    H = 50
    one = Engine(strict=True)
    one.set_train(tr)
    one.set_test(te)
    traj1, trajg = [], []
    one.run("cocoa+", tr.n, 20, H, 1e-3, debug_iter=5, callback=lambda t, ev: traj1.append((t, ev["gap"].hex())))
    g = group(tr, te, 2, strict=True)
    g.run("cocoa+", tr.n, 20, H, 1e-3, debug_iter=5, callback=lambda t, ev: trajg.append((t, ev["gap"].hex())))
    assert traj1 == trajg and len(traj1) == 4
    assert np.array_equal(one.w(), g.w()) and np.array_equal(one.alpha(), g.alpha())

    # group -> file -> one device, 5 more rounds each way
    g.init("cocoa+", tr.n, 20, H, 1e-3)
    for t in range(1, 6):
        g.round(t)
    path = str(tmp_path / "g.ck")
    g.save_checkpoint(path, 5)
    one.init("cocoa+", tr.n, 20, H, 1e-3)
    assert one.load_checkpoint(path) == 5
    for t in range(6, 11):
        g.round(t)
        one.round(t)
    assert np.array_equal(one.w(), g.w()) and np.array_equal(one.alpha(), g.alpha())
    path2 = str(tmp_path / "one.ck")
    one.save_checkpoint(path2, 10)
    g.init("cocoa+", tr.n, 20, H, 1e-3)
    assert g.load_checkpoint(path2) == 10
    g.round(11)
    one.round(11)
    assert np.array_equal(one.w(), g.w()) and np.array_equal(one.alpha(), g.alpha())


def test_unit_entry_points_route_to_the_owning_device(c1):
    tr, te, od, ot = c1
    g = group(tr, te, 3, strict=True)
    one = Engine(strict=True)
    one.set_train(tr)
    for part in range(4):
        assert np.array_equal(g.samples(part, 7, 40), one.samples(part, 7, 40))
        n_k = int(tr.part_ptr[part + 1] - tr.part_ptr[part])
        w1 = np.zeros(tr.num_features)
        a1 = np.zeros(n_k)
        w2, a2 = w1.copy(), a1.copy()
        da1, dw1 = one.local_sdca(part, w1, 50, 1e-3, tr.n, a1, 3, True, 4.0)
        da2, dw2 = g.local_sdca(part, w2, 50, 1e-3, tr.n, a2, 3, True, 4.0)
        assert np.array_equal(dw1, dw2) and np.array_equal(da1, da2) and np.array_equal(a1, a2)


def test_caller_driven_exchange_is_rejected(c1):
    tr, te, od, ot = c1
    g = group(tr, te, 2, strict=False)
    g.init("cocoa+", tr.n, 2, 50, 1e-3)
    with pytest.raises(CocoaError):
        g.round_local(1)
    with pytest.raises(CocoaError):
        g.round_apply()
    with pytest.raises(CocoaError):
        g.dw_sum_ptr()
    stats_on = g.stats_enable(True)  # noqa: F841
    g.round(1)
    ks = g.kernel_stats()
    assert ks["solver"]["launches"] == 2  # one solver launch per device


def _tiny(d, n=48, K=4, seed=7):
    """n rows over d features (d may be below the member count: some members'
    column slices of the exchange are then empty)."""
    from cocoa_amd.data import LabeledData
    rng = np.random.default_rng(seed)
    cols, vals, rp = [], [], [0]
    for _ in range(n):
        z = int(rng.integers(0, d + 1))
        c = np.sort(rng.choice(d, size=z, replace=False)).astype(np.int32)
        cols.append(c)
        vals.append(rng.standard_normal(z))
        rp.append(rp[-1] + z)
    y = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    pp = np.array([(n * k) // K for k in range(K + 1)], np.int64)
    return LabeledData(np.array(rp, np.int64), np.concatenate(cols).astype(np.int32), np.concatenate(vals), y, pp, d)


@pytest.mark.parametrize("strict", [True, False])
def test_fewer_features_than_members(strict):
    """d = 3 over 4 members: member 0's slice of the fast exchange is empty."""
    tr = _tiny(3)
    od = odata(tr)
    e = Engine(devices=[0] * 4, strict=strict)
    e.set_train(tr)
    e.set_test(tr)
    e.init("cocoa+", tr.n, 5, 10, 1e-2)
    run = oracle.Run(od, "cocoa+", tr.n, 10, 1e-2)
    for t in range(1, 6):
        e.round(t)
        run.round(t)
    wr = run.w()
    if strict:
        assert np.array_equal(e.w(), wr) and np.array_equal(e.alpha(), run.alpha())
    else:
        assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    ev, rv = e.eval(), run.eval(od)
    assert ev["test_err_count"] == rv["test_err"]


@pytest.mark.parametrize("n_dev", [None, 2])
def test_null_column_array_with_empty_rows(n_dev):
    """cocoa_set_train / cocoa_set_test with col == NULL and every
    row empty is an (empty) CSR, not the dense layout; init, round and eval run
    and match the oracle (all-zero rows leave w = 0 and alpha = 0)."""
    from cocoa_amd import _capi as C
    n, d, K = 8, 5, 2
    rp = np.zeros(n + 1, np.int64)
    pp = np.array([0, 4, 8], np.int64)
    y = np.array([1, -1, 1, 1, -1, -1, 1, -1], np.float64)
    e = Engine(strict=False) if n_dev is None else Engine(devices=[0] * n_dev, strict=False)
    lib = C.lib()
    C.check(lib.cocoa_set_train(e.h, K, C.i64p(pp), C.i64p(rp), None, None, C.f64p(y), n, d, 0, K), e.h)
    e.d, e.n_rows, e.K_loc, e.K_glob, e.part_begin = d, n, K, K, 0
    C.check(lib.cocoa_set_test(e.h, C.i64p(rp), None, None, C.f64p(y), n), e.h)
    assert e.plan()["solver"] != "dense"
    e.init("cocoa+", n, 2, 3, 1e-2)
    e.round(1)
    e.round(2)
    ev = e.eval()
    assert np.array_equal(e.w(), np.zeros(d))
    assert ev["primal"] == 1.0 and ev["test_err_count"] == n  # hinge 1 on every row; x.w = 0 is an error
