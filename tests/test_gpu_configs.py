"""GPU parity on every BASELINE.json config (C2-C5) against the CPU oracle.

Strict mode must be bitwise identical to the oracle; fast mode (the bench's
mode) must agree within the north_star tolerance, 1e-9 relative in fp64, with
exact test-error counts.  For the duality gap, which is a difference of two
objectives of size ~0.1-1, the tolerance is taken relative to the primal:
|gap - gap_ref| <= 1e-9 |P_ref|.  Problems are built by cocoa_amd.configs
exactly as bench.py builds them (the same seeded generators).  Every line
DESIGN.md publishes is parity-tested at the size it is benchmarked at: C2 /
C5 at the full BASELINE size, C3 at n = 400,000 for CoCoA+ and CoCoA (and a
25,600-row cut for the quicker strict checks), C4 as the one-GPU K = 1,024
problem (and one GPU's strong-scaling share of the 8-GPU problem); the 8-GPU
splits of C3 and C4 run as one 8-member context (cocoa_create_multi).
Reference: CoCoA.scala:148-188 (local SDCA), MinibatchCD.scala:95-125,
SGD.scala:104-135, OptUtils.scala:57-98.
"""
import numpy as np
import pytest

from cocoa_amd import Engine, configs
from oracle import oracle

pytestmark = pytest.mark.gpu
REL = 1e-9
THREADS = 16


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def make_engine(sh, strict):
    e = Engine(strict=strict)
    e.set_train(sh.train, part_begin=sh.part_begin, num_parts_global=sh.k_glob)
    e.set_test(sh.test)
    return e


def make_run(sh, od, method):
    run = oracle.Run(od, method, sh.n_glob, sh.H, sh.lam, nthreads=THREADS)
    run.set_global_parts(sh.k_glob)
    return run


def assert_close(ev, rv, sdca, t):
    P = rv["primal"]
    assert abs(ev["primal"] - P) <= REL * abs(P), (t, ev["primal"], P)
    if sdca:
        assert abs(ev["dual"] - rv["dual"]) <= REL * abs(rv["dual"]), (t, ev["dual"], rv["dual"])
        assert abs(ev["gap"] - rv["gap"]) <= REL * abs(P), (t, ev["gap"], rv["gap"])
    assert ev["test_err_count"] == rv["test_err"], t


def assert_state_close(e, run, sdca):
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    if sdca:
        assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


# ------------------------------------------------------------------ C2 --
@pytest.fixture(scope="module")
def c2():
    sh = configs.share("c2")
    return sh, odata(sh.train), odata(sh.test)


def test_c2_fast_cocoaplus_gap_trajectory_vs_oracle(c2):
    """The bench's fresh run to duality gap 1e-4 (fast mode): P, D and gap every
    10 rounds and at the end, against the oracle's 75-round trajectory."""
    sh, od, ot = c2
    e = make_engine(sh, strict=False)
    e.init("cocoa+", sh.n_glob, 1 << 30, sh.H, sh.lam)
    run = make_run(sh, od, "cocoa+")
    last = None
    for t in range(1, 76):
        e.round(t)
        run.round(t)
        if t % 10 == 0 or t == 75:
            ev, rv = e.eval(), run.eval(ot)
            assert_close(ev, rv, True, t)
            last = rv
    assert last["gap"] <= 1e-4 * 1.01  # the trajectory reaches the bench's target
    assert_state_close(e, run, True)


@pytest.mark.parametrize("method", ["cocoa", "mbcd"])
def test_c5_strict_bitwise_vs_oracle(c2, method):
    """C5 at the C2 shape: CoCoA and mini-batch SDCA, 2 rounds, bitwise."""
    sh, od, ot = c2
    e = make_engine(sh, strict=True)
    e.init(method, sh.n_glob, 2, sh.H, sh.lam)
    run = make_run(sh, od, method)
    for t in (1, 2):
        e.round(t)
        run.round(t)
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())
    ev, rv = e.eval(), run.eval(ot)
    assert ev["primal"].hex() == rv["primal"].hex() and ev["gap"].hex() == rv["gap"].hex()
    assert ev["test_err_count"] == rv["test_err"]


@pytest.mark.parametrize("method", ["cocoa", "mbcd"])
def test_c5_fast_10_rounds_vs_oracle(c2, method):
    sh, od, ot = c2
    e = make_engine(sh, strict=False)
    e.init(method, sh.n_glob, 10, sh.H, sh.lam)
    run = make_run(sh, od, method)
    for t in range(1, 11):
        e.round(t)
        run.round(t)
        if t % 5 == 0:
            assert_close(e.eval(), run.eval(ot), True, t)
    assert_state_close(e, run, True)


@pytest.mark.parametrize("method", ["mbsgd", "localsgd"])
def test_c5_sgd_strict_vs_oracle_and_fast(c2, method):
    """mb-SGD and local SGD at the C2 shape: the strict kernels follow SGD.scala
    step for step (bitwise), the fast kernels agree within 1e-9."""
    sh, od, ot = c2
    s = make_engine(sh, strict=True)
    f = make_engine(sh, strict=False)
    s.init(method, sh.n_glob, 2, sh.H, sh.lam)
    f.init(method, sh.n_glob, 2, sh.H, sh.lam)
    run = make_run(sh, od, method)
    for t in (1, 2):
        s.round(t)
        f.round(t)
        run.round(t)
    assert np.array_equal(s.w(), run.w())
    rv = run.eval(ot)
    ev = s.eval()
    assert ev["primal"].hex() == rv["primal"].hex()
    assert ev["test_err_count"] == rv["test_err"]
    assert_close(f.eval(), rv, False, 2)
    assert_state_close(f, run, False)


def test_c5_localsgd_fast_gram_solver_vs_oracle(c2):
    """The C5 local-SGD line: the Gram-window solver (MODE_LSGD: w = s (wInit +
    v), the shrink in the scalar s, x.v split into base + Gram corrections) for 6
    rounds -- round 1 has the zero shrink of step 1 -- against the oracle's
    step-by-step SGD.scala restatement."""
    sh, od, ot = c2
    e = make_engine(sh, strict=False)
    e.init("localsgd", sh.n_glob, 6, sh.H, sh.lam)
    assert e.plan()["solver"] == "gram"
    run = make_run(sh, od, "localsgd")
    for t in range(1, 7):
        e.round(t)
        run.round(t)
        if t % 2 == 0:
            assert_close(e.eval(), run.eval(ot), False, t)
    assert_state_close(e, run, False)


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
def test_c5_eight_member_context_vs_oracle(c2, method):
    """BASELINE config 5's 8-GPU split as one 8-member context
    (cocoa_create_multi): the C2 problem's K = 64 partitions as 8 members x 8
    partitions, each member its own solver, fold and exchange (the peer-copy
    reduce-scatter / all-gather: the members repeat ordinal 0 on the one-GPU
    box, so the mirrored solver is off), 2 rounds of every method against the
    oracle (MinibatchCD.scala:34-58, SGD.scala:41-67, CoCoA.scala:39-56)."""
    sh, od, ot = c2
    sdca = method in ("cocoa+", "cocoa", "mbcd")
    e = Engine(devices=[0] * 8, strict=False)
    e.set_train(sh.train)
    e.set_test(sh.test)
    e.init(method, sh.n_glob, 2, sh.H, sh.lam)
    plan = e.plan()
    assert plan["n_devices"] == 8 and plan["K_loc"] == 8 and plan["gram_mirror"] == 0, plan
    run = make_run(sh, od, method)
    for t in (1, 2):
        e.round(t)
        run.round(t)
    assert_close(e.eval(), run.eval(ot), sdca, 2)
    assert_state_close(e, run, sdca)


# ------------------------------------------------------------------ C3 --
@pytest.fixture(scope="module")
def c3():
    # epsilon-shaped dense rows (d = 2,000), K = 64, 25,600 rows (H = 400)
    sh = configs.share("c3", n=25600, n_test=2000)
    return sh, odata(sh.train), odata(sh.test)


@pytest.mark.parametrize("method", ["cocoa+", "cocoa"])
def test_c3_strict_bitwise_vs_oracle(c3, method):
    sh, od, ot = c3
    e = make_engine(sh, strict=True)
    e.init(method, sh.n_glob, 3, sh.H, sh.lam)
    run = make_run(sh, od, method)
    for t in (1, 2, 3):
        e.round(t)
        run.round(t)
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())
    ev, rv = e.eval(), run.eval(ot)
    assert ev["gap"].hex() == rv["gap"].hex()
    assert ev["test_err_count"] == rv["test_err"]


@pytest.mark.parametrize("method", ["cocoa+", "cocoa"])
def test_c3_fast_vs_oracle(c3, method):
    sh, od, ot = c3
    e = make_engine(sh, strict=False)
    e.init(method, sh.n_glob, 10, sh.H, sh.lam)
    run = make_run(sh, od, method)
    for t in range(1, 11):
        e.round(t)
        run.round(t)
        if t % 5 == 0:
            assert_close(e.eval(), run.eval(ot), True, t)
    assert_state_close(e, run, True)


# ------------------------------------------------------------------ C4 --
@pytest.fixture(scope="module")
def c4():
    # url-shaped, one GPU's share of the 8-GPU problem: partitions [0, 128) of
    # K = 1,024, n = 2,396,130 globally (~300 k rows here), d = 3,231,961
    sh = configs.share("c4", rank=0, world=8, scaling="strong", n_test=8000)
    return sh, odata(sh.train), odata(sh.test)


def test_c4_strict_bitwise_vs_oracle(c4):
    """C4 with the deltaW layout at its default: compact slices (each partition's
    distinct columns only, instead of 128 x 3.23 M dense doubles = 3.3 GB)."""
    sh, od, ot = c4
    e = make_engine(sh, strict=True)
    e.init("cocoa+", sh.n_glob, 2, sh.H, sh.lam)
    assert e.plan()["dw_compact"] == 1
    run = make_run(sh, od, "cocoa+")
    for t in (1, 2):
        e.round(t)
        run.round(t)
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())
    ev, rv = e.eval(), run.eval(ot)
    assert ev["gap"].hex() == rv["gap"].hex()
    assert ev["test_err_count"] == rv["test_err"]


def test_c4_fast_vs_oracle(c4):
    sh, od, ot = c4
    e = make_engine(sh, strict=False)
    e.init("cocoa+", sh.n_glob, 3, sh.H, sh.lam)
    run = make_run(sh, od, "cocoa+")
    for t in (1, 2, 3):
        e.round(t)
        run.round(t)
    assert_close(e.eval(), run.eval(ot), True, 3)
    assert_state_close(e, run, True)


# ------------------------------------------- full-size published lines --
@pytest.fixture(scope="module")
def c3_full():
    # the bench's C3 line: n = 400,000 dense rows of d = 2,000, K = 64, H = 6,250
    sh = configs.share("c3")
    return sh, odata(sh.train), odata(sh.test)


@pytest.mark.timeout(900)
def test_c3_full_strict_bitwise_vs_oracle(c3_full):
    sh, od, ot = c3_full
    assert sh.train.n == 400000 and sh.H == 6250
    e = make_engine(sh, strict=True)
    e.init("cocoa+", sh.n_glob, 2, sh.H, sh.lam)
    run = make_run(sh, od, "cocoa+")
    for t in (1, 2):
        e.round(t)
        run.round(t)
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())
    ev, rv = e.eval(), run.eval(ot)
    assert ev["gap"].hex() == rv["gap"].hex()
    assert ev["test_err_count"] == rv["test_err"]
    del e


@pytest.mark.timeout(900)
def test_c3_full_fast_10_rounds_vs_oracle(c3_full):
    sh, od, ot = c3_full
    e = make_engine(sh, strict=False)
    e.init("cocoa+", sh.n_glob, 10, sh.H, sh.lam)
    assert e.plan()["solver"] == "dense"
    run = make_run(sh, od, "cocoa+")
    for t in range(1, 11):
        e.round(t)
        run.round(t)
        if t % 5 == 0:
            assert_close(e.eval(), run.eval(ot), True, t)
    assert_state_close(e, run, True)
    del e


@pytest.mark.timeout(900)
def test_c3_full_cocoa_strict_bitwise_vs_oracle(c3_full):
    """C3's other half, CoCoA (plus = false): scaling beta/K (CoCoA.scala:37)
    and the local solver updating the task's w in place (the alias,
    CoCoA.scala:182-184), at the benchmarked n = 400,000, 2 rounds bitwise."""
    sh, od, ot = c3_full
    e = make_engine(sh, strict=True)
    e.init("cocoa", sh.n_glob, 2, sh.H, sh.lam)
    run = make_run(sh, od, "cocoa")
    for t in (1, 2):
        e.round(t)
        run.round(t)
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())
    ev, rv = e.eval(), run.eval(ot)
    assert ev["gap"].hex() == rv["gap"].hex()
    assert ev["test_err_count"] == rv["test_err"]
    del e


@pytest.mark.timeout(900)
def test_c3_full_cocoa_fast_10_rounds_vs_oracle(c3_full):
    sh, od, ot = c3_full
    e = make_engine(sh, strict=False)
    e.init("cocoa", sh.n_glob, 10, sh.H, sh.lam)
    assert e.plan()["solver"] == "dense"
    run = make_run(sh, od, "cocoa")
    for t in range(1, 11):
        e.round(t)
        run.round(t)
        if t % 5 == 0:
            assert_close(e.eval(), run.eval(ot), True, t)
    assert_state_close(e, run, True)
    del e


@pytest.mark.timeout(900)
@pytest.mark.parametrize("method", ["cocoa+", "cocoa"])
def test_c3_full_eight_member_context_fast_vs_oracle(c3_full, method):
    """C3's 8-GPU split as ONE context over 8 members (cocoa_create_multi; the
    one-GPU pool repeats ordinal 0): 8 partitions per member, the 16 KB deltaW
    reduce-scatter + all-gather every round (CoCoA.scala:45-48), 5 rounds."""
    sh, od, ot = c3_full
    e = Engine(devices=[0] * 8, strict=False)
    e.set_train(sh.train)
    e.set_test(sh.test)
    e.init(method, sh.n_glob, 5, sh.H, sh.lam)
    plan = e.plan()
    assert plan["solver"] == "dense" and plan["n_devices"] == 8, plan
    run = make_run(sh, od, method)
    for t in range(1, 6):
        e.round(t)
        run.round(t)
    assert_close(e.eval(), run.eval(ot), True, 5)
    assert_state_close(e, run, True)
    del e


@pytest.fixture(scope="module")
def c4_full():
    # the C4 problem: n = 2,396,130, d = 3,231,961, K = 1,024
    sh = configs.share("c4", n_test=20000)
    assert sh.k_glob == 1024 and sh.train.num_parts == 1024
    return sh, odata(sh.train), odata(sh.test)


@pytest.mark.timeout(1200)
def test_c4_one_gpu_k1024_fast_vs_oracle(c4_full):
    """The C4 one-GPU line: n = 2,396,130, d = 3,231,961, K = 1,024 on one
    GPU (chain solver on compact deltaW slices), 3 rounds, exact error counts."""
    sh, od, ot = c4_full
    e = make_engine(sh, strict=False)
    e.init("cocoa+", sh.n_glob, 3, sh.H, sh.lam)
    plan = e.plan()
    assert plan["solver"] == "chain" and plan["dw_compact"] == 1 and plan["fold"] == "blocks", plan
    # four chain workgroups per CU: 1,024 partitions on 256 CUs all resident at once
    assert plan["lds_bytes"] <= 40 * 1024 and plan["stream_cap"] == 1024 and plan["alpha_lds"] == 0, plan
    assert plan["chain_hot"] >= 512, plan  # the LDS left over: each slice's most frequent columns
    run = make_run(sh, od, "cocoa+")
    for t in (1, 2, 3):
        e.round(t)
        run.round(t)
    assert_close(e.eval(), run.eval(ot), True, 3)
    assert_state_close(e, run, True)
    del e


@pytest.mark.timeout(1200)
def test_c4_eight_member_context_fast_vs_oracle(c4_full):
    """C4's "deltaW all-reduce on 8 GPUs" shape as ONE context over 8 members:
    128 partitions each (Gram-window solvers on compact slices), the 25.9 MB
    deltaW reduce-scatter + all-gather every round, 2 rounds against the
    oracle's single-process partition-order run."""
    sh, od, ot = c4_full
    e = Engine(devices=[0] * 8, strict=False)
    e.set_train(sh.train)
    e.set_test(sh.test)
    e.init("cocoa+", sh.n_glob, 2, sh.H, sh.lam)
    plan = e.plan()
    assert plan["n_devices"] == 8 and plan["dw_compact"] == 1, plan
    run = make_run(sh, od, "cocoa+")
    for t in (1, 2):
        e.round(t)
        run.round(t)
    assert_close(e.eval(), run.eval(ot), True, 2)
    assert_state_close(e, run, True)
    del e
