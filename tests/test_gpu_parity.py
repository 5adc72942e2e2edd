"""GPU parity: the HIP path (through the C ABI) against the oracle and the
golden fixtures.  Strict mode must be bitwise identical; fast mode must agree
within the north_star tolerance of 1e-9 relative (error counts exact)."""
import hashlib
import json
import os

import numpy as np
import pytest

import cocoa_amd
from cocoa_amd import Engine
from cocoa_amd.data import LabeledData
from oracle import oracle

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
TRAIN = os.path.join(G, "data", "small_train.dat")
TEST = os.path.join(G, "data", "small_test.dat")
REL = 1e-9  # BASELINE.json north_star tolerance (fp64, relative)


def _j(name):
    return json.load(open(os.path.join(G, name)))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, "<f8").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def c1():
    return cocoa_amd.load_libsvm(TRAIN, 4, 9947), cocoa_amd.load_libsvm(TEST, 4, 9947)


def odata(d):
    return oracle.Data(d.row_ptr, d.col, d.val, d.y, d.part_ptr, d.num_features)


def engine(tr, te=None, strict=True):
    e = Engine(strict=strict)
    e.set_train(tr)
    if te is not None:
        e.set_test(te)
    return e


# ---------------------------------------------------------------- sampler --
@pytest.mark.parametrize("seed", [1, 2, 7, 100, -3, 2**31 - 1])
def test_device_sampler_matches_java_random(c1, seed):
    tr, _ = c1
    e = engine(tr)
    for k in range(4):
        nl = int(tr.part_ptr[k + 1] - tr.part_ptr[k])
        got = e.samples(k, seed, 5000)
        assert np.array_equal(got, oracle.samples(seed, nl, 5000)), (k, seed)


def test_device_sampler_power_of_two_and_odd_bounds():
    # partitions of 512, 1, 3, 1000 rows: power-of-two fast path and rejection loop
    sizes = [512, 1, 3, 1000]
    n = sum(sizes)
    d = cocoa_amd.gen_synthetic("rcv1", n, 500, 10.0, 1, 5)
    d.part_ptr = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    e = engine(d)
    for k, nl in enumerate(sizes):
        for seed in (0, 9, 12345):
            assert np.array_equal(e.samples(k, seed, 3000), oracle.samples(seed, nl, 3000))


# ------------------------------------------------------ unit: localSDCA --
@pytest.mark.parametrize("plus", [True, False])
def test_local_sdca_unit_strict_matches_golden(c1, plus):
    tr, _ = c1
    fx = _j("c1_localsdca_%s.json" % ("plus" if plus else "cocoa"))
    w = np.zeros(9947)
    w[::7] = ((np.arange(0, 9947, 7) % 13) - 6) * 1e-3
    part = fx["part"]
    nl = int(tr.part_ptr[part + 1] - tr.part_ptr[part])
    a = np.zeros(nl)
    a[::3] = 0.5
    e = engine(tr, strict=True)
    da, dw = e.local_sdca(part, w, fx["H"], fx["lam"], fx["n"], a, fx["seed"], plus, fx["sigma"])
    assert sha(dw) == fx["dw_sha256"]
    assert sha(a) == fx["alpha_sha256"]
    assert sha(w) == fx["w_out_sha256"]


@pytest.mark.parametrize("plus", [True, False])
def test_local_sdca_unit_fast_within_tolerance(c1, plus):
    tr, _ = c1
    od = odata(tr)
    w = np.linspace(-0.01, 0.01, 9947)
    a0 = np.zeros(int(tr.part_ptr[3] - tr.part_ptr[2]))
    a0[::5] = 0.3
    wr, ar = w.copy(), a0.copy()
    _, dwr = oracle.local_sdca(od, 2, wr, 400, 1e-3, 2000, ar, 11, plus, 4.0)
    wg, ag = w.copy(), a0.copy()
    _, dwg = engine(tr, strict=False).local_sdca(2, wg, 400, 1e-3, 2000, ag, 11, plus, 4.0)
    assert np.max(np.abs(dwg - dwr)) <= REL * np.max(np.abs(dwr))
    assert np.max(np.abs(ag - ar)) <= REL
    assert np.max(np.abs(wg - wr)) <= REL * np.max(np.abs(wr))


# --------------------------------------------------- full runs: config C1 --
@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
def test_c1_strict_run_bitwise_golden(c1, method):
    tr, te = c1
    fx = _j("c1_%s.json" % method.replace("+", "plus"))
    cfg = _j("c1_meta.json")["config"]
    e = engine(tr, te, strict=True)
    e.init(method, tr.n, cfg["T"], cfg["H"], cfg["lam"], cfg["beta"], cfg["gamma"], cfg["debug_iter"], cfg["seed"])
    recs = {r["t"]: r for r in fx["trace"]}
    for t in range(1, cfg["T"] + 1):
        e.round(t)
        if t in recs:
            ev = e.eval()
            assert ev["primal"].hex() == recs[t]["primal"], t
            if "dual" in recs[t]:
                assert ev["dual"].hex() == recs[t]["dual"], t
                assert ev["gap"].hex() == recs[t]["gap"], t
            assert ev["test_err_count"] == recs[t]["test_err"], t
    assert sha(e.w()) == fx["w_sha256"]
    if method in ("cocoa+", "cocoa", "mbcd"):
        assert sha(e.alpha()) == fx["alpha_sha256"]


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
def test_c1_fast_run_within_tolerance(c1, method):
    tr, te = c1
    fx = _j("c1_%s.json" % method.replace("+", "plus"))
    cfg = _j("c1_meta.json")["config"]
    e = engine(tr, te, strict=False)
    e.init(method, tr.n, cfg["T"], cfg["H"], cfg["lam"], cfg["beta"], cfg["gamma"], cfg["debug_iter"], cfg["seed"])
    recs = {r["t"]: r for r in fx["trace"]}
    for t in range(1, cfg["T"] + 1):
        e.round(t)
        if t in recs:
            ev = e.eval()
            P = float.fromhex(recs[t]["primal"])
            assert abs(ev["primal"] - P) <= REL * abs(P)
            if "dual" in recs[t]:
                D = float.fromhex(recs[t]["dual"])
                assert abs(ev["dual"] - D) <= REL * abs(D)
                assert abs(ev["gap"] - (P - D)) <= REL * abs(P)
            assert ev["test_err_count"] == recs[t]["test_err"]


def test_c1_run_api_and_callback(c1):
    tr, te = c1
    seen = []
    e = engine(tr, te, strict=True)
    e.run("cocoa+", tr.n, 30, 50, 1e-3, debug_iter=10, callback=lambda t, ev: seen.append((t, ev["primal"])))
    fx = _j("c1_cocoaplus.json")
    assert [t for t, _ in seen] == [10, 20, 30]
    assert [p.hex() for _, p in seen] == [r["primal"] for r in fx["trace"][:3]]


# ------------------------------------------------------------- edge cases --
def _dataset_with_edges(seed=3):
    rng = np.random.default_rng(seed)
    d = 3000
    rows = []
    for r in range(900):
        if r % 97 == 5:
            z = 0                                   # empty row
        elif r % 131 == 7:
            z = 2500                                # longer than the LDS stream buffer
        elif r % 53 == 3:
            z = 300                                 # beyond the register fast path
        else:
            z = int(rng.integers(1, 80))
        cols = np.sort(rng.choice(d, size=z, replace=False)).astype(np.int32)
        if r % 71 == 9 and z > 3:
            cols[2] = cols[1]                       # duplicate column index in a row
        vals = rng.standard_normal(z)
        vals /= max(np.linalg.norm(vals), 1e-300)
        rows.append((cols, vals))
    row_ptr = np.concatenate([[0], np.cumsum([len(c) for c, _ in rows])]).astype(np.int64)
    y = np.where(rng.random(900) < 0.5, 1.0, -1.0)
    part = np.array([0, 250, 251, 600, 900], np.int64)   # includes a 1-row partition
    return LabeledData(row_ptr, np.concatenate([c for c, _ in rows]).astype(np.int32),
                       np.concatenate([v for _, v in rows]), y, part, d)


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
@pytest.mark.parametrize("gamma,beta", [(1.0, 1.0), (0.25, 2.0)])
def test_edge_rows_strict_bitwise_vs_oracle(method, gamma, beta):
    tr = _dataset_with_edges()
    te = tr.row_range(0, 400)
    od, ot = odata(tr), odata(te)
    H = 120
    run = oracle.Run(od, method, tr.n, H, 2e-3, beta, gamma, seed=5)
    e = engine(tr, te, strict=True)
    e.init(method, tr.n, 6, H, 2e-3, beta, gamma, 1, 5)
    for t in range(1, 7):
        run.round(t)
        e.round(t)
        ev, rv = e.eval(), run.eval(ot)
        assert ev["primal"].hex() == rv["primal"].hex(), t
        if method in ("cocoa+", "cocoa", "mbcd"):
            assert ev["gap"].hex() == rv["gap"].hex(), t
        assert ev["test_err_count"] == rv["test_err"]
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
def test_edge_rows_fast_within_tolerance(method):
    tr = _dataset_with_edges(4)
    od = odata(tr)
    run = oracle.Run(od, method, tr.n, 150, 2e-3, seed=1)
    e = engine(tr, strict=False)
    e.init(method, tr.n, 5, 150, 2e-3, 1.0, 1.0, 1, 1)
    for t in range(1, 6):
        run.round(t)
        e.round(t)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
    if method in ("cocoa+", "cocoa", "mbcd"):
        assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


def test_empty_partition_is_an_error():
    tr = _dataset_with_edges()
    tr.part_ptr = np.array([0, 250, 250, 900], np.int64)
    e = engine(tr)
    with pytest.raises(cocoa_amd.IllegalArgumentError):
        e.init("cocoa+", tr.n, 1, 10, 1e-3)


def test_fast_eval_matches_oracle_on_same_state(c1):
    tr, te = c1
    od, ot = odata(tr), odata(te)
    run = oracle.Run(od, "cocoa+", tr.n, 50, 1e-3)
    for t in range(1, 21):
        run.round(t)
    e = engine(tr, te, strict=False)
    e.init("cocoa+", tr.n, 0, 50, 1e-3)
    e.set_w(run.w())
    e.set_alpha(run.alpha())
    ev, rv = e.eval(), run.eval(ot)
    for k in ("primal", "dual"):
        assert abs(ev[k] - rv[k]) <= 1e-13 * abs(rv[k])
    assert ev["test_err_count"] == rv["test_err"]


# ------------------------------------------------ full BASELINE-size shape --
@pytest.fixture(scope="module")
def c2():
    # config C2: rcv1-shaped, n=677,399, d=47,236, K=64
    return cocoa_amd.gen_synthetic("rcv1", 677399, 47236, 75.6, 64, 12345)


def test_c2_strict_round_bitwise_vs_oracle(c2):
    H = 677399 // 64
    od = odata(c2)
    run = oracle.Run(od, "cocoa+", c2.n, H, 1e-4, nthreads=16)
    e = engine(c2, strict=True)
    e.init("cocoa+", c2.n, 2, H, 1e-4, debug_iter=1)
    for t in (1, 2):
        run.round(t)
        e.round(t)
    assert np.array_equal(e.w(), run.w())
    assert np.array_equal(e.alpha(), run.alpha())
    ev = e.eval()
    assert ev["primal"].hex() == od.primal(run.w(), 1e-4).hex()


def test_c2_fast_properties(c2):
    """Size-independent properties at full size: fast agrees with strict within
    1e-9, weak duality holds, alpha stays in the box, the gap shrinks."""
    H = 677399 // 64
    f = engine(c2, strict=False)
    s = engine(c2, strict=True)
    f.init("cocoa+", c2.n, 4, H, 1e-4)
    s.init("cocoa+", c2.n, 4, H, 1e-4)
    gaps = []
    for t in range(1, 5):
        f.round(t)
        s.round(t)
        ev = f.eval()
        assert ev["gap"] >= 0.0
        gaps.append(ev["gap"])
    ws, wf = s.w(), f.w()
    assert np.max(np.abs(wf - ws)) <= REL * np.max(np.abs(ws))
    a = f.alpha()
    assert a.min() >= 0.0 and a.max() <= 1.0
    assert gaps[-1] < gaps[0]
    es = s.eval()
    assert abs(es["primal"] - f.eval()["primal"]) <= REL * es["primal"]


def _eval_edge_data(seed=11):
    """Rows longer than both eval tile sizes (2048 / 4096 entries), empty rows
    and ragged lengths, so tiles start at every alignment mod 4."""
    rng = np.random.default_rng(seed)
    d = 9000
    rows = []
    for r in range(1500):
        if r % 89 == 4:
            z = 0
        elif r % 211 == 17:
            z = 5000
        elif r % 113 == 50:
            z = 3000
        else:
            z = int(rng.integers(1, 120))
        cols = np.sort(rng.choice(d, size=z, replace=False)).astype(np.int32)
        vals = rng.standard_normal(z)
        rows.append((cols, vals / max(np.linalg.norm(vals), 1e-300)))
    row_ptr = np.concatenate([[0], np.cumsum([len(c) for c, _ in rows])]).astype(np.int64)
    y = np.where(rng.random(1500) < 0.5, 1.0, -1.0)
    part = np.array([0, 400, 800, 1100, 1500], np.int64)
    return LabeledData(row_ptr, np.concatenate([c for c, _ in rows]).astype(np.int32),
                       np.concatenate([v for _, v in rows]), y, part, d)


def test_fast_eval_matches_oracle_edge_rows():
    """The fast eval stream kernel (OptUtils.scala:57-98) against the oracle on
    the same (w, alpha), including rows longer than a tile and empty rows."""
    tr = _eval_edge_data()
    te = tr.row_range(200, 1300)
    od, ot = odata(tr), odata(te)
    run = oracle.Run(od, "cocoa+", tr.n, 200, 2e-3, seed=3)
    for t in range(1, 4):
        run.round(t)
    e = engine(tr, te, strict=False)
    e.init("cocoa+", tr.n, 0, 200, 2e-3)
    e.set_w(run.w())
    e.set_alpha(run.alpha())
    ev, rv = e.eval(), run.eval(ot)
    for k in ("primal", "dual", "gap"):
        assert abs(ev[k] - rv[k]) <= 1e-12 * abs(rv["primal"]), k
    assert ev["test_err_count"] == rv["test_err"]


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"])
def test_double_buffered_deltaw_is_bitwise(c1, method, monkeypatch):
    """Double-buffered deltaW slices (set t & 1, the folded set re-zeroed by a
    memset on a side stream; on by default only for K_loc*d >= 1 GiB, i.e. C4)
    give the single-buffer run's w and alpha bit for bit."""
    tr, te = c1
    H = max(int(0.1 * tr.n / 4), 1)
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("COCOA_DW_DBUF", flag)
        e = engine(tr, te, strict=True)
        e.init(method, tr.n, 5, H, 1e-3)
        for t in range(1, 6):
            e.round(t)
        out.append((e.w(), e.alpha(), e.eval()["primal"]))
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2]


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd"])
def test_run_periodic_checkpoint_and_resume(c1, tmp_path, method):
    """cocoa_run saves (t, w, alpha) every chkptIter rounds (CoCoA.scala:58-62);
    cocoa_resume from the round-4 save lands bitwise on the uninterrupted
    6-round run, with the same debug evaluations after the resume point."""
    tr, te = c1
    H = max(int(0.1 * tr.n / 4), 1)
    full, evs = engine(tr, te, strict=True), {}
    full.run(method, tr.n, 6, H, 1e-3, debug_iter=1, callback=lambda t, ev: evs.__setitem__(t, ev["gap"]))
    a = engine(tr, te, strict=True)
    a.set_checkpoint_dir(str(tmp_path))
    a.run(method, tr.n, 5, H, 1e-3, debug_iter=0, chkpt_iter=2)  # saves at t = 2, 4
    path = a.checkpoint_file(method)
    assert os.path.exists(path)
    b, evb = engine(tr, te, strict=True), {}
    b.run(method, tr.n, 6, H, 1e-3, debug_iter=1, resume_from=path,
          callback=lambda t, ev: evb.__setitem__(t, ev["gap"]))
    assert sorted(evb) == [5, 6]
    assert evb == {t: evs[t] for t in (5, 6)}
    assert np.array_equal(full.w(), b.w())
    assert np.array_equal(full.alpha(), b.alpha())


@pytest.mark.parametrize("method", ["mbsgd", "localsgd"])
def test_c2_fast_sgd_matches_strict(c2, method):
    """Full-size C5 check: the fast SGD kernels (parallel mb-SGD steps, local
    SGD with the shrink folded into a scalar) against the strict kernels that
    follow SGD.scala step for step."""
    H = 677399 // 64
    f = engine(c2, strict=False)
    s = engine(c2, strict=True)
    f.init(method, c2.n, 3, H, 1e-4)
    s.init(method, c2.n, 3, H, 1e-4)
    for t in range(1, 4):
        f.round(t)
        s.round(t)
    ws, wf = s.w(), f.w()
    assert np.max(np.abs(wf - ws)) <= REL * np.max(np.abs(ws))
    es, ef = s.eval(), f.eval()
    assert abs(es["primal"] - ef["primal"]) <= REL * es["primal"]


@pytest.mark.parametrize("t", [1, 2, 3579141])
def test_localsgd_fast_step_counter_rounds(t):
    """Local SGD's step counter t0 = (t-1) H K is a Scala Int (SGD.scala:53):
    round 1 (t0 = 0, a zero shrink at step 1), round 2, and a round whose counter
    wrapped negative (the engine hands that round to the per-step kernel), each
    from a fresh w = 0 against the oracle."""
    tr = _dataset_with_edges(5)
    od = odata(tr)
    H = 150
    assert t < 10 or (t - 1) * H * 4 >= 2**31  # t = 3579141: the Int counter wraps
    run = oracle.Run(od, "localsgd", tr.n, H, 2e-3, seed=2)
    e = engine(tr, strict=False)
    e.init("localsgd", tr.n, t, H, 2e-3, 1.0, 1.0, 1, 2)
    assert e.plan()["solver"] == "gram"
    run.round(t)
    e.round(t)
    wr = run.w()
    assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))


def test_checkpoint_resume_is_bitwise(c1, tmp_path):
    """Stop after round 3, resume from the (t, w, alpha) checkpoint in a fresh
    context: rounds 4..6 land on exactly the uninterrupted run's w and alpha."""
    tr, te = c1
    H = max(int(0.1 * tr.n / 4), 1)
    a = engine(tr, te, strict=True)
    a.init("cocoa+", tr.n, 6, H, 1e-3)
    path = str(tmp_path / "c1.ckpt")
    for t in range(1, 7):
        a.round(t)
        if t == 3:
            a.save_checkpoint(path, t)
    b = engine(tr, te, strict=True)
    b.init("cocoa+", tr.n, 6, H, 1e-3)
    t0 = b.load_checkpoint(path)
    assert t0 == 3
    for t in range(t0 + 1, 7):
        b.round(t)
    assert np.array_equal(a.w(), b.w())
    assert np.array_equal(a.alpha(), b.alpha())
    # a different method / partitioning is refused, a damaged file is refused
    c = engine(tr, te, strict=True)
    c.init("cocoa", tr.n, 6, H, 1e-3)
    with pytest.raises(cocoa_amd.IllegalArgumentError):
        c.load_checkpoint(path)
    raw = bytearray(open(path, "rb").read())
    raw[200] ^= 0xFF
    bad = str(tmp_path / "bad.ckpt")
    open(bad, "wb").write(bytes(raw))
    with pytest.raises(cocoa_amd.CocoaError):
        b.load_checkpoint(bad)


@pytest.mark.parametrize("strict", [True, False])
def test_two_rank_split_round_in_one_process(c1, strict):
    """The N>1 data path on one GPU without a process group: two engines own
    partition blocks [0,2) and [2,4) of C1 (cocoa_set_train part_begin /
    num_parts_global), each runs cocoa_round_local into a torch-owned deltaW
    sum, the sums are added (what the RCCL all-reduce does), then every rank
    runs cocoa_round_apply; objectives go through cocoa_eval_finish with the
    summed scalars (DistributedCoCoA.eval).  Against a single-process oracle
    run: equal up to the re-association of the cross-rank sum."""
    import torch
    tr, te = c1
    H, lam, Kg = 50, 1e-3, 4
    engines, sums = [], []
    for r in range(2):
        k0, k1 = 2 * r, 2 * r + 2
        r0, r1 = int(tr.part_ptr[k0]), int(tr.part_ptr[k1])
        sh = tr.row_range(r0, r1)
        sh.part_ptr = (tr.part_ptr[k0:k1 + 1] - r0).astype(np.int64)
        e = Engine(strict=strict)
        e.set_train(sh, part_begin=k0, num_parts_global=Kg)
        t0, t1 = (0, 300) if r == 0 else (300, te.n)
        e.set_test(te.row_range(t0, t1))
        e.init("cocoa+", tr.n, 6, H, lam)
        buf = torch.zeros(tr.num_features, dtype=torch.float64, device="cuda")
        e.set_dw_sum_buffer(buf.data_ptr())
        engines.append(e)
        sums.append(buf)
    run = oracle.Run(odata(tr), "cocoa+", tr.n, H, lam)
    for t in range(1, 7):
        run.round(t)
        for e in engines:
            e.round_local(t)
            e.sync()
        torch.cuda.synchronize()
        tot = sums[0] + sums[1]
        for b in sums:
            b.copy_(tot)
        torch.cuda.synchronize()
        for e in engines:
            e.round_apply()
            e.sync()
    w0, w1, wr = engines[0].w(), engines[1].w(), run.w()
    assert np.array_equal(w0, w1)                      # identical bytes on every rank
    assert np.max(np.abs(w0 - wr)) <= REL * np.max(np.abs(wr))
    a = np.concatenate([engines[0].alpha(), engines[1].alpha()])
    assert np.max(np.abs(a - run.alpha())) <= REL
    evs = [e.eval() for e in engines]
    fin = engines[0].eval_finish(sum(v["hinge_sum"] for v in evs), sum(v["alpha_sum"] for v in evs),
                                 evs[0]["w_sqnorm"], sum(v["test_err_count"] for v in evs),
                                 sum(v["test_rows"] for v in evs))
    rv = run.eval(odata(te))
    assert abs(fin["primal"] - rv["primal"]) <= REL * abs(rv["primal"])
    assert abs(fin["gap"] - rv["gap"]) <= REL * abs(rv["primal"])
    assert fin["test_err_count"] == rv["test_err"]


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd"])
@pytest.mark.parametrize("strict", [True, False])
def test_dense_rows_double_stream(method, strict):
    """Dense rows (C3-like, average z > 512): the solver plan doubles the LDS
    entry stream and keeps alpha in HBM.  Strict stays bitwise, fast within
    1e-9 of the oracle."""
    rng = np.random.default_rng(5)
    # 6,000-row partitions: alpha (48 KB) no longer fits next to the doubled stream
    # and the LDS-resident vector
    n, d = 12000, 1500
    z = rng.integers(900, 1500, size=n)
    cols = [np.sort(rng.choice(d, size=int(k), replace=False)).astype(np.int32) for k in z]
    vals = [rng.standard_normal(int(k)) / np.sqrt(k) for k in z]
    row_ptr = np.concatenate([[0], np.cumsum(z)]).astype(np.int64)
    y = np.where(rng.random(n) < 0.5, 1.0, -1.0)
    tr = LabeledData(row_ptr, np.concatenate(cols), np.concatenate(vals), y,
                     np.array([0, 6000, 12000], np.int64), d)
    e = engine(tr, strict=strict)
    e.init(method, n, 4, 100, 1e-3, 1.0, 1.0, 1, 3)
    plan = e.plan()
    assert plan["stream_cap"] == 4096 and plan["alpha_lds"] == 0
    run = oracle.Run(odata(tr), method, n, 100, 1e-3, seed=3)
    for t in range(1, 5):
        e.round(t)
        run.round(t)
    if strict:
        assert np.array_equal(e.w(), run.w())
        assert np.array_equal(e.alpha(), run.alpha())
    else:
        wr = run.w()
        assert np.max(np.abs(e.w() - wr)) <= REL * np.max(np.abs(wr))
        assert np.max(np.abs(e.alpha() - run.alpha())) <= REL


# ------------------------------------------------------ pipelined evaluation --
@pytest.mark.parametrize("method", ["cocoa+", "localsgd"])
def test_eval_async_equals_eval_and_overlaps_next_round(c1, method):
    """cocoa_eval_async snapshots (w, alpha) and evaluates beside the next round:
    what eval_wait returns is bitwise what cocoa_eval returns for that state
    (same kernels, same fixed-order reductions), and a pipelined run's
    trajectory matches the in-line one within the fast-mode tolerance (the
    Gram solver's atomics differ from run to run)."""
    tr, te = c1
    H = 150
    a = engine(tr, te, strict=False)
    b = engine(tr, te, strict=False)
    for e in (a, b):
        e.init(method, tr.n, 10, H, 1e-3)
    inline, piped = [], []
    for t in range(1, 7):
        a.round(t)
        inline.append(a.eval())
        b.round(t)
        if t > 1:
            piped.append(b.eval_wait())  # round t-1's, collected while round t runs
        b.eval_async()
    piped.append(b.eval_wait())
    for t, (x, y) in enumerate(zip(inline, piped), 1):
        assert abs(x["primal"] - y["primal"]) <= REL * abs(x["primal"]), t
        if method == "cocoa+":
            assert abs(x["gap"] - y["gap"]) <= REL * abs(x["primal"]), t
        assert x["test_err_count"] == y["test_err_count"], t
    # bitwise on one state
    b.eval_async()
    z = b.eval_wait()
    w = b.eval()
    assert z["primal"].hex() == w["primal"].hex() and z["dual"].hex() == w["dual"].hex()
    assert z["test_err_count"] == w["test_err_count"]


def test_eval_async_state_errors(c1):
    tr, te = c1
    e = engine(tr, te, strict=False)
    e.init("cocoa+", tr.n, 4, 50, 1e-3)
    e.round(1)
    with pytest.raises(cocoa_amd.CocoaError):
        e.eval_wait()  # nothing pending
    e.eval_async()
    with pytest.raises(cocoa_amd.CocoaError):
        e.eval_async()  # one at a time
    with pytest.raises(cocoa_amd.CocoaError):
        e.eval()  # in-line refused while one is pending
    e.eval_wait()
    s = engine(tr, te, strict=True)
    s.init("cocoa+", tr.n, 4, 50, 1e-3)
    with pytest.raises(cocoa_amd.CocoaError):
        s.eval_async()  # strict: in line only


# ------------------------------------------- in-line eval, deferred read-back --
@pytest.mark.parametrize("strict", [False, True])
def test_eval_begin_end_is_bitwise_the_inline_eval(c1, strict):
    """cocoa_eval_begin / cocoa_eval_end with the next round enqueued in
    between (the bench's loop): every collected record is bitwise what
    cocoa_eval returned on a twin engine (strict) or within tolerance (fast:
    the Gram solver's atomics differ from run to run), and the rounds after it
    see the same x.w cache (the trajectory continues identically)."""
    tr, te = c1
    H = 150
    a = engine(tr, te, strict=strict)
    b = engine(tr, te, strict=strict)
    for e in (a, b):
        e.init("cocoa+", tr.n, 10, H, 1e-3)
    inline, deferred = [], []
    for t in range(1, 7):
        a.round(t)
        inline.append(a.eval())
        b.round(t)
        if t > 1:
            deferred.append(b.eval_end())  # round t-1's, read back with round t queued
        b.eval_begin()
    deferred.append(b.eval_end())
    for t, (x, y) in enumerate(zip(inline, deferred), 1):
        if strict:
            assert x["primal"].hex() == y["primal"].hex() and x["gap"].hex() == y["gap"].hex(), t
        else:
            assert abs(x["gap"] - y["gap"]) <= REL * abs(x["primal"]), t
        assert x["test_err_count"] == y["test_err_count"], t
    if strict:
        assert np.array_equal(a.w(), b.w()) and np.array_equal(a.alpha(), b.alpha())
    with pytest.raises(cocoa_amd.CocoaError):
        b.eval_end()  # nothing pending
    b.eval_begin()
    with pytest.raises(cocoa_amd.CocoaError):
        b.eval()  # refused while one is pending
    b.eval_end()


def test_eval_begin_end_on_a_multi_device_context(c1):
    tr, te = c1
    g = cocoa_amd.Engine(devices=[0, 0], strict=True)
    g.set_train(tr)
    g.set_test(te)
    one = engine(tr, te, strict=True)
    for e in (g, one):
        e.init("cocoa+", tr.n, 4, 50, 1e-3)
    for t in (1, 2):
        g.round(t)
        one.round(t)
    g.eval_begin()
    g.round(3)
    x = g.eval_end()
    y = one.eval()
    assert x["gap"].hex() == y["gap"].hex()
