"""Multi-rank runs through the C ABI's own exchange (cocoa_comm_init): no torch
collective in the data path, exactly what a JVM caller over FFM would drive.

* world 1 over RCCL: cocoa_round / cocoa_eval take the communicator path
  (fold -> ncclAllReduce / chain -> apply) and must give the golden C1
  results bit for bit, as the fused single-rank path does;
* 2 and 4 processes sharing the box's one GPU over the HOST transport (RCCL
  refuses two ranks on one device): contiguous partition blocks per rank
  (CoCoA.scala:28), deltaW exchanged every round (CoCoA.scala:47-48), the
  objective sums every evaluation (OptUtils.scala:65-98).  Strict mode passes
  the partition-order fold from rank to rank, so it must equal the
  single-process oracle bit for bit; fast mode (allreduce) within 1e-9.
"""
import json
import multiprocessing as mp
import os

import numpy as np
import pytest

import cocoa_amd
from cocoa_amd import Engine
from cocoa_amd.configs import shard_bounds
from cocoa_amd.engine import comm_unique_id
from oracle import oracle

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
TRAIN = os.path.join(G, "data", "small_train.dat")
TEST = os.path.join(G, "data", "small_test.dat")
METHODS = ["cocoa+", "cocoa", "mbcd", "mbsgd", "localsgd"]
T, H, LAM = 12, 50, 1e-3


def _j(name):
    return json.load(open(os.path.join(G, name)))


@pytest.mark.parametrize("method", METHODS)
def test_world1_rccl_comm_path_is_bitwise_golden(method):
    tr, te = cocoa_amd.load_libsvm(TRAIN, 4, 9947), cocoa_amd.load_libsvm(TEST, 4, 9947)
    fx = _j("c1_%s.json" % method.replace("+", "plus"))
    cfg = _j("c1_meta.json")["config"]
    e = Engine(strict=True)
    e.set_train(tr)
    e.set_test(te)
    e.comm_init("rccl", 0, 1, comm_unique_id("rccl"))
    assert e.comm_info() == {"transport": "rccl", "rank": 0, "world": 1}
    e.init(method, tr.n, cfg["T"], cfg["H"], cfg["lam"], cfg["beta"], cfg["gamma"], cfg["debug_iter"], cfg["seed"])
    recs = {r["t"]: r for r in fx["trace"]}
    for t in range(1, cfg["T"] + 1):
        e.round(t)
        if t in recs:
            ev = e.eval()
            assert ev["primal"].hex() == recs[t]["primal"], t
            assert ev["test_err_count"] == recs[t]["test_err"], t
    import hashlib
    assert hashlib.sha256(np.ascontiguousarray(e.w(), "<f8").tobytes()).hexdigest() == fx["w_sha256"]


def _rank_worker(rank, world, strict, methods, uid_q, out_q):
    try:
        tr = cocoa_amd.load_libsvm(TRAIN, 4, 9947)
        te = cocoa_amd.load_libsvm(TEST, 4, 9947)
        k0, k1 = shard_bounds(4, world, rank)
        r0, r1 = shard_bounds(te.n, world, rank)
        if rank == 0:
            uid = comm_unique_id("host")
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        e = Engine(device=0, strict=strict)
        e.set_train(tr.shard(k0, k1), part_begin=k0, num_parts_global=4)
        e.set_test(te.row_range(r0, r1))
        e.comm_init("host", rank, world, uid)
        res = {}
        for m in methods:
            e.init(m, tr.n, T, H, LAM, 1.0, 1.0, 4, 0)
            evs = []
            for t in range(1, T + 1):
                e.round(t)
                if t % 4 == 0:
                    evs.append(e.eval())
            res[m] = (e.w(), e.alpha(), evs)
        # cocoa_run drives the same exchange (the FFM / JNI caller's entry point)
        seen = []
        e.run("cocoa+", tr.n, 8, H, LAM, debug_iter=4, callback=lambda t, ev: seen.append((t, ev)))
        res["run"] = (e.w(), seen)
        e.close()
        out_q.put((rank, res))
    except Exception as ex:
        out_q.put((rank, repr(ex)))


def _spawn(world, strict, methods, target=None):
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    target = target or _rank_worker
    procs = [ctx.Process(target=target, args=(r, world, strict, methods, uid_q, out_q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(out_q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    return out


def _oracle(method, Tr=T):
    od = oracle.Data.load_libsvm(TRAIN, 4, 9947)
    ot = oracle.Data.load_libsvm(TEST, 4, 9947)
    run = oracle.Run(od, method, od.n, H, LAM)
    evs = []
    for t in range(1, Tr + 1):
        run.round(t)
        if t % 4 == 0:
            evs.append(run.eval(ot))
    return run, evs


@pytest.mark.parametrize("world", [2, 4])
def test_multirank_strict_chain_is_bitwise_single_process(world):
    out = _spawn(world, True, METHODS)
    for m in METHODS:
        run, revs = _oracle(m)
        w_ref = run.w()
        for r in range(world):
            assert out[r][m][0].tobytes() == w_ref.tobytes(), (m, r)          # identical bytes on every rank
        if m in ("cocoa+", "cocoa", "mbcd"):
            a = np.concatenate([out[r][m][1] for r in range(world)])
            assert a.tobytes() == run.alpha().tobytes(), m
        for ev, rv in zip(out[0][m][2], revs):
            assert ev["primal"].hex() == rv["primal"].hex(), m
            if m in ("cocoa+", "cocoa", "mbcd"):
                assert ev["gap"].hex() == rv["gap"].hex(), m
            assert ev["test_err_count"] == rv["test_err"] and ev["test_rows"] == 600
    run, revs = _oracle("cocoa+", 8)
    assert out[0]["run"][0].tobytes() == run.w().tobytes()
    assert [t for t, _ in out[0]["run"][1]] == [4, 8]
    assert [ev["gap"].hex() for _, ev in out[0]["run"][1]] == [rv["gap"].hex() for rv in revs]


def _defer_worker(rank, world, strict, methods, uid_q, out_q):
    """Fast CoCoA+ with each evaluation's read-back deferred past the next round
    (cocoa_eval_begin / _end): the rank sums are all-reduced on the device."""
    try:
        tr = cocoa_amd.load_libsvm(TRAIN, 4, 9947)
        te = cocoa_amd.load_libsvm(TEST, 4, 9947)
        k0, k1 = shard_bounds(4, world, rank)
        r0, r1 = shard_bounds(te.n, world, rank)
        if rank == 0:
            uid = comm_unique_id("host")
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        e = Engine(device=0, strict=False)
        e.set_train(tr.shard(k0, k1), part_begin=k0, num_parts_global=4)
        e.set_test(te.row_range(r0, r1))
        e.comm_init("host", rank, world, uid)
        e.init("cocoa+", tr.n, T + 1, H, LAM, 1.0, 1.0, 4, 0)
        evs, pending = [], False
        for t in range(1, T + 2):
            e.round(t)  # (round t+1 is enqueued before round t's evaluation is read back)
            if pending:
                evs.append(e.eval_end())
                pending = False
            if t % 4 == 0 and t <= T:
                e.eval_begin()
                pending = True
        out_q.put((rank, evs))
    except Exception as ex:
        out_q.put((rank, repr(ex)))


def test_multirank_fast_deferred_eval_device_allreduce():
    """cocoa_eval_begin on a fast multi-rank context all-reduces the objective
    sums on the device and cocoa_eval_end reads them back: the oracle's values
    within 1e-9, the same bytes on every rank, the global test-row count."""
    world = 2
    out = _spawn(world, False, None, target=_defer_worker)
    _, revs = _oracle("cocoa+")
    assert len(out[0]) == len(revs) == T // 4
    for a, b, rv in zip(out[0], out[1], revs):
        assert a["gap"].hex() == b["gap"].hex() and a["primal"].hex() == b["primal"].hex()
        assert abs(a["primal"] - rv["primal"]) <= 1e-9 * abs(rv["primal"])
        assert abs(a["gap"] - rv["gap"]) <= 1e-9 * abs(rv["primal"])
        assert a["test_err_count"] == rv["test_err"] and a["test_rows"] == 600


def test_multirank_fast_allreduce_within_tolerance():
    world = 2
    out = _spawn(world, False, ["cocoa+", "mbcd", "mbsgd"])
    for m in ("cocoa+", "mbcd", "mbsgd"):
        run, revs = _oracle(m)
        w_ref = run.w()
        assert out[0][m][0].tobytes() == out[1][m][0].tobytes()                # allreduce: same bytes
        assert np.max(np.abs(out[0][m][0] - w_ref)) <= 1e-9 * np.max(np.abs(w_ref))
        for ev, rv in zip(out[0][m][2], revs):
            assert abs(ev["primal"] - rv["primal"]) <= 1e-9 * abs(rv["primal"])
            assert ev["test_err_count"] == rv["test_err"]


# ---- dense rows (dense solver) and compact deltaW slices across ranks ----
def _cfg_worker(rank, world, strict, cfg, uid_q, out_q):
    try:
        from cocoa_amd import configs
        if cfg.get("compact"):
            os.environ["COCOA_DW_COMPACT"] = "1"
        sh = configs.share(cfg["config"], rank=rank, world=world, scaling="strong", n=cfg["n"], d=cfg.get("d"),
                           parts=cfg["parts"], n_test=cfg["n_test"])
        if rank == 0:
            uid = comm_unique_id("host")
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        e = Engine(device=0, strict=strict)
        e.set_train(sh.train, part_begin=sh.part_begin, num_parts_global=sh.k_glob)
        e.set_test(sh.test)
        e.set_solver(cfg.get("solver", "auto"))
        e.comm_init("host", rank, world, uid)
        e.init("cocoa+", sh.n_glob, 4, sh.H, sh.lam)
        plan = e.plan()
        for t in range(1, 5):
            e.round(t)
        out_q.put((rank, (e.w(), e.alpha(), e.eval(), plan)))
        e.close()
    except Exception as ex:
        out_q.put((rank, repr(ex)))


@pytest.mark.parametrize("cfg,strict", [
    (dict(config="c3", n=4096, parts=8, n_test=256), False),
    (dict(config="c4", n=16000, d=200000, parts=8, n_test=400, compact=True), False),
    (dict(config="c4", n=16000, d=200000, parts=8, n_test=400, compact=True), True),
    # fast CoCoA+ on the chain solver: private columns (test_gpu_private.py) on each rank
    (dict(config="c4", n=16000, d=200000, parts=8, n_test=400, compact=True, solver="chain"), False),
])
def test_multirank_dense_and_compact_layouts(cfg, strict):
    from cocoa_amd import configs
    world = 2
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_cfg_worker, args=(r, world, strict, cfg, uid_q, out_q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(out_q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    want = "dense" if cfg["config"] == "c3" and not strict else ("gram" if not strict else "chain")
    assert out[0][3]["solver"] == cfg.get("solver", want)
    if cfg.get("compact"):
        assert out[0][3]["dw_compact"] == 1
    if cfg.get("solver") == "chain" and not strict:
        assert out[0][3]["dw_private"] == 1 and out[1][3]["dw_private"] == 1
    sh = configs.share(cfg["config"], n=cfg["n"], d=cfg.get("d"), parts=cfg["parts"], n_test=cfg["n_test"],
                       scaling="strong")
    od = oracle.Data(sh.train.row_ptr, sh.train.col, sh.train.val, sh.train.y, sh.train.part_ptr,
                     sh.train.num_features)
    ot = oracle.Data(sh.test.row_ptr, sh.test.col, sh.test.val, sh.test.y, sh.test.part_ptr, sh.test.num_features)
    run = oracle.Run(od, "cocoa+", sh.n_glob, sh.H, sh.lam, nthreads=16)
    for t in range(1, 5):
        run.round(t)
    rv = run.eval(ot)
    w_ref = run.w()
    a = np.concatenate([out[r][1] for r in range(world)])
    ev = out[0][2]
    assert out[0][0].tobytes() == out[1][0].tobytes()  # w identical on every rank
    if strict:
        assert out[0][0].tobytes() == w_ref.tobytes()
        assert a.tobytes() == run.alpha().tobytes()
        assert ev["gap"].hex() == rv["gap"].hex()
    else:
        assert np.max(np.abs(out[0][0] - w_ref)) <= 1e-9 * np.max(np.abs(w_ref))
        assert np.max(np.abs(a - run.alpha())) <= 1e-9
        assert abs(ev["gap"] - rv["gap"]) <= 1e-9 * abs(rv["primal"])
    assert ev["test_err_count"] == rv["test_err"]
