"""Abort reporting and mixed solvers across ranks.

* A Gram-solver launch that aborts (a wave hand-off timed out: the status word
  is set) must make the evaluation that covers it raise, in the deferred
  (cocoa_eval_begin / _end) and pipelined (cocoa_eval_async / _wait) flows,
  without any stream sync of its own.  COCOA_INJECT_ABORT=t marks round t's
  launch as aborted (fault injection; read once per process).
* Fast multi-rank rounds exchange d + 1 values (the abort slot) whichever
  solver a rank's shard took: a rank on the chain solver beside a rank on the
  Gram solver must neither hang nor mis-sum, and must see the other rank's
  abort.
"""
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
H, LAM, T = 50, 1e-3, 8


def _abort_worker(flow, out_q):
    try:
        os.environ["COCOA_INJECT_ABORT"] = "3"
        tr, te = cocoa_amd.load_libsvm(TRAIN, 4, 9947), cocoa_amd.load_libsvm(TEST, 4, 9947)
        e = Engine(device=0, strict=False)
        e.set_train(tr)
        e.set_test(te)
        e.set_solver("gram")
        e.init("cocoa+", tr.n, T, H, LAM)
        assert e.plan()["solver"] == "gram"
        got, raised_at = [], None
        pending = None
        for t in range(1, T + 1):
            e.round(t)
            try:
                if pending is not None:
                    got.append(e.eval_wait() if flow == "pipelined" else e.eval_end())
                    pending = None
                if flow == "pipelined":
                    e.eval_async()
                else:
                    e.eval_begin()
                pending = t
            except cocoa_amd.CocoaError as ex:
                raised_at = (pending, str(ex))
                break
        out_q.put(("ok", len(got), raised_at))
    except Exception as ex:  # noqa: BLE001
        out_q.put(("error", repr(ex), None))


@pytest.mark.timeout(180)
@pytest.mark.parametrize("flow", ["deferred", "pipelined"])
def test_aborted_gram_launch_raises_at_collection(flow):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_abort_worker, args=(flow, q))
    p.start()
    try:
        kind, n_ok, raised = q.get(timeout=150)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert kind == "ok", n_ok
    # rounds 1 and 2 evaluate normally; the evaluation behind round 3 (the
    # aborted launch) raises when it is collected
    assert n_ok == 2 and raised is not None and raised[0] == 3, (n_ok, raised)
    assert "timed out" in raised[1]


def _mixed_worker(rank, world, inject, uid_q, out_q):
    try:
        if inject and rank == 1:
            os.environ["COCOA_INJECT_ABORT"] = "2"
        tr, te = cocoa_amd.load_libsvm(TRAIN, 4, 9947), cocoa_amd.load_libsvm(TEST, 4, 9947)
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
        e.set_solver("chain" if rank == 0 else "gram")  # rank 0 without the Gram solver's status word
        e.comm_init("host", rank, world, uid)
        e.init("cocoa+", tr.n, T, H, LAM)
        solver = e.plan()["solver"]
        evs = []
        try:
            for t in range(1, T + 1):
                e.round(t)
                if t % 4 == 0:
                    evs.append(e.eval())
        except cocoa_amd.CocoaError as ex:
            out_q.put((rank, ("raised", str(ex), solver)))
            return
        out_q.put((rank, (e.w(), evs, solver)))
    except Exception as ex:  # noqa: BLE001
        out_q.put((rank, repr(ex)))


def _spawn_mixed(inject):
    world = 2
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_mixed_worker, args=(r, world, inject, uid_q, out_q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = dict(out_q.get(timeout=150) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    return out


@pytest.mark.timeout(200)
def test_mixed_solvers_across_ranks_exchange_and_match_oracle():
    out = _spawn_mixed(False)
    assert out[0][2] == "chain" and out[1][2] == "gram"
    od, ot = oracle.Data.load_libsvm(TRAIN, 4, 9947), oracle.Data.load_libsvm(TEST, 4, 9947)
    run = oracle.Run(od, "cocoa+", od.n, H, LAM)
    revs = []
    for t in range(1, T + 1):
        run.round(t)
        if t % 4 == 0:
            revs.append(run.eval(ot))
    w_ref = run.w()
    assert out[0][0].tobytes() == out[1][0].tobytes()
    assert np.max(np.abs(out[0][0] - w_ref)) <= 1e-9 * np.max(np.abs(w_ref))
    for ev, rv in zip(out[0][1], revs):
        assert abs(ev["gap"] - rv["gap"]) <= 1e-9 * abs(rv["primal"])
        assert ev["test_err_count"] == rv["test_err"]


@pytest.mark.timeout(200)
def test_abort_on_one_rank_is_seen_by_a_chain_rank():
    out = _spawn_mixed(True)
    for r in range(2):
        assert out[r][0] == "raised" and "timed out" in out[r][1], (r, out[r])
