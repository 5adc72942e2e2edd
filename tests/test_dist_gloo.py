"""N>1 path on CPU: two ranks (a gloo group for the launcher's id exchange)
run the multi-rank round structure -- contiguous partition shards, ordered
local fold, the library's rank exchange (cocoa_comm_allreduce, HOST
transport) of the deltaW sum, identical w update on every rank, exchange of
the objective sums.  The per-rank compute is the oracle here (this test has
no GPU); the result must equal a single-process oracle run up to the
re-association of the cross-rank sum."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cocoa_amd.data import load_libsvm
from cocoa_amd.dist import shard_bounds
from cocoa_amd.engine import Comm, comm_unique_id
from oracle import oracle

G = os.path.join(os.path.dirname(__file__), "golden", "data")


class OracleEngine:
    """One rank of the multi-rank round (cocoa_round with a communicator), with
    the oracle doing the rank-local compute and the library's HOST-transport
    communicator doing the exchange."""

    def __init__(self, shard, test_shard, method, n, H, lam, Kg):
        self.data = oracle.Data(shard.row_ptr, shard.col, shard.val, shard.y, shard.part_ptr, shard.num_features)
        self.test = oracle.Data(test_shard.row_ptr, test_shard.col, test_shard.val, test_shard.y,
                                test_shard.part_ptr, test_shard.num_features)
        self.run = oracle.Run(self.data, method, n, H, lam)
        self.run.set_global_parts(Kg)
        self.n, self.lam = n, lam
        self.comm = None

    def round(self, t):
        buf = np.zeros(self.data.d)
        self.run.round_local(t, buf)
        self.run.round_apply(self.comm.allreduce(buf))

    def eval(self):
        ev = self.run.eval(self.test)
        w = self.run.w()
        w2 = 0.0
        for x in w:
            w2 += x * x
        h, a, e, r = self.comm.allreduce([ev["hinge_sum"], ev["alpha_sum"], ev["test_err"], self.test.n])
        return self.eval_finish(h, a, w2, e, r)

    def eval_finish(self, h, a, w2, e, r):
        nw = np.sqrt(w2)
        P = h / self.n + (0.5 * self.lam * (nw * nw))
        D = (-self.lam / 2 * (nw * nw)) + (a / self.n)
        return {"primal": P, "dual": D, "gap": P - D, "test_error": e / r}


def _worker(rank, world, port, method, T, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = load_libsvm(os.path.join(G, "small_train.dat"), 4, 9947)
    te = load_libsvm(os.path.join(G, "small_test.dat"), 4, 9947)
    k0, k1 = shard_bounds(4, world, rank)
    r0, r1 = shard_bounds(te.n, world, rank)
    eng = OracleEngine(tr.shard(k0, k1), te.row_range(r0, r1), method, tr.n, 50, 1e-3, 4)
    obj = [comm_unique_id("host") if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)   # the launcher's job (cocoa_amd.dist)
    eng.comm = Comm("host", rank, world, obj[0])
    evs = []
    for t in range(1, T + 1):
        eng.round(t)
        if t % 5 == 0:
            evs.append(eng.eval())
    q.put((rank, eng.run.w(), eng.run.alpha(), evs))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("method", ["cocoa+", "cocoa", "mbcd", "mbsgd"])
def test_two_gloo_ranks_match_single_process(method):
    T, world = 15, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, method, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (w, a, e)) for r, w, a, e in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: one process, all 4 partitions
    tr = oracle.Data.load_libsvm(os.path.join(G, "small_train.dat"), 4, 9947)
    te = oracle.Data.load_libsvm(os.path.join(G, "small_test.dat"), 4, 9947)
    run = oracle.Run(tr, method, tr.n, 50, 1e-3)
    ref_ev = []
    for t in range(1, T + 1):
        run.round(t)
        if t % 5 == 0:
            ref_ev.append(run.eval(te))
    w_ref = run.w()
    w0, w1 = res[0][0], res[1][0]
    assert np.array_equal(w0, w1)                       # replicated w stays identical
    assert np.max(np.abs(w0 - w_ref)) <= 1e-12 * np.max(np.abs(w_ref))
    if method in ("cocoa+", "cocoa", "mbcd"):
        a = np.concatenate([res[0][1], res[1][1]])
        assert np.max(np.abs(a - run.alpha())) <= 1e-12
    for e, r in zip(res[0][2], ref_ev):
        assert abs(e["primal"] - r["primal"]) <= 1e-12 * abs(r["primal"])
        assert abs(e["gap"] - r["gap"]) <= 1e-12 * abs(r["primal"])
        assert round(e["test_error"] * 600) == r["test_err"]
