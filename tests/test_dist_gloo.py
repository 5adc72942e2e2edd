"""N>1 path on CPU: two gloo ranks run cocoa_amd.dist.DistributedCoCoA (the
product's multi-GPU orchestration: contiguous partition shards, ordered local
fold, all-reduce of the deltaW sum, identical w update on every rank, scalar
all-reduce for the objectives).  The per-rank compute is the oracle here (this
test has no GPU); the result must equal a single-process oracle run up to the
re-association of the cross-rank sum."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cocoa_amd.data import load_libsvm
from cocoa_amd.dist import DistributedCoCoA, shard_bounds
from oracle import oracle

G = os.path.join(os.path.dirname(__file__), "golden", "data")


class OracleEngine:
    """Implements the engine interface DistributedCoCoA drives, on the oracle."""

    def __init__(self, shard, test_shard, method, n, H, lam, Kg):
        self.data = oracle.Data(shard.row_ptr, shard.col, shard.val, shard.y, shard.part_ptr, shard.num_features)
        self.test = oracle.Data(test_shard.row_ptr, test_shard.col, test_shard.val, test_shard.y,
                                test_shard.part_ptr, test_shard.num_features)
        self.run = oracle.Run(self.data, method, n, H, lam)
        self.run.set_global_parts(Kg)
        self.n, self.lam = n, lam
        self.dw_sum = torch.zeros(shard.num_features, dtype=torch.float64)

    def round_local(self, t):
        buf = np.zeros(self.data.d)
        self.run.round_local(t, buf)
        self.dw_sum.copy_(torch.from_numpy(buf))

    def round_apply(self):
        self.run.round_apply(self.dw_sum.numpy())

    def eval(self):
        ev = self.run.eval(self.test)
        w = self.run.w()
        w2 = 0.0
        for x in w:
            w2 += x * x
        return {"hinge_sum": ev["hinge_sum"], "alpha_sum": ev["alpha_sum"], "w_sqnorm": w2,
                "test_err_count": ev["test_err"], "test_rows": self.test.n}

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
    runner = DistributedCoCoA(eng)
    evs = []
    for t in range(1, T + 1):
        runner.round(t)
        if t % 5 == 0:
            evs.append(runner.eval())
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
