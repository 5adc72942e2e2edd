"""The library's rank exchange (cocoa_comm_*, HOST transport) in real
multi-process runs on the CPU: the two reductions cocoa_round / cocoa_eval use
between ranks (CoCoA.scala:47 reduce(_ + _), OptUtils.scala:65-98), checked
bit for bit against the single-process sums they stand for."""
import multiprocessing as mp

import numpy as np
import pytest

from cocoa_amd import _capi
from cocoa_amd.engine import Comm, comm_unique_id

SIZES = [0, 1, 3, 4096, 1 << 20]


def _worker(rank, world, uid_q, out_q):
    try:
        if rank == 0:
            uid = comm_unique_id("host")
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        c = Comm("host", rank, world, uid)
        res = []
        for n in SIZES:
            x = np.random.default_rng(1000 * rank + n).standard_normal(n) * 10.0 ** (rank - 1)
            res.append((c.allreduce(x), c.ordered_sum(x)))
        c.close()
        out_q.put((rank, res))
    except Exception as e:  # report instead of hanging the parent
        out_q.put((rank, repr(e)))


def _run(world):
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, uid_q, out_q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(out_q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world", [2, 3, 4])
def test_host_transport_sums_are_rank_ordered_and_identical(world):
    out = _run(world)
    for r in range(world):
        assert not isinstance(out[r], str), out[r]
    for i, n in enumerate(SIZES):
        xs = [np.random.default_rng(1000 * r + n).standard_normal(n) * 10.0 ** (r - 1) for r in range(world)]
        ref = xs[0].copy()
        for x in xs[1:]:
            ref = ref + x                        # ((x_0 + x_1) + x_2) + ...
        for r in range(world):
            ar, osum = out[r][i]
            assert ar.tobytes() == ref.tobytes()  # every rank gets identical bytes
            assert osum.tobytes() == ref.tobytes()


def test_comm_argument_errors():
    uid = comm_unique_id("host")
    with pytest.raises(_capi.IllegalArgumentError):
        Comm("host", 2, 2, uid)                   # rank outside [0, world)
    with pytest.raises(_capi.IllegalArgumentError):
        Comm("host", 0, 1, b"\0" * 128)           # not a HOST uid
    c = Comm("host", 0, 1, uid)                   # world 1: sums are the identity
    x = np.arange(5.0)
    assert np.array_equal(c.allreduce(x), x) and np.array_equal(c.ordered_sum(x), x)
