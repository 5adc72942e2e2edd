"""Multi-GPU CoCoA: one process (and one engine) per GPU, torch.distributed
for the exchange (backend "nccl" = RCCL over xGMI on ROCm).

Each rank owns a contiguous block of the K partitions (CoCoA.scala:28: the
partitions are the unit of parallelism).  Per round t (CoCoA.scala:39-63):

    engine.round_local(t)      sampling + K_loc local solvers + ordered local
                               fold of deltaW into the rank's dw_sum buffer
    all_reduce(dw_sum, SUM)    the only data-path collective (8*d bytes)
    engine.round_apply()       w += sum * scaling  (identical on every rank:
                               the ring all-reduce delivers identical bytes)

Evaluation all-reduces four scalars (hinge sum, alpha sum, test errors, test
rows).  The fold order differs from the single-process left fold by the
grouping of partitions into ranks (Spark's own merge order is the task
completion order, so the reference is not bit-reproducible here either);
results agree within the north_star tolerance (1e-9 relative).

The engine is any object with round_local/round_apply/eval/eval_finish and a
`dw_sum` torch tensor; the GPU engine is `TorchEngine`.
"""
import os

import numpy as np

from .engine import Engine


def shard_bounds(K, world, rank):
    """Contiguous partition block [k0, k1) of rank `rank`."""
    return (K * rank) // world, (K * (rank + 1)) // world


class TorchEngine(Engine):
    """Engine on torch's current HIP stream whose deltaW sum is a torch tensor
    (so torch.distributed / RCCL can all-reduce it in place)."""

    def __init__(self, device=0, strict=False):
        import torch
        torch.cuda.set_device(device)
        self.torch = torch
        # a dedicated stream, made torch's current one, so the engine's kernels
        # and torch.distributed's collectives are ordered on the same queue
        self.stream = torch.cuda.Stream(device=device)
        torch.cuda.set_stream(self.stream)
        super().__init__(device=device, strict=strict, stream=self.stream.cuda_stream)
        self.dw_sum = None

    def init(self, *args, **kw):
        super().init(*args, **kw)
        self.dw_sum = self.torch.zeros(self.d, dtype=self.torch.float64, device="cuda")
        self.set_dw_sum_buffer(self.dw_sum.data_ptr())


class DistributedCoCoA:
    def __init__(self, engine, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.engine = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def round(self, t):
        eng = self.engine
        eng.round_local(t)
        if self.world > 1:
            self.dist.all_reduce(eng.dw_sum, op=self.dist.ReduceOp.SUM, group=self.group)
        eng.round_apply()

    def eval(self):
        ev = self.engine.eval()
        if self.world == 1:
            return ev
        t = self.torch.tensor([ev["hinge_sum"], ev["alpha_sum"], float(ev["test_err_count"]),
                               float(ev["test_rows"])], dtype=self.torch.float64,
                              device=self.engine.dw_sum.device)
        self.dist.all_reduce(t, group=self.group)
        h, a, e, r = t.tolist()
        return self.engine.eval_finish(h, a, ev["w_sqnorm"], int(e), int(r))


def env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))
