"""Multi-GPU launcher: one process (and one engine) per GPU.

The exchange itself lives in libcocoa_hip.so (cocoa_comm_init, RCCL over
xGMI): each rank owns a contiguous block of the K partitions (CoCoA.scala:28)
and every cocoa_round / cocoa_eval sums deltaW and the objective terms across
ranks inside the library (CoCoA.scala:45-48, OptUtils.scala:65-98).  This
module only hands rank 0's communicator id to the other ranks through
torch.distributed (any process group: gloo is enough, no data goes through
it) and forwards the calls.
"""
import os

from .configs import shard_bounds  # noqa: F401  (re-exported)
from .engine import comm_unique_id


def env_rank():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


class DistributedCoCoA:
    """Attach the engine to the ranks of the torch.distributed group (or run
    single-rank when none is initialised) and drive its rounds."""

    def __init__(self, engine, transport="rccl", group=None):
        import torch.distributed as dist
        self.engine = engine
        if dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1
        if self.world > 1:
            obj = [comm_unique_id(transport) if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            engine.comm_init(transport, self.rank, self.world, obj[0])

    def round(self, t):
        self.engine.round(t)

    def eval(self):
        return self.engine.eval()

    def eval_begin(self):
        self.engine.eval_begin()

    def eval_end(self):
        return self.engine.eval_end()
