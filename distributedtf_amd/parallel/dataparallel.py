"""Intra-member data parallelism: one population member trained by a group of ranks.

Reference: ``resnet/official/utils/misc/distribution_utils.py:24-78`` (TF ``MirroredStrategy`` with an in-graph
all-reduce), which the reference's main path hard-wires off (``resnet_run_loop.py:390-392``; SURVEY.md §2.5
C19).  Here it is the optional extension for ``population < #GPUs``: ``--dp_size k`` splits the world into
``world / k`` member groups of ``k`` consecutive ranks.  Every rank of a group holds a replica of the group's
members (same ids, same initialisation, same exploit/explore decisions) and trains on its own shard of each
batch; before every optimizer step the gradient rows of the members are all-reduced over the group -- RCCL over
xGMI on GPUs, gloo on CPU -- so the replicas stay bit-identical.  Each replica's gradient is the mean over its own
shard, so it is weighted by ``local batch / member batch`` before the sum: an uneven split (a member batch of 129
over 2 replicas = 65 + 64 images) then yields exactly the gradient of the mean loss over the whole member batch
(equal weights would over-count the larger shard).  The weighting and the all-reduce are device ops on the step's
stream, so the HIP backends capture them in the step graph with the rest of the step.  BatchNorm normalises with
the replica's own batch statistics (as MirroredStrategy's per-replica BN did); the running statistics are averaged
over the group at the end of every round.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional


@dataclass
class DPContext:
    group: object          # torch.distributed process group of this rank's member group
    size: int              # ranks per member group
    rank: int              # this rank's index inside the group
    group_index: int       # which member group this rank belongs to
    n_groups: int

    def local_batch(self, batch_size: int) -> int:
        """This replica's share of a member's batch (the remainder goes to the first replicas)."""
        b = int(batch_size)
        return b // self.size + (1 if self.rank < b % self.size else 0)

    def allreduce_mean_(self, t) -> None:
        import torch.distributed as dist
        dist.all_reduce(t, group=self.group)
        t.div_(self.size)

    def allreduce_weighted_(self, t, w) -> None:
        """``t[i] <- sum over replicas of w_r[i] * t_r[i]`` (rows ``t[i]``, per-row replica weights ``w[i]``)."""
        import torch.distributed as dist
        t.mul_(w.reshape(-1, *([1] * (t.dim() - 1))))
        dist.all_reduce(t, group=self.group)


def make_dp_context(comm, dp_size: int) -> Optional[DPContext]:
    """Create every member group's process group (a collective over the whole world) and return this rank's
    context; ``None`` for ``dp_size <= 1``."""
    if dp_size <= 1:
        return None
    import torch.distributed as dist
    world, rank = comm.Get_size(), comm.Get_rank()
    if world % dp_size:
        raise ValueError("--dp_size %d must divide the world size %d" % (dp_size, world))
    n_groups = world // dp_size
    mine = None
    for g in range(n_groups):
        ranks: List[int] = list(range(g * dp_size, (g + 1) * dp_size))
        pg = dist.new_group(ranks)
        if rank in ranks:
            mine = pg
    return DPContext(group=mine, size=dp_size, rank=rank % dp_size, group_index=rank // dp_size, n_groups=n_groups)
