"""Exploit data plane: move a member's whole training state winner -> loser.

Replaces the reference's ``cp`` of TF checkpoint files on a shared filesystem
(``pbt_cluster.py:145-147,168-181``).

Each member exposes its state as ONE contiguous tensor (``export_state()``; the
population engine keeps it as a row of a ``[G, S]`` buffer, so nothing is packed
per exploit).  A transfer ``(src_id, src_rank, dst_id, dst_rank)`` is:

* same rank   -> on-device copy (``hipMemcpyAsync`` D2D via ``Tensor.copy_``);
* cross rank  -> ``torch.distributed`` P2P ``isend``/``irecv`` -- RCCL
  ``ncclSend``/``ncclRecv`` over the direct xGMI link between the two GPUs.
  All P2P ops of one exploit are issued as ONE ``batch_isend_irecv`` group, so
  disjoint pairs run concurrently on disjoint links and no ordering deadlock is
  possible.  The receive lands directly in the loser's state row (zero-copy).

On CPU worlds (tests) the same code runs over gloo.

The receiving member's host-side step counter (it drives the LR schedule of the
next step) is never read back from the imported device row: the caller passes
the winners' host steps (``steps``: all-gathered with the scores), or, when it
has none (master/worker mode), each source rank posts its member's step to the
destination rank on the control plane (a host message, no device sync).
"""

from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence, Tuple

Transfer = Tuple[int, int, int, int]  # (src_id, src_rank, dst_id, dst_rank)


class DataPlane:
    def __init__(self, comm, group=None):
        self.comm = comm
        self.rank = comm.Get_rank()
        self.group = group
        self.bytes_moved = 0
        self.seconds = 0.0
        self.transfers_done = 0
        self.step_timeout = 600.0

    @staticmethod
    def _state_of(member):
        view = getattr(member, "state_view", None)
        return view() if view is not None else member.export_state()

    def execute(self, transfers: Sequence[Transfer], local_members: Dict[int, object],
                steps: Optional[Dict[int, int]] = None) -> None:
        """Run one exploit's copies.  ``steps``: member id -> host step counter of every SOURCE (None: exchanged
        over the control plane for cross-rank pairs)."""
        import torch
        t0 = time.time()
        ops = []
        pending: List[Tuple[object, "torch.Tensor", bool]] = []
        # Snapshot every local source first: sources and destinations are disjoint
        # quantiles, but a local copy must never observe a half-written winner.
        for (src_id, src_rank, dst_id, dst_rank) in transfers:
            if src_rank == self.rank and dst_rank == self.rank:
                src = self._state_of(local_members[src_id])
                dst_m = local_members[dst_id]
                dst = self._state_of(dst_m)
                if dst.data_ptr() != src.data_ptr():
                    if hasattr(dst_m, "state_view"):
                        dst.copy_(src)
                        hook = getattr(dst_m, "on_state_imported", None)
                        if hook is not None:
                            # the winner's step counter is known on the host: no device round trip
                            hook(int(local_members[src_id].global_step))
                    else:
                        dst_m.import_state(src.clone())
                self.bytes_moved += src.numel() * src.element_size()
            elif src_rank == self.rank:
                src = self._state_of(local_members[src_id])
                if not src.is_contiguous():
                    src = src.contiguous()
                ops.append(("send", src, dst_rank))
                self.bytes_moved += src.numel() * src.element_size()
                if steps is None:
                    # always posted for a cross-rank pair (and always consumed below), whatever the two members'
                    # types: a condition only one side can evaluate would leave a message unread or a recv hanging
                    self.comm.send(("dtf_step", src_id, int(getattr(local_members[src_id], "global_step", 0) or 0)),
                                   dst_rank)
            elif dst_rank == self.rank:
                dst_m = local_members[dst_id]
                inplace = hasattr(dst_m, "state_view")
                buf = self._state_of(dst_m) if inplace else torch.empty_like(dst_m.export_state())
                ops.append(("recv", buf, src_rank))
                pending.append((dst_m, buf, inplace, src_id, src_rank))
        if ops:
            if hasattr(self.comm, "tensor_send"):
                # in-process worlds (LocalComm): sends are buffered, so issue them first
                for kind, t, peer in ops:
                    if kind == "send":
                        self.comm.tensor_send(t, peer)
                for kind, t, peer in ops:
                    if kind == "recv":
                        self.comm.tensor_recv(t, peer)
            else:
                dist = torch.distributed
                p2p = [dist.P2POp(dist.isend if k == "send" else dist.irecv, t, peer, group=self.group)
                       for k, t, peer in ops]
                for r in dist.batch_isend_irecv(p2p):
                    r.wait()
        for dst_m, buf, inplace, src_id, src_rank in pending:
            if steps is not None:
                step = int(steps.get(src_id, 0))
            else:
                tag, sid, step = self.comm.recv(src_rank, timeout=self.step_timeout)
                assert tag == "dtf_step" and sid == src_id, ("exploit step message out of order", tag, sid, src_id)
            if not inplace:
                dst_m.import_state(buf)
                continue
            hook = getattr(dst_m, "on_state_imported", None)
            if hook is not None:
                hook(int(step))
        self.transfers_done += len(transfers)
        self.seconds += time.time() - t0


def plan_transfers(plan, owner_rank: Dict[int, int]) -> List[Transfer]:
    """Attach owning ranks to an exploit plan (``ExploitPair`` list)."""
    return [(p.src_id, owner_rank[p.src_id], p.dst_id, owner_rank[p.dst_id]) for p in plan]
