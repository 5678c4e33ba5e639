"""Control-plane communicators.

The reference moves pickled Python objects point-to-point with mpi4py
(``pbt_cluster.py`` / ``training_worker.py``, every call site in SURVEY.md §2.4).
Here the control plane is split from the data plane:

* ``Comm`` -- an MPI-``COMM_WORLD``-like object API (``Get_rank``, ``Get_size``,
  ``send``/``isend``/``recv`` of picklable objects, plus the collectives the SPMD
  engine needs: ``allgather``, ``bcast``, ``barrier``).
* ``LocalComm`` -- in-process implementation (threads + queues) used by unit tests
  as the fake / loopback backend the reference never had.
* ``TorchComm`` -- multi-process implementation. Point-to-point object messages go
  through a ``TCPStore`` mailbox (non-blocking sends, per-pair FIFO like MPI's
  non-overtaking rule, bounded waits instead of the reference's unbounded
  ``recv``); collectives go through a ``gloo`` CPU group.  Bulk tensors (exploit
  weight copies) never use this path: see ``parallel/dataplane.py`` (RCCL).
"""

from __future__ import annotations

import datetime
import os
import pickle
import queue
import threading
from typing import Any, List, Optional


class Request:
    """Completed-on-creation request (sends are buffered)."""

    def wait(self):
        return None

    def test(self):
        return True


class Comm:
    def Get_rank(self) -> int:
        raise NotImplementedError

    def Get_size(self) -> int:
        raise NotImplementedError

    # point to point -------------------------------------------------------
    def send(self, obj: Any, dest: int) -> None:
        raise NotImplementedError

    def isend(self, obj: Any, dest: int) -> Request:
        self.send(obj, dest)
        return Request()

    def recv(self, source: int, timeout: Optional[float] = None) -> Any:
        raise NotImplementedError

    # collectives ------------------------------------------------------------
    def allgather(self, obj: Any) -> List[Any]:
        raise NotImplementedError

    def bcast(self, obj: Any, root: int = 0) -> Any:
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    # convenience ----------------------------------------------------------
    @property
    def rank(self) -> int:
        return self.Get_rank()

    @property
    def size(self) -> int:
        return self.Get_size()


# ---------------------------------------------------------------- local (threads)

class _LocalWorld:
    def __init__(self, size: int):
        self.size = size
        self.boxes = {(s, d): queue.Queue() for s in range(size) for d in range(size)}
        self.tensor_boxes = {(s, d): queue.Queue() for s in range(size) for d in range(size)}
        self.barrier = threading.Barrier(size)
        self.lock = threading.Lock()
        self.slots: List[Any] = [None] * size


class LocalComm(Comm):
    """A communicator for ``size`` threads in one process."""

    def __init__(self, world: _LocalWorld, rank: int, default_timeout: float = 120.0):
        self._world = world
        self._rank = rank
        self.default_timeout = default_timeout

    @staticmethod
    def create(size: int) -> List["LocalComm"]:
        world = _LocalWorld(size)
        return [LocalComm(world, r) for r in range(size)]

    def Get_rank(self):
        return self._rank

    def Get_size(self):
        return self._world.size

    def send(self, obj, dest):
        # pickle round-trip gives MPI's by-value semantics
        self._world.boxes[(self._rank, dest)].put(pickle.dumps(obj))

    def recv(self, source, timeout=None):
        t = self.default_timeout if timeout is None else timeout
        try:
            data = self._world.boxes[(source, self._rank)].get(timeout=t)
        except queue.Empty:
            raise TimeoutError(f"rank {self._rank}: no message from {source} within {t}s")
        return pickle.loads(data)

    # tensor channel used by DataPlane when there is no torch.distributed group
    def tensor_send(self, t, dest):
        self._world.tensor_boxes[(self._rank, dest)].put(t.detach().cpu().clone())

    def tensor_recv(self, out, source, timeout=None):
        t = self.default_timeout if timeout is None else timeout
        try:
            data = self._world.tensor_boxes[(source, self._rank)].get(timeout=t)
        except queue.Empty:
            raise TimeoutError(f"rank {self._rank}: no tensor from {source} within {t}s")
        out.copy_(data.to(out.device))

    def allgather(self, obj):
        w = self._world
        w.barrier.wait()
        w.slots[self._rank] = pickle.dumps(obj)
        w.barrier.wait()
        out = [pickle.loads(s) for s in w.slots]
        w.barrier.wait()
        return out

    def bcast(self, obj, root=0):
        return self.allgather(obj if self._rank == root else None)[root]

    def barrier(self):
        self._world.barrier.wait()


# ------------------------------------------------------------ torch.distributed

class TorchComm(Comm):
    """Multi-process communicator over ``torch.distributed``.

    Call :func:`init_distributed` first (it creates the default process group,
    RCCL on GPU / gloo on CPU, and a gloo group for objects).
    """

    def __init__(self, store, cpu_group, rank: int, size: int, default_timeout: float = 1800.0):
        self._store = store
        self._group = cpu_group
        self._rank = rank
        self._size = size
        self._send_seq = {}
        self._recv_seq = {}
        self.default_timeout = default_timeout

    def Get_rank(self):
        return self._rank

    def Get_size(self):
        return self._size

    def _key(self, src, dst, seq):
        return f"dtf/mb/{src}->{dst}/{seq}"

    def send(self, obj, dest):
        seq = self._send_seq.get(dest, 0)
        self._send_seq[dest] = seq + 1
        self._store.set(self._key(self._rank, dest, seq), pickle.dumps(obj))

    def recv(self, source, timeout=None):
        seq = self._recv_seq.get(source, 0)
        key = self._key(source, self._rank, seq)
        t = self.default_timeout if timeout is None else timeout
        try:
            self._store.wait([key], datetime.timedelta(seconds=t))
        except RuntimeError as e:  # torch raises RuntimeError/DistStoreError on timeout
            raise TimeoutError(f"rank {self._rank}: no message from {source} within {t}s") from e
        data = self._store.get(key)
        self._recv_seq[source] = seq + 1
        try:
            self._store.delete_key(key)
        except Exception:
            pass
        return pickle.loads(data)

    # payload bytes per rank of the one-collective allgather; larger payloads fall back to all_gather_object
    GATHER_SLOT = 8192

    def allgather(self, obj):
        """All-gather of a picklable object in ONE fixed-size byte all_gather on the gloo group (length header
        + pickle per rank).  ``all_gather_object`` needs two collectives (sizes, then data) plus storage
        round trips: at world 8 the exploit metric gather goes 5.4 -> 3.0 ms on an 8-CPU host.  A rank whose
        payload exceeds the slot writes length -1; every rank sees it and all fall back together."""
        import torch
        import torch.distributed as dist
        data = pickle.dumps(obj)
        slot = self.GATHER_SLOT
        buf = torch.zeros(slot + 8, dtype=torch.uint8)
        n = len(data) if len(data) <= slot else -1
        buf[:8] = torch.tensor([n], dtype=torch.int64).view(torch.uint8)
        if n > 0:
            buf[8:8 + n] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        outs = [torch.empty_like(buf) for _ in range(self._size)]
        dist.all_gather(outs, buf, group=self._group)
        lens = [int(o[:8].view(torch.int64)[0]) for o in outs]
        if min(lens) < 0:
            out = [None] * self._size
            dist.all_gather_object(out, obj, group=self._group)
            return out
        return [pickle.loads(o[8:8 + k].numpy().tobytes()) for o, k in zip(outs, lens)]

    def bcast(self, obj, root=0):
        import torch.distributed as dist
        buf = [obj]
        dist.broadcast_object_list(buf, src=root, group=self._group)
        return buf[0]

    def barrier(self):
        import torch.distributed as dist
        dist.barrier(group=self._group)


class SingleComm(Comm):
    """World of one (no process group needed)."""

    def __init__(self):
        self._box = queue.Queue()

    def Get_rank(self):
        return 0

    def Get_size(self):
        return 1

    def send(self, obj, dest):
        assert dest == 0
        self._box.put(pickle.dumps(obj))

    def recv(self, source, timeout=None):
        return pickle.loads(self._box.get(timeout=timeout or 60))

    def allgather(self, obj):
        return [pickle.loads(pickle.dumps(obj))]

    def bcast(self, obj, root=0):
        return obj

    def barrier(self):
        pass


_CTX = {}


def init_distributed(backend: Optional[str] = None, timeout_s: float = 1800.0) -> Comm:
    """Initialise ``torch.distributed`` from torchrun env vars and return a Comm.

    ``backend`` defaults to ``nccl`` (= RCCL on ROCm) when a GPU is visible, else
    ``gloo``.  A world of one returns :class:`SingleComm` without a process group.
    """
    if "comm" in _CTX:
        return _CTX["comm"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        comm = SingleComm()
        _CTX["comm"] = comm
        return comm
    import torch
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    device_index = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "nccl" and os.environ.get("DTF_SHARE_GPU", "0") == "1":
        device_index = configure_shared_gpu(rank, device_index)
    if backend == "nccl":
        torch.cuda.set_device(device_index)
    td = datetime.timedelta(seconds=timeout_s)
    _CTX["preconnected"] = False
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=td)
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", device_index)
        dist.init_process_group(**kw)
        if backend == "nccl":
            # create the RCCL communicator now (all ranks), so later P2P batches that involve only some
            # ranks (exploit copies) never trigger a lazy, partial-world communicator init
            t = torch.ones(1, device="cuda")
            dist.all_reduce(t)
            if os.environ.get("DTF_RCCL_PRECONNECT", "1") == "1":
                preconnect_p2p(world, rank)
                _CTX["preconnected"] = True
            torch.cuda.synchronize()
    cpu_group = dist.new_group(backend="gloo", timeout=td) if backend != "gloo" else dist.group.WORLD
    try:
        from torch.distributed.distributed_c10d import _get_default_store
        store = dist.PrefixStore("dtf_ctrl", _get_default_store())
    except Exception:  # pragma: no cover - older torch
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500")) + 1
        store = dist.TCPStore(host, port, world, is_master=(rank == 0), timeout=td)
    comm = TorchComm(store, cpu_group, rank, world, default_timeout=timeout_s)
    _CTX["comm"] = comm
    _CTX["backend"] = backend
    return comm


def configure_shared_gpu(rank: int, local_rank: int) -> int:
    """``DTF_SHARE_GPU=1``: rehearse a multi-rank RCCL job on fewer GPUs than ranks (the 1-GPU test box).

    RCCL refuses two ranks of one communicator on one device ("Duplicate GPU detected") when they share a host
    hash.  Giving every rank its own ``NCCL_HOSTID`` makes each rank a one-GPU "node": the communicator then forms,
    and ranks exchange data through RCCL's network (socket, loopback) transport instead of xGMI P2P.  Every RCCL
    call of the product -- the exploit ``send``/``recv`` of state rows, the data-parallel all-reduce captured in the
    step graph, the pre-connect -- then really executes RCCL kernels and proxy progress on the GPU, only over a
    slower wire.  Must run before the communicator is created.  Returns the device index (local rank modulo the
    visible devices)."""
    import torch
    os.environ["NCCL_HOSTID"] = "dtf-shared-gpu-rank%d" % rank
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    n = max(1, torch.cuda.device_count())
    return local_rank % n


def preconnected() -> bool:
    """True when init_distributed opened every RCCL P2P pair (exploit copies then pay no lazy connection setup)."""
    return bool(_CTX.get("preconnected", False))


def preconnect_p2p(world: int, rank: int) -> None:
    """Open the RCCL point-to-point connection of EVERY ordered rank pair now, in one ``batch_isend_irecv`` group
    (each rank sends one element to and receives one from every peer).  RCCL sets P2P channels up lazily on a
    pair's first send/recv; exploit winner/loser pairs change every cycle, so without this a pair's first copy
    would pay the connection setup inside a (timed) training round."""
    import torch
    import torch.distributed as dist
    if world <= 1:
        return
    dev = torch.device("cuda", torch.cuda.current_device())
    out = [torch.full((1,), float(rank), device=dev) for _ in range(world)]
    inp = [torch.empty(1, device=dev) for _ in range(world)]
    ops = []
    for peer in range(world):
        if peer == rank:
            continue
        ops.append(dist.P2POp(dist.isend, out[peer], peer))
        ops.append(dist.P2POp(dist.irecv, inp[peer], peer))
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    got = torch.stack([inp[p] for p in range(world) if p != rank]).cpu().tolist()
    want = [[float(p)] for p in range(world) if p != rank]
    if got != want:
        raise RuntimeError("RCCL P2P pre-connect exchanged wrong values: %r" % (got,))


def backend_name() -> str:
    return _CTX.get("backend", "none")


def shutdown_distributed():
    """Tear the process groups down.  Captured HIP step graphs that recorded RCCL collectives (the data-parallel
    all-reduce) are released first: ``destroy_process_group`` blocks forever while such a graph is alive."""
    import sys
    import torch.distributed as dist
    _CTX.clear()
    hr = sys.modules.get("distributedtf_amd.engine.hip_resnet")
    if hr is not None and hr.release_graphs():
        import gc
        import torch
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
