"""Population engine: every member of one GPU resident in HBM, trained together.

Replaces the reference's per-member serial loop that rebuilt a TF graph and
restored a checkpoint from disk for every ``train`` call
(``training_worker.py:64-69``, ``resnet_run_loop.py:397-406``).

State layout (one row per member slot, fp32)::

    state[g] = [ params (P) | slot1 (P) | slot2 (P) | bn running stats (R) | step | pad ]

so a member's full training state -- the exploit payload -- is one contiguous
row: an exploit is a single RCCL send/recv (or D2D copy) of ``state[g]`` with no
packing.  Gradients live in ``grads[G, P]``; bf16 shadow weights, activations
and workspaces belong to the backend.

Backends:
  * ``TorchBackend`` -- per-member PyTorch autograd on views of the flat
    buffers.  Numerics oracle, CPU path, and the path for architectures without
    HIP kernels.
  * ``HipResNetBackend`` (``engine/hip_resnet.py``) -- population-batched
    CDNA4 kernels: all members' images in one launch per layer.
The optimizer is one fused launch over every row (``ops.fused_optimizer``) or
the PyTorch reference on CPU.
"""

from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from . import optim as _optim
from ..data.datasets import IndexBatch


def _align(n: int, a: int = 64) -> int:
    return (n + a - 1) // a * a


class PopulationEngine:
    def __init__(self, arch, capacity: int, device, backend: str = "auto", compute_dtype=torch.bfloat16,
                 optimizer_impl: str = "auto", loss_scale: float = 1.0):
        self.arch = arch
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.P = arch.n_params
        self.R = arch.n_running
        self.n_reg = arch.n_reg
        self.Pp = _align(self.P, 64)   # 256-B aligned slot offsets -> float4 kernels
        self.S = _align(3 * self.Pp + self.R + 1)
        self.state = torch.zeros(self.capacity, self.S, dtype=torch.float32, device=self.device)
        self.grads = torch.zeros(self.capacity, self.Pp, dtype=torch.float32, device=self.device)
        self.hyper = torch.zeros(self.capacity, _optim.N_HYPER, dtype=torch.float32, device=self.device)
        self.free_slots = list(range(self.capacity))
        self.members: Dict[int, object] = {}
        self.host_step = [0] * self.capacity
        self.compute_dtype = compute_dtype
        if self.device.type == "cpu" and compute_dtype == torch.bfloat16:
            self.compute_dtype = torch.float32
        self.loss_scale = float(loss_scale)  # static loss scaling of the PyTorch path (fp16; resnet_run_loop.py:284)
        self.dp = None  # parallel.dataparallel.DPContext when a member is trained by a group of ranks
        # data parallelism: this replica's gradient weight per member row (local shard / member batch), a device
        # buffer so the captured step graph reads the current step's weights
        self.dp_weight = torch.zeros(self.capacity, dtype=torch.float32, device=self.device)
        self.backend = make_backend(self, backend)
        if optimizer_impl == "auto":
            optimizer_impl = "hip" if self.device.type == "cuda" else "reference"
        self.optimizer_impl = optimizer_impl

    # ----------------------------------------------------------------- views
    @property
    def params(self):
        return self.state[:, :self.P]

    @property
    def slot1(self):
        return self.state[:, self.Pp:self.Pp + self.P]

    @property
    def slot2(self):
        return self.state[:, 2 * self.Pp:2 * self.Pp + self.P]

    @property
    def running(self):
        return self.state[:, 3 * self.Pp:3 * self.Pp + self.R]

    def step_col(self):
        return self.state[:, 3 * self.Pp + self.R]

    def state_row(self, slot: int) -> torch.Tensor:
        return self.state[slot]

    # --------------------------------------------------------------- members
    def add_member(self, member, hparams: Dict, seed: int) -> int:
        if not self.free_slots:
            raise RuntimeError("population engine is full (capacity %d)" % self.capacity)
        slot = self.free_slots.pop(0)
        self.members[slot] = member
        p, r = self.arch.init_params(hparams.get("initializer"), seed)
        row = self.state[slot]
        row.zero_()
        row[:self.P] = p.to(self.device)
        row[3 * self.Pp:3 * self.Pp + self.R] = r.to(self.device)
        s1, s2 = _optim.slot_init_values(hparams["opt_case"]["optimizer"])
        if s1:
            row[self.Pp:self.Pp + self.P] = s1
        if s2:
            row[2 * self.Pp:2 * self.Pp + self.P] = s2
        self.host_step[slot] = 0
        self.backend.on_params_changed([slot])
        return slot

    def remove_member(self, slot: int) -> None:
        self.members.pop(slot, None)
        if slot not in self.free_slots:
            self.free_slots.append(slot)
            self.free_slots.sort()

    def on_state_imported(self, slot: int, step: int) -> None:
        """A member's state row was overwritten (exploit / checkpoint import).  ``step``: the source's host step
        counter -- always known on the host (all-gathered with the scores, or sent on the control plane), so an
        import never reads the device row back (no sync that would drain the queued steps)."""
        self.host_step[slot] = int(step)
        self.backend.on_params_changed([slot])

    # --------------------------------------------------------------- training
    def set_hyper(self, slot: int, hparams: Dict, lr: float, active: bool = True) -> None:
        row = _optim.hyper_row(hparams, lr, self.host_step[slot] + 1, active)
        self.hyper[slot] = torch.tensor(row, dtype=torch.float32)
        self._hyper_dev = None  # invalidate the HIP backends' upload cache

    def train_step(self, slots: Sequence[int], batches: Sequence[Tuple[torch.Tensor, torch.Tensor]],
                   hparams: Sequence[Dict], lrs: Sequence[float]) -> torch.Tensor:
        """One optimizer step for ``slots`` (each with its own batch). Returns
        per-member cross-entropy losses (device tensor)."""
        if not getattr(self.backend, "accepts_index_batches", False):
            batches = [b.materialize() if isinstance(b, IndexBatch) else b for b in batches]
        if self.dp is not None:
            self._set_dp_weights(slots, batches, hparams)
        if hasattr(self.backend, "train_step"):
            # whole step (fwd, bwd, optimizer, step counters) inside one HIP graph
            losses = self.backend.train_step(slots, batches, hparams, lrs)
            for s in slots:
                self.host_step[s] += 1
            return losses
        hy = torch.zeros(self.capacity, _optim.N_HYPER, dtype=torch.float32)
        for s, hp, lr in zip(slots, hparams, lrs):
            hy[s] = torch.tensor(_optim.hyper_row(hp, lr, self.host_step[s] + 1, True))
        self.hyper.copy_(hy.to(self.device), non_blocking=True)
        self._hyper_dev = None
        losses = self.backend.forward_backward(slots, batches)
        self.dp_sync_grads(slots)
        self.apply_optimizer(slots)
        for s in slots:
            self.host_step[s] += 1
        sc = self.step_col()
        idx = torch.tensor(list(slots), device=self.device, dtype=torch.long)
        sc.index_add_(0, idx, torch.ones(len(slots), device=self.device))
        self.backend.on_params_changed(slots)
        return losses

    # ------------------------------------------------------- data parallelism
    def set_data_parallel(self, dp) -> None:
        self.dp = dp
        self._dp_idx = {}

    def _set_dp_weights(self, slots, batches, hparams) -> None:
        """This replica's share of each member's batch: local images / member batch size (the hparam)."""
        from ..data.datasets import batch_len
        w = [0.0] * self.capacity
        for s, b, hp in zip(slots, batches, hparams):
            w[s] = batch_len(b) / float(max(1, int(hp["batch_size"])))
        key = tuple(w)
        if getattr(self, "_dp_w_host", None) != key:
            self.dp_weight.copy_(torch.tensor(w, dtype=torch.float32))
            self._dp_w_host = key

    def dp_sync_grads(self, slots: Sequence[int]) -> None:
        """Gradient rows of the members summed over the member group, each replica's row weighted by its share of
        the member batch (before the optimizer; inside the captured step on the HIP backends)."""
        if self.dp is None or not slots:
            return
        key = tuple(sorted(slots))
        idx = self._dp_idx.get(key)
        if idx is None:
            idx = self._dp_idx[key] = torch.tensor(key, device=self.device, dtype=torch.long)
        g = self.grads.index_select(0, idx)
        self.dp.allreduce_weighted_(g, self.dp_weight.index_select(0, idx))
        self.grads.index_copy_(0, idx, g)

    def dp_sync_running(self, slots: Sequence[int]) -> None:
        """Mean of the BatchNorm running statistics over the member group (end of a round)."""
        if self.dp is None or not slots or self.R == 0:
            return
        idx = torch.tensor(sorted(slots), device=self.device, dtype=torch.long)
        lo, hi = 3 * self.Pp, 3 * self.Pp + self.R
        r = self.state[:, lo:hi].index_select(0, idx)
        self.dp.allreduce_mean_(r)
        self.state[:, lo:hi].index_copy_(0, idx, r)

    def apply_optimizer(self, slots: Sequence[int]) -> None:
        if self.optimizer_impl == "hip":
            from ..ops import fused_optimizer
            fused_optimizer(self.state, self.grads, self.hyper, self.Pp, self.P, self.n_reg,
                            shadow=self.backend.shadow_weights(), zero_grads=True)
        else:
            _optim.apply_reference(self.params, self.grads[:, :self.P], self.slot1, self.slot2, self.hyper,
                                   self.n_reg, rows=list(slots))
            self.grads.zero_()

    @torch.no_grad()
    def evaluate_population(self, slots: Sequence[int], x: torch.Tensor, y: torch.Tensor) -> Dict[int, float]:
        """Eval accuracy of every member in ``slots`` (moving BN statistics): one population-batched forward per
        chunk on backends that have it (HIP), else member by member."""
        slots = list(slots)
        if hasattr(self.backend, "evaluate_population") and slots:
            return self.backend.evaluate_population(slots, x, y)
        return {s: self.evaluate(s, x, y) for s in slots}

    @torch.no_grad()
    def evaluate(self, slot: int, x: torch.Tensor, y: torch.Tensor, batch: int = 1000) -> float:
        if hasattr(self.backend, "evaluate_population"):
            return self.backend.evaluate_population([slot], x, y)[slot]
        correct = 0
        for i in range(0, x.shape[0], batch):
            logits = self.backend.infer(slot, x[i:i + batch])
            correct += int((logits.argmax(dim=1) == y[i:i + batch].to(logits.device)).sum().item())
        return correct / float(max(1, x.shape[0]))


# ----------------------------------------------------------------------- backends

class TorchBackend:
    """Per-member autograd on flat-buffer views (oracle / fallback path)."""

    name = "torch"

    def __init__(self, engine: PopulationEngine):
        self.e = engine
        if engine.device.type == "cuda" and os.environ.get("DTF_MIOPEN_FIND", "0") == "1":
            # MIOpen: benchmark the conv solvers once per shape instead of immediate-mode heuristics.  Off by
            # default: on a cold MIOpen cache the bf16 backward find ran a solver that faulted the GPU
            # ("illegal memory access" surfacing at MIOpen's next module load).
            torch.backends.cudnn.benchmark = True

    def on_params_changed(self, slots):
        pass

    def shadow_weights(self):
        return None

    keep_probs = False  # the "probabilities" hook: keep each member's training softmax (train_probabilities)

    def train_probabilities(self, slots):
        probs = getattr(self, "_probs", {})
        return [probs.get(s) for s in slots]

    def forward_backward(self, slots, batches):
        e = self.e
        losses = []
        if self.keep_probs:
            self._probs = {}
        for s, (x, y) in zip(slots, batches):
            p = e.params[s].detach().clone().requires_grad_(True)
            logits = e.arch.forward(p, e.running[s], x, training=True, dtype=e.compute_dtype)
            if self.keep_probs:
                self._probs[s] = torch.softmax(logits.detach().float(), dim=1)
            loss = F.cross_entropy(logits.float(), y.long())
            if e.loss_scale != 1.0:
                g, = torch.autograd.grad(loss * e.loss_scale, p)
                g = g / e.loss_scale
            else:
                g, = torch.autograd.grad(loss, p)
            e.grads[s, :e.P].copy_(g)
            losses.append(loss.detach())
        return torch.stack(losses) if losses else torch.zeros(0, device=e.device)

    def infer(self, slot, x):
        e = self.e
        return e.arch.forward(e.params[slot], e.running[slot], x, training=False, dtype=e.compute_dtype)


def _half_lib_loaded() -> bool:
    """The process runs the fp16 kernel build (DTF_HALF=1): its 16-bit kernels cannot serve a bf16 engine."""
    from .. import ops
    return ops.half_mode()


def _hip_f32_ok(engine) -> bool:
    """fp32 HIP steps: CIFAR-shape building-block ResNets (engine/hip_f32.py), the MNIST CNN
    (engine/hip_mnist_f32.py), the ImageNet-shape bottleneck ResNets (engine/hip_imagenet_f32.py)."""
    if engine.compute_dtype != torch.float32:
        return False
    from .. import ops
    if ops.half_mode():  # the fp32 step shares 16-bit helper kernels (input packing) with the bf16 build
        return False
    if getattr(engine.arch, "name", "") == "mnist_cnn":
        return True
    from .hip_f32 import supports
    from .hip_imagenet_f32 import supports as supports_bottleneck
    return supports(engine.arch) or supports_bottleneck(engine.arch)


def _hip_f16_ok(engine) -> bool:
    """fp16 HIP step: the half build of the bf16 kernels (ops/csrc/common.h DTF_HALF; loaded for DTF_HALF=1, which
    --dtype fp16 sets) for the ResNet v2 families -- the reference's fp16 mode exists for ResNet only and forbids v1
    (resnet_run_loop.py:546-549)."""
    if engine.compute_dtype != torch.float16:
        return False
    from .. import ops
    if not ops.half_mode() or ops.debug_mode():  # deterministic: the deterministic half build
        return False
    cfg = getattr(engine.arch, "cfg", None)
    return cfg is not None and getattr(cfg, "version", 0) == 2 and getattr(engine.arch, "name", "") != "mnist_cnn"


def make_backend(engine: PopulationEngine, name: str):
    ok16 = engine.compute_dtype == torch.bfloat16 and not (engine.device.type == "cuda" and _half_lib_loaded())
    if name == "auto":
        name = "hip" if (engine.device.type == "cuda" and getattr(engine.arch, "hip_supported", False)
                         and (ok16 or _hip_f32_ok(engine) or _hip_f16_ok(engine))) else "torch"
    if name == "hip" and not (ok16 or _hip_f32_ok(engine) or _hip_f16_ok(engine)):
        raise ValueError("no HIP step for compute dtype %s here (bf16 and fp32: every family; fp16: "
                         "the ResNet v2 families under DTF_HALF=1, which --dtype fp16 sets): use the torch backend"
                         % engine.compute_dtype)
    if name == "torch":
        return TorchBackend(engine)
    if name == "hip" and engine.compute_dtype == torch.float32:
        if getattr(engine.arch, "name", "") == "mnist_cnn":
            from .hip_mnist_f32 import HipMnistF32Backend
            return HipMnistF32Backend(engine)
        if getattr(getattr(engine.arch, "cfg", None), "bottleneck", False):
            from .hip_imagenet_f32 import HipImageNetF32Backend
            return HipImageNetF32Backend(engine)
        from .hip_f32 import HipResNetF32Backend
        return HipResNetF32Backend(engine)
    if name == "hip":
        if getattr(engine.arch, "name", "") == "mnist_cnn":
            from .hip_mnist import HipMnistBackend
            return HipMnistBackend(engine)
        if getattr(getattr(engine.arch, "cfg", None), "bottleneck", False):
            from .hip_imagenet import HipImageNetBackend
            return HipImageNetBackend(engine)
        from .hip_resnet import HipResNetBackend
        return HipResNetBackend(engine)
    raise ValueError("unknown backend %r" % name)
