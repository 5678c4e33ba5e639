"""Population-batched MNIST CNN training step on hand-written gfx950 kernels.

Reference model: ``mnist_model.py:62-126`` (conv5x5x32 -> pool -> conv5x5x64 -> pool -> dense 1024 ->
dropout 0.4 -> dense 10, sparse softmax CE).  One optimizer step of every resident member is a fixed
launch sequence over population-packed tensors (``ops/csrc/mnist.hip``, ``ops/csrc/gemm.hip``):

  wd_prep      conv2 weights -> flipped/transposed bf16 dgrad layout (tiny)
  conv1        fp32 direct conv + bias + ReLU + max-pool (argmax kept)        -> P1 [N,14,14,32] bf16
  conv2_fwd    MFMA implicit GEMM + bias + ReLU + max-pool in the epilogue   -> P2 [N,3136] bf16
  gemm NT      Z = P2 . W1^T per member (bf16 shadow weights)                -> Z [N,1024] fp32
  head         bias + ReLU + dropout + dense2 + CE, dense2 grads, dZ          -> dZ [N,1024] bf16
  gemm NN      dP2 = dZ . W1                                                   -> dP2 [N,3136] bf16
  gemm TN      dW1 += dZ^T . P2   (fp32, straight into the member's gradient row)
  conv2_dgrad  un-pool/mask + MFMA dgrad                                       -> dP1
  conv2_wgrad  dW2, db2 (ds_read_b64_tr_b16 fragments)
  conv1_wgrad  dW1c, db1c
  optimizer    fused launch over all members; also refreshes the bf16 shadow read by conv2 / dense1

The sequence is captured once per batch composition into a HIP graph and replayed.
Eval runs the forward kernels (conv1, conv2, the dense1 grouped GEMM, the head with dropout off) for every
member at once over chunks of the eval set (``evaluate_population``).
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Sequence

import numpy as np
import torch

from .. import ops
from ..data.datasets import IndexBatch, batch_len
from .hip_resnet import PinnedStager, advance_steps, note_step_advanced, run_captured, same_batches, upload_hyper

c_void_p, c_int, c_long, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float


class MnistArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("labels", c_void_p), ("img_slot", c_void_p), ("work", c_void_p),
        ("params", c_void_p), ("p_mstride", c_long), ("grads", c_void_p), ("g_mstride", c_long),
        ("shadow", c_void_p), ("s_mstride", c_long), ("wd", c_void_p), ("wd_mstride", c_long),
        ("p1", c_void_p), ("am1", c_void_p), ("p2", c_void_p), ("am2", c_void_p), ("z", c_void_p), ("dz", c_void_p),
        ("dp2", c_void_p), ("dp1", c_void_p), ("loss", c_void_p), ("correct", c_void_p), ("cnt", c_void_p),
        ("rng", c_void_p), ("logits_out", c_void_p),
        ("off_c1w", c_int), ("off_c1b", c_int), ("off_c2w", c_int), ("off_c2b", c_int),
        ("off_d1w", c_int), ("off_d1b", c_int), ("off_d2w", c_int), ("off_d2b", c_int),
        ("drop_rate", c_float), ("train", c_int), ("dz32", c_void_p),
    ]


class GemmGroup(ctypes.Structure):
    _fields_ = [("a_off", c_long), ("b_off", c_long), ("c_off", c_long), ("M", c_int), ("N", c_int), ("K", c_int),
                ("Ms", c_int)]


class GemmArgs(ctypes.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("C", c_void_p), ("lda", c_long), ("ldb", c_long), ("ldc", c_long),
                ("groups", c_void_p), ("work", c_void_p)]


GEMM_OUT_F32, GEMM_OUT_BF16, GEMM_OUT_ACC = 0, 1, 2

_REGISTERED = False


def _register():
    global _REGISTERED
    if _REGISTERED:
        return
    P = ctypes.POINTER
    for name in ("dtf_mnist_conv1", "dtf_mnist_conv2_fwd", "dtf_mnist_head", "dtf_mnist_conv2_dgrad",
                 "dtf_mnist_conv2_wgrad", "dtf_mnist_conv1_wgrad"):
        ops.register(name, [P(MnistArgs), c_int, c_void_p])
    ops.register("dtf_mnist_wd_prep", [P(MnistArgs), c_void_p, c_int, c_void_p])
    ops.register("dtf_gemm_bf16", [P(GemmArgs), c_int, c_int, c_void_p])
    for name in ("dtf_mnist_args_size", "dtf_gemm_args_size", "dtf_gemm_group_size"):
        ops.register(name, [])
    L = ops.lib()
    for name, args in ops._SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes = args
            fn.restype = c_int
    assert L.dtf_mnist_args_size() == ctypes.sizeof(MnistArgs), "MnistArgs ABI mismatch"
    assert L.dtf_gemm_args_size() == ctypes.sizeof(GemmArgs), "GemmArgs ABI mismatch"
    assert L.dtf_gemm_group_size() == ctypes.sizeof(GemmGroup), "GemmGroup ABI mismatch"
    _REGISTERED = True


def _p(t):
    return None if t is None else t.data_ptr()


def dropout_keep_mask(seed: int, counter: int, n_img: int, rate: float, features: int = 1024) -> np.ndarray:
    """Host replica of the head kernel's dropout hash: bool [n_img, features] (True = kept)."""
    from ..data.datasets import _mix32
    with np.errstate(over="ignore"):
        idx = (np.arange(n_img, dtype=np.uint32)[:, None] * np.uint32(features)
               + np.arange(features, dtype=np.uint32)[None, :])
        inner = _mix32((np.uint32(counter & 0xFFFFFFFF) * np.uint32(0x9E3779B9)).astype(np.uint32) + idx)
        h = _mix32(np.uint32(seed & 0xFFFFFFFF) ^ inner)
    thresh = np.uint32(min(int(rate * 4294967296.0), 0xFFFFFFFF))
    return h >= thresh


class GroupedGemm:
    """One grouped GEMM launch (a list of per-member problems) with its device tables."""

    def __init__(self, A, B, C, lda, ldb, ldc, problems, a_km, b_km, out, device):
        """problems: [(a_off, b_off, c_off, M, N, K[, Ms])] in elements; Ms = rows actually stored (<= M)."""
        problems = [tuple(p) + (0,) * (7 - len(p)) for p in problems]
        for (_, _, _, M, N, K, _) in problems:
            if not a_km:
                assert K % 32 == 0, "row-major A needs K % 32 == 0"
            else:
                assert M % 8 == 0
            if not b_km:
                assert K % 32 == 0, "[N][K] B needs K % 32 == 0"
            else:
                assert N % 8 == 0
        assert lda % 8 == 0 and ldb % 8 == 0
        groups = (GemmGroup * len(problems))()
        work = []
        for gi, (ao, bo, co, M, N, K, Ms) in enumerate(problems):
            groups[gi] = GemmGroup(ao, bo, co, M, N, K, Ms)
            for m0 in range(0, M, 64):
                for n0 in range(0, N, 64):
                    work.append([gi, m0, n0, 0])
        gbytes = torch.frombuffer(bytearray(bytes(groups)), dtype=torch.uint8)
        self.groups_t = gbytes.to(device)
        self.work_t = torch.tensor(work, dtype=torch.int32, device=device)
        self.args = GemmArgs(_p(A), _p(B), _p(C), lda, ldb, ldc, _p(self.groups_t), _p(self.work_t))
        self.mode = int(a_km) | (int(b_km) << 1) | (out << 2)
        self.nwork = len(work)
        self._keep = (A, B, C)

    def launch(self, stream):
        err = ops.lib().dtf_gemm_bf16(ctypes.byref(self.args), self.mode, self.nwork, stream)
        if err != 0:
            raise RuntimeError("gemm_bf16 launch failed: %d" % err)


class HipMnistBackend:
    name = "hip"
    accepts_index_batches = False

    def __init__(self, engine):
        _register()
        self.e = engine
        self.dev = engine.device
        arch = engine.arch
        self.offs = {n: arch.offsets[n][0] for n in arch.offsets}
        for n in ("conv2_w", "dense1_w"):
            assert self.offs[n] % 8 == 0, "bf16 shadow operands must be 16-byte aligned"
        cap = engine.capacity
        self.shadow = torch.zeros(cap, engine.Pp, dtype=torch.bfloat16, device=self.dev)
        self.wd = torch.zeros(cap, 51200, dtype=torch.bfloat16, device=self.dev)
        self.loss = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.correct = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.rng = torch.zeros(2, dtype=torch.int32, device=self.dev)
        self.rng_seed = 0x5EED
        self.rng_counter = 0
        self.drop_rate = float(getattr(arch, "dropout", 0.4))
        self._plans: Dict[tuple, "_MnistPlan"] = {}
        # training plans also write the head's logits (the "probabilities" hook, reference mnist_model.py:149-151);
        # set before the first step (EngineModel._hooks): the flag is baked into a plan's captured launches
        self.keep_probs = False
        self._last_plan = None
        self.use_graph = (os.environ.get("DTF_HIP_GRAPH", "1") == "1" and os.environ.get("DTF_DEBUG", "0") != "1")

    # engine hooks ----------------------------------------------------------------------------
    def on_params_changed(self, slots):
        slots = [s for s in slots]
        if slots:
            e = self.e
            self._rows = ops.shadow_refresh(e.state, self.shadow, slots, e.Pp, e.P)

    def shadow_weights(self):
        return self.shadow

    def _upload_rng(self, v):
        if getattr(self, "_rng_stage", None) is None:
            self._rng_stage = PinnedStager(2, torch.int32)
        self._rng_stage.upload(self.rng, v)

    def next_rng(self):
        self.rng_counter = (self.rng_counter + 1) & 0x7FFFFFFF
        return self.rng_seed, self.rng_counter

    def plan(self, slots, sizes):
        key = (tuple(slots), tuple(sizes))
        p = self._plans.get(key)
        if p is None:
            if len(self._plans) > 16:
                self._plans.clear()
            p = _MnistPlan(self, list(slots), list(sizes))
            self._plans[key] = p
        return p

    def train_step(self, slots, batches, hparams, lrs):
        e = self.e
        batches = [b.materialize() if isinstance(b, IndexBatch) else b for b in batches]
        sizes = [batch_len(b) for b in batches]
        p = self.plan(slots, sizes)
        upload_hyper(e, slots, hparams, lrs)
        self.last_rng = self.next_rng()
        self._upload_rng(self.last_rng)
        p.load_batch(batches)
        p.run()
        self._last_plan = p
        note_step_advanced(e, slots)
        return p.loss_sel.clone()  # gathered inside the step graph

    def forward_backward(self, slots, batches):
        raise RuntimeError("HipMnistBackend runs whole steps: use train_step")

    def train_correct(self, slots):
        """Correct predictions of each member's last training batch (head kernel count; device tensor)."""
        return self.correct[torch.as_tensor(list(slots), dtype=torch.long, device=self.dev)]

    def train_probabilities(self, slots):
        """Softmax of each member's last training batch (with dropout, as the reference's ``softmax_tensor`` in
        training mode): a list of [batch, 10] device tensors, or None when the plans do not keep logits."""
        p = self._last_plan
        if p is None or p.logits is None or p.eval:
            return None
        out = []
        for s in slots:
            if s not in p.first:
                out.append(None)
                continue
            f, n = p.first[s], p.sizes[p.slots.index(s)]
            out.append(torch.softmax(p.logits[f:f + n], dim=1))
        return out

    def eval_plan(self, slots, m):
        """Eval plans live in their own bounded cache: an eval pass never evicts the captured training graph."""
        key = (tuple(slots), int(m))
        plans = self.__dict__.setdefault("_eval_plans", {})
        p = plans.get(key)
        if p is None:
            if len(plans) >= 4:
                plans.pop(next(iter(plans)))  # oldest first
            p = _MnistPlan(self, list(slots), [int(m)] * len(slots), eval_mode=True)
            plans[key] = p
        return p

    @torch.no_grad()
    def infer(self, slot, x):
        """Eval-mode logits of one member on the HIP forward kernels (dropout off)."""
        p = self.eval_plan([slot], int(x.shape[0]))
        logits = p.want_logits()
        p.load_eval(x, torch.zeros(x.shape[0], dtype=torch.int32, device=x.device))
        p.run_eval()
        return logits.clone()

    @torch.no_grad()
    def evaluate_population(self, slots, x, y, chunk=None):
        """Eval accuracy of every member in ``slots``: one population-batched forward (conv1, conv2, dense1 grouped
        GEMM, head without dropout) per chunk of the eval set; one host sync at the end."""
        n = int(x.shape[0])
        if n == 0 or not slots:
            return {s: 0.0 for s in slots}
        chunk = min(n, int(chunk or os.environ.get("DTF_EVAL_CHUNK", "2500")))
        used = []
        for i in range(0, n, chunk):
            m = min(chunk, n - i)
            p = self.eval_plan(slots, m)
            if all(p is not q for q in used):
                p.ev_acc.zero_()
                used.append(p)
            p.load_eval(x[i:i + m], y[i:i + m])
            p.run_eval()
        correct = used[0].ev_acc[0].clone()
        for p in used[1:]:
            correct += p.ev_acc[0]
        vals = correct.cpu().tolist()
        return {s: vals[s] / float(n) for s in slots}


class _MnistPlan:
    def __init__(self, be: HipMnistBackend, slots: List[int], sizes: List[int], eval_mode: bool = False):
        self.be, self.e = be, be.e
        self.eval = bool(eval_mode)
        e, dev = be.e, be.dev
        self.slots, self.sizes = slots, sizes
        N = sum(sizes)
        self.N = N
        img_slot, self.first = [], {}
        for s, n in zip(slots, sizes):
            self.first[s] = len(img_slot)
            img_slot += [s] * n
        self.img_slot = torch.tensor(img_slot, dtype=torch.int32, device=dev)
        cnt = torch.zeros(e.capacity, dtype=torch.float32)
        for s, n in zip(slots, sizes):
            cnt[s] = float(n)
        self.cnt = cnt.to(dev)
        self.slots_t = torch.tensor(slots, dtype=torch.int32, device=dev)
        self.slots_long = torch.tensor(slots, dtype=torch.long, device=dev)
        self.loss_sel = torch.zeros(len(slots), dtype=be.loss.dtype, device=dev)
        bf = torch.bfloat16
        self.x = torch.zeros(N, 28, 28, dtype=torch.float32, device=dev)
        self.labels = torch.zeros(N, dtype=torch.int32, device=dev)
        self.p1 = torch.empty(N, 196, 32, dtype=bf, device=dev)
        self.am1 = torch.empty(N, 196, 32, dtype=torch.uint8, device=dev)
        self.p2 = torch.empty(N, 3136, dtype=bf, device=dev)
        self.am2 = torch.empty(N, 3136, dtype=torch.uint8, device=dev)
        self.z = torch.empty(N, 1024, dtype=torch.float32, device=dev)
        # backward temporaries (eval plans: forward only)
        nb = 1 if self.eval else N
        self.dz = torch.empty(nb, 1024, dtype=bf, device=dev)
        self.dp2 = torch.empty(nb, 3136, dtype=bf, device=dev)
        self.dp1 = torch.empty(nb, 196, 32, dtype=bf, device=dev)
        self.ev_acc = torch.zeros(2, e.capacity, dtype=torch.float32, device=dev)  # eval: [correct, summed CE]
        self.logits = None
        o = be.offs
        a = MnistArgs()
        a.x, a.labels, a.img_slot = _p(self.x), _p(self.labels), _p(self.img_slot)
        a.params, a.p_mstride = _p(e.state), e.S
        a.grads, a.g_mstride = _p(e.grads), e.Pp
        a.shadow, a.s_mstride = _p(be.shadow), e.Pp
        a.wd, a.wd_mstride = _p(be.wd), 51200
        a.p1, a.am1, a.p2, a.am2 = _p(self.p1), _p(self.am1), _p(self.p2), _p(self.am2)
        a.z, a.dz, a.dp2, a.dp1 = _p(self.z), _p(self.dz), _p(self.dp2), _p(self.dp1)
        a.loss, a.correct, a.cnt, a.rng = _p(be.loss), _p(be.correct), _p(self.cnt), _p(be.rng)
        a.logits_out = None
        if be.keep_probs and not self.eval:
            self.logits = torch.zeros(N, 10, dtype=torch.float32, device=dev)
            a.logits_out = _p(self.logits)
        a.off_c1w, a.off_c1b, a.off_c2w, a.off_c2b = o["conv1_w"], o["conv1_b"], o["conv2_w"], o["conv2_b"]
        a.off_d1w, a.off_d1b, a.off_d2w, a.off_d2b = o["dense1_w"], o["dense1_b"], o["dense2_w"], o["dense2_b"]
        a.drop_rate = be.drop_rate
        a.train = 0 if self.eval else 1
        if self.eval:  # counts accumulate over the eval chunks in the plan's own buffers
            a.loss, a.correct = _p(self.ev_acc[1]), _p(self.ev_acc[0])
        self.args = a
        # work lists (img0, nimg, 0, slot): image chunks of one member.  Deterministic build: ONE chunk per member
        # for every launch that adds into per-member accumulators (dense / conv weight gradients, bias gradients,
        # loss, correct count) -- each address then receives a single add onto zero, and every partial sum is
        # formed in a fixed order inside its workgroup, so the step replays bitwise (the GEMMs own their tiles)
        det = ops.build_deterministic()
        whole = 1 << 30
        self.w_fwd = self._chunks(max(1, -(-N // 512)))
        self.w_head = self._chunks(whole if det else 16)
        self.w_dgrad = self._chunks(max(1, -(-N // 512)))
        self.w_c2w = self._chunks(whole if det else max(4, -(-N * 5 // 320)))
        self.w_c1w = self._chunks(whole if det else max(4, -(-N // 256)))
        Pp, S = e.Pp, e.S
        d1 = o["dense1_w"]
        fwd, dgr, wgr = [], [], []
        for s, n in zip(slots, sizes):
            f = self.first[s]
            fwd.append((f * 3136, s * Pp + d1, f * 1024, n, 1024, 3136))     # Z = P2 W^T
            dgr.append((f * 1024, s * Pp + d1, f * 3136, n, 3136, 1024))     # dP2 = dZ W
            wgr.append((f * 1024, f * 3136, s * Pp + d1, 1024, 3136, n))     # dW += dZ^T P2
        self.g_fwd = GroupedGemm(self.p2, be.shadow, self.z, 3136, 3136, 1024, fwd, False, False, GEMM_OUT_F32, dev)
        if not self.eval:
            self.g_dgr = GroupedGemm(self.dz, be.shadow, self.dp2, 1024, 3136, 3136, dgr, False, True, GEMM_OUT_BF16,
                                     dev)
            self.g_wgr = GroupedGemm(self.dz, self.p2, e.grads, 1024, 3136, 3136, wgr, True, True, GEMM_OUT_ACC, dev)
        self.graph = None

    # ---- eval (mnist_model.py:167-172 ``mnist_classifier.evaluate``: dropout off)
    def want_logits(self):
        if self.logits is None:
            self.logits = torch.zeros(self.N, 10, dtype=torch.float32, device=self.be.dev)
            self.args.logits_out = _p(self.logits)
        return self.logits

    def load_eval(self, x, y):
        m, k = x.shape[0], len(self.slots)
        assert all(n == m for n in self.sizes)
        self.x.view(k, m, 28, 28).copy_(x.reshape(1, m, 28, 28).expand(k, -1, -1, -1))
        self.labels.view(k, m).copy_(y.reshape(1, m).expand(k, -1))

    def run_eval(self):
        assert self.eval
        L, st = ops.lib(), ops.stream()
        self._launch(L.dtf_mnist_conv1, n=self.N)
        self._launch(L.dtf_mnist_conv2_fwd, self.w_fwd)
        self.g_fwd.launch(st)
        self._launch(L.dtf_mnist_head, self.w_head)

    def _chunks(self, chunk):
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for i in range(0, n, chunk):
                items.append([f + i, min(chunk, n - i), 0, s])
        return torch.tensor(items, dtype=torch.int32, device=self.be.dev)

    def load_batch(self, batches):
        if same_batches(self, batches):
            return
        off = 0
        for (x, y) in batches:
            n = x.shape[0]
            self.x[off:off + n].copy_(x.reshape(n, 28, 28), non_blocking=True)
            self.labels[off:off + n].copy_(y, non_blocking=True)
            off += n

    def _launch(self, fn, work=None, n=None):
        a = self.args
        if work is not None:
            a.work = _p(work)
            n = work.shape[0]
        err = fn(ctypes.byref(a), n, ops.stream())
        if err != 0:
            raise RuntimeError("%s launch failed: %d" % (getattr(fn, "__name__", "mnist kernel"), err))

    def _run_eager(self):
        be, e, L = self.be, self.e, ops.lib()
        st = ops.stream()
        err = L.dtf_mnist_wd_prep(ctypes.byref(self.args), _p(self.slots_t), len(self.slots), st)
        if err:
            raise RuntimeError("mnist_wd_prep failed: %d" % err)
        be.loss.zero_()
        be.correct.zero_()
        self._launch(L.dtf_mnist_conv1, n=self.N)
        self._launch(L.dtf_mnist_conv2_fwd, self.w_fwd)
        self.g_fwd.launch(st)
        self._launch(L.dtf_mnist_head, self.w_head)
        self.g_dgr.launch(st)
        self.g_wgr.launch(st)
        self._launch(L.dtf_mnist_conv2_dgrad, self.w_dgrad)
        self._launch(L.dtf_mnist_conv2_wgrad, self.w_c2w)
        self._launch(L.dtf_mnist_conv1_wgrad, self.w_c1w)
        e.dp_sync_grads(self.slots)  # data-parallel member groups only (no-op otherwise)
        ops.fused_optimizer(e.state, e.grads, e.hyper, e.Pp, e.P, e.n_reg, shadow=be.shadow, zero_grads=True)
        advance_steps(e, self.slots_long, self.slots_t, be.loss, self.loss_sel)

    def run(self):
        run_captured(self)
