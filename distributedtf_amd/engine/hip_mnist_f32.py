"""Population-batched fp32 MNIST CNN training step on gfx950 kernels: ``--dtype fp32 --model mnist``.

Reference model: ``mnist_model.py:62-126`` (conv5x5x32 -> pool -> conv5x5x64 -> pool -> dense 1024 -> dropout 0.4
-> dense 10), trained in fp32 (the reference's default dtype).  The bf16 step (engine/hip_mnist.py) stores
activations and GEMM operands in bf16; this one keeps every tensor, weight and accumulation in fp32 and runs every
matrix product on v_mfma_f32_16x16x4_f32 through the generic fp32 conv kernels of the CIFAR fp32 step
(ops/csrc/f32conv.hip):

  prep          x [N,28,28] -> [N,28,28,4] (channel 0 = pixel; the conv gathers 4 channels, the weight row has 1)
  conv1         f32conv 5x5 SAME, 4 (1 real) -> 32                                    -> H1 [N,28,28,32]
  pool1         bias + ReLU + 2x2 max-pool, argmax kept (mnist.hip)                    -> P1 [N,14,14,32]
  conv2         f32conv 5x5 SAME, 32 -> 64                                             -> H2 [N,14,14,64]
  pool2                                                                                -> P2 [N,7,7,64]
  dense1        f32conv 7x7 VALID over P2 (= P2 flattened in TF's (h, w, c) order . W1^T) -> Z [N,1024]
  head          bias + ReLU + dropout + dense2 + CE, dense2 / dense1-bias grads (mnist.hip head, fp32 dZ)
  dense1 dgrad  f32conv data gradient of a 1x1 conv: dP2[n][j] = sum_f dZ[n][f] W1[f][j]   -> dP2 [N,7,7,64]
  dense1 wgrad  f32 weight gradient of the 7x7 conv: dW1[f][j] += sum_n dZ[n][f] P2[n][j]
  unpool2       ReLU mask + un-pool + conv2 bias gradient                               -> dH2
  conv2 dgrad / wgrad, unpool1, conv1 wgrad
  optimizer     fused multi-optimizer kernel on the fp32 rows (no bf16 shadow)

Deterministic build (``--deterministic --dtype fp32``): the weight and bias gradients accumulate as int64 fixed
point (common.h DTF_FIXED_ACC, order-free integer atomics) and ``cg_det_finish`` folds them into the fp32 rows;
the head runs one workgroup per member (each of its gradient addresses gets one add onto zero).  The step is
captured in one HIP graph per batch composition.
"""

from __future__ import annotations

import ctypes
import os
from typing import List

import torch

from .. import ops
from .hip_f32 import F32Args, TP, WG_CHUNK, _register as _register_f32
from .hip_mnist import HipMnistBackend, MnistArgs, _register as _register_mnist
from .hip_resnet import advance_steps, run_captured

c_void_p, c_int, c_long = ctypes.c_void_p, ctypes.c_int, ctypes.c_long


class PoolArgs(ctypes.Structure):
    _fields_ = [("h", c_void_p), ("p", c_void_p), ("am", c_void_p), ("dp", c_void_p), ("dh", c_void_p),
                ("img_slot", c_void_p), ("work", c_void_p), ("params", c_void_p), ("p_mstride", c_long),
                ("grads", c_void_p), ("g_mstride", c_long), ("b_off", c_int), ("H", c_int), ("C", c_int),
                ("pad_", c_int), ("nimg", c_long)]


_REGISTERED = False


def _register():
    global _REGISTERED
    if _REGISTERED:
        return
    _register_mnist()
    _register_f32()
    from .hip_imagenet import _register as _reg_cg
    _reg_cg()  # dtf_cg_det_finish
    P = ctypes.POINTER
    ops.register("dtf_mnist_f32_prep", [c_void_p, c_void_p, c_long, c_void_p])
    ops.register("dtf_mnist_f32_pool", [P(PoolArgs), c_void_p])
    ops.register("dtf_mnist_f32_unpool", [P(PoolArgs), c_int, c_void_p])
    ops.register("dtf_mnist_pool_args_size", [])
    L = ops.lib()
    for name, args in ops._SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes = args
            fn.restype = c_int
    assert L.dtf_mnist_pool_args_size() == ctypes.sizeof(PoolArgs), "PoolArgs ABI mismatch"
    _REGISTERED = True


def _p(t):
    return None if t is None else t.data_ptr()


class HipMnistF32Backend(HipMnistBackend):
    """fp32 MNIST step: the bf16 backend's engine hooks, rng and eval drivers over fp32 plans."""

    def __init__(self, engine):
        _register()
        e = engine
        self.e = e
        self.dev = e.device
        arch = e.arch
        self.offs = {n: arch.offsets[n][0] for n in arch.offsets}
        for n in ("dense1_b", "dense2_w"):
            assert self.offs[n] % 4 == 0, "the head reads float4 rows"
        cap = e.capacity
        self.det = bool(ops.lib().dtf_fixed_acc())
        self.gacc = torch.zeros(cap, e.Pp, dtype=torch.int64, device=self.dev) if self.det else None
        self.loss_sink = torch.zeros(cap, dtype=torch.float32, device=self.dev) if self.det else None
        self.loss64_sink = torch.zeros(cap, dtype=torch.int64, device=self.dev) if self.det else None
        self.shadow = None
        self.loss = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.correct = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.rng = torch.zeros(2, dtype=torch.int32, device=self.dev)
        self.rng_seed = 0x5EED
        self.rng_counter = 0
        self.drop_rate = float(getattr(arch, "dropout", 0.4))
        self._plans = {}
        self.keep_probs = False
        self._last_plan = None
        self.use_graph = (os.environ.get("DTF_HIP_GRAPH", "1") == "1" and os.environ.get("DTF_DEBUG", "0") != "1")

    def on_params_changed(self, slots):
        pass  # the kernels read the fp32 master rows directly

    def shadow_weights(self):
        return None

    def plan(self, slots, sizes):
        key = (tuple(slots), tuple(sizes))
        p = self._plans.get(key)
        if p is None:
            if len(self._plans) > 16:
                self._plans.clear()
            p = _MnistF32Plan(self, list(slots), list(sizes))
            self._plans[key] = p
        return p

    def eval_plan(self, slots, m):
        key = (tuple(slots), int(m))
        plans = self.__dict__.setdefault("_eval_plans", {})
        p = plans.get(key)
        if p is None:
            if len(plans) >= 4:
                plans.pop(next(iter(plans)))
            p = _MnistF32Plan(self, list(slots), [int(m)] * len(slots), eval_mode=True)
            plans[key] = p
        return p


class _MnistF32Plan:
    def __init__(self, be: HipMnistF32Backend, slots: List[int], sizes: List[int], eval_mode: bool = False):
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
        self.loss_sel = torch.zeros(len(slots), dtype=torch.float32, device=dev)
        f32 = torch.float32

        def t(*shape, dtype=f32):
            return torch.empty(*shape, dtype=dtype, device=dev)

        self.x = torch.zeros(N, 28, 28, dtype=f32, device=dev)
        self.labels = torch.zeros(N, dtype=torch.int32, device=dev)
        self.x4 = t(N, 28, 28, 4)
        self.h1, self.p1, self.am1 = t(N, 28, 28, 32), t(N, 14, 14, 32), t(N, 14, 14, 32, dtype=torch.uint8)
        self.h2, self.p2, self.am2 = t(N, 14, 14, 64), t(N, 7, 7, 64), t(N, 7, 7, 64, dtype=torch.uint8)
        self.z = t(N, 1024)
        if not self.eval:
            self.dz, self.dp2, self.dh2 = t(N, 1024), t(N, 7, 7, 64), t(N, 14, 14, 64)
            self.dp1, self.dh1 = t(N, 14, 14, 32), t(N, 28, 28, 32)
        self.ev_acc = torch.zeros(2, e.capacity, dtype=f32, device=dev)  # eval: [correct, summed CE]
        self.logits = None
        self._keep = []
        self.launches = []
        self.graph = None
        o = be.offs
        a = MnistArgs()
        a.labels, a.img_slot = _p(self.labels), _p(self.img_slot)
        a.params, a.p_mstride = _p(e.state), e.S
        a.grads, a.g_mstride = _p(e.grads), e.Pp
        a.z, a.dz32 = _p(self.z), None if self.eval else _p(self.dz)
        a.loss, a.correct, a.cnt, a.rng = _p(be.loss), _p(be.correct), _p(self.cnt), _p(be.rng)
        a.off_c1w, a.off_c1b, a.off_c2w, a.off_c2b = o["conv1_w"], o["conv1_b"], o["conv2_w"], o["conv2_b"]
        a.off_d1w, a.off_d1b, a.off_d2w, a.off_d2b = o["dense1_w"], o["dense1_b"], o["dense2_w"], o["dense2_b"]
        a.drop_rate = be.drop_rate
        a.train = 0 if self.eval else 1
        if self.eval:
            a.loss, a.correct = _p(self.ev_acc[1]), _p(self.ev_acc[0])
        self.head_args = a
        if be.keep_probs and not self.eval:  # the "probabilities" hook (HipMnistBackend.train_probabilities)
            self.logits = torch.zeros(N, 10, dtype=torch.float32, device=dev)
            a.logits_out = _p(self.logits)
        # head chunks (img0, nimg, 0, slot): deterministic build -> one workgroup per member
        self.w_head = self._chunks(1 << 30 if be.det else 16)
        self._build()

    # ------------------------------------------------------------------------------------------------ helpers
    def _chunks(self, chunk):
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for i in range(0, n, chunk):
                items.append([f + i, min(chunk, n - i), 0, s])
        return torch.tensor(items, dtype=torch.int32, device=self.be.dev)

    def _add(self, fn, *args):
        self.launches.append((fn, args))

    def _hold(self, o):
        self._keep.append(o)
        return o

    def _f32args(self, w_off, Hi, Ci, wci, Ho, Co, k, pad):
        e = self.e
        a = F32Args()
        a.w, a.w_mstride, a.w_off = _p(e.state), e.S, w_off
        a.grads, a.g_mstride, a.g_off = _p(self.be.gacc if self.be.det else e.grads), e.Pp, w_off
        a.Hi = a.Wi = Hi
        a.Ho = a.Wo = Ho
        a.Ci, a.wci, a.Co = Ci, wci, Co
        a.kh = a.kw = k
        a.stride, a.pad = 1, pad
        a.cmax = 64
        a.log2ci = Ci.bit_length() - 1
        assert Ci >= 4 and Ci & (Ci - 1) == 0 and Co % 4 == 0, (Ci, Co)
        return a

    def conv(self, src, out, w_off, Hi, Ci, wci, Ho, Co, k, pad, dgrad=False):
        """Forward conv (gather src [N,Hi,Hi,Ci] -> out [N,Ho,Ho,Co]) or the data gradient of a conv whose
        OUTPUT has Ci channels (src = dy) and whose input has Co (weights OHWI [Ci][k][k][Co])."""
        a = self._f32args(w_off, Hi, Ci, wci, Ho, Co, k, pad)
        assert src.shape == (self.N, Hi, Hi, Ci) or src.numel() == self.N * Hi * Hi * Ci, (src.shape, Hi, Ci)
        assert out.numel() == self.N * Ho * Ho * Co, (out.shape, Ho, Co)
        a.x, a.y = _p(src), _p(out)
        tc = min(64, Co)
        assert Co % tc == 0
        hwo = Ho * Ho
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for p0 in range(f * hwo, (f + n) * hwo, TP[tc]):
                for o0 in range(0, Co, tc):
                    items.append([s, p0, min(p0 + TP[tc], (f + n) * hwo), o0])
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_f32_conv, ctypes.byref(a), tc, 0, 0, int(dgrad), work.shape[0])

    def wgrad(self, x, dy, w_off, Hi, Ci, wci, Ho, Co, k, pad):
        a = self._f32args(w_off, Hi, Ci, wci, Ho, Co, k, pad)
        assert x.numel() == self.N * Hi * Hi * Ci and dy.numel() == self.N * Ho * Ho * Co
        a.x, a.dy = _p(x), _p(dy)
        K = k * k * Ci
        tc = min(64, Co)
        hwo = Ho * Ho
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for p0 in range(f * hwo, (f + n) * hwo, WG_CHUNK):
                for o0 in range(0, Co, tc):
                    for n0 in range(0, K, 64):
                        items.append([s, p0, min(p0 + WG_CHUNK, (f + n) * hwo), o0 | ((n0 // 16) << 16)])
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_f32_wgrad, ctypes.byref(a), tc, 0, 0, work.shape[0])

    def _pool_args(self, h, p, am, b_off, H, C):
        e = self.e
        a = PoolArgs()
        a.h, a.p, a.am = _p(h), _p(p), _p(am)
        a.img_slot, a.params, a.p_mstride = _p(self.img_slot), _p(e.state), e.S
        a.grads, a.g_mstride = _p(self.be.gacc if self.be.det else e.grads), e.Pp
        a.b_off, a.H, a.C, a.nimg = b_off, H, C, self.N
        return a

    def pool(self, h, p, am, b_off, H, C):
        a = self._hold(self._pool_args(h, p, am, b_off, H, C))
        self._add(ops.lib().dtf_mnist_f32_pool, ctypes.byref(a))

    def unpool(self, dp, p, am, dh, b_off, H, C):
        a = self._pool_args(None, p, am, b_off, H, C)
        a.dp, a.dh = _p(dp), _p(dh)
        work = self._hold(self._chunks(max(1, -(-self.N // 1024))))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_mnist_f32_unpool, ctypes.byref(a), work.shape[0])

    # ------------------------------------------------------------------------------------------------ program
    def _forward(self):
        o, N = self.be.offs, self.N
        self._add(ops.lib().dtf_mnist_f32_prep, _p(self.x), _p(self.x4), N * 784)
        self.conv(self.x4, self.h1, o["conv1_w"], 28, 4, 1, 28, 32, 5, 2)
        self.pool(self.h1, self.p1, self.am1, o["conv1_b"], 28, 32)
        self.conv(self.p1, self.h2, o["conv2_w"], 14, 32, 32, 14, 64, 5, 2)
        self.pool(self.h2, self.p2, self.am2, o["conv2_b"], 14, 64)
        self.conv(self.p2, self.z, o["dense1_w"], 7, 64, 64, 1, 1024, 7, 0)
        self._add("head", None)

    def _build(self):
        o, be, e = self.be.offs, self.be, self.e
        if not self.eval:
            self._add("zero", be.loss)
            self._add("zero", be.correct)
        self._forward()
        if self.eval:
            return
        # dense1: dP2 = dZ . W1 (the 1x1-conv data gradient: A[k = f][m = j] = W1[f][j]) and dW1 += dZ^T . P2
        self.conv(self.dz, self.dp2, o["dense1_w"], 1, 1024, 1024, 1, 3136, 1, 0, dgrad=True)
        self.wgrad(self.p2, self.dz, o["dense1_w"], 7, 64, 64, 1, 1024, 7, 0)
        self.unpool(self.dp2, self.p2, self.am2, self.dh2, o["conv2_b"], 14, 64)
        self.conv(self.dh2, self.dp1, o["conv2_w"], 14, 64, 64, 14, 32, 5, 2, dgrad=True)
        self.wgrad(self.p1, self.dh2, o["conv2_w"], 14, 32, 32, 14, 64, 5, 2)
        self.unpool(self.dp1, self.p1, self.am1, self.dh1, o["conv1_b"], 28, 32)
        self.wgrad(self.x4, self.dh1, o["conv1_w"], 28, 4, 1, 28, 32, 5, 2)
        if be.det:
            self._add(ops.lib().dtf_cg_det_finish, _p(be.gacc), _p(e.grads), e.Pp, e.Pp, _p(self.slots_t),
                      len(self.slots), _p(be.loss64_sink), _p(be.loss_sink))
        self._add("optim", None)
        self._add("step", None)

    # ------------------------------------------------------------------------------------------------ execution
    def want_logits(self):
        if self.logits is None:
            self.logits = torch.zeros(self.N, 10, dtype=torch.float32, device=self.be.dev)
            self.head_args.logits_out = _p(self.logits)
        return self.logits

    def load_eval(self, x, y):
        m, k = x.shape[0], len(self.slots)
        assert all(n == m for n in self.sizes)
        self.x.view(k, m, 28, 28).copy_(x.reshape(1, m, 28, 28).expand(k, -1, -1, -1))
        self.labels.view(k, m).copy_(y.reshape(1, m).expand(k, -1))

    def load_batch(self, batches):
        from .hip_resnet import same_batches
        if same_batches(self, batches):
            return
        off = 0
        for (x, y) in batches:
            n = x.shape[0]
            self.x[off:off + n].copy_(x.reshape(n, 28, 28), non_blocking=True)
            self.labels[off:off + n].copy_(y, non_blocking=True)
            off += n

    def run_eval(self):
        assert self.eval
        self._run_eager()

    def run(self):
        run_captured(self)

    def _run_eager(self):
        e, be = self.e, self.be
        st = ops.stream()
        for fn, args in self.launches:
            if fn == "zero":
                args[0].zero_()
            elif fn == "head":
                ops.check(ops.lib().dtf_mnist_head(ctypes.byref(self._head_with_work()), self.w_head.shape[0], st),
                          "mnist_head (fp32)")
            elif fn == "optim":
                e.dp_sync_grads(self.slots)
                ops.fused_optimizer(e.state, e.grads, e.hyper, e.Pp, e.P, e.n_reg, shadow=None, zero_grads=True)
            elif fn == "step":
                advance_steps(e, self.slots_long, self.slots_t, be.loss, self.loss_sel)
            else:
                err = fn(*args, st)
                if err != 0:
                    raise RuntimeError("kernel launch %s failed with %d" % (getattr(fn, "__name__", fn), err))

    def _head_with_work(self):
        self.head_args.work = _p(self.w_head)
        return self.head_args
