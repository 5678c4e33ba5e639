"""Population-batched fp32 CIFAR ResNet (v1 / v2 building blocks) training step on gfx950 kernels: ``--dtype fp32``.

The reference trains in fp32 by default (``resnet/official/utils/flags/_performance.py:30-33,105-108``; the dtype
flag feeds ``resnet_model.Model``'s custom getter, ``resnet_model.py:439-474``).  The bf16 engine
(``engine/hip_resnet.py``) is the throughput path; this one keeps every tensor, weight and accumulation in fp32
(``ops/csrc/f32conv.hip``: v_mfma_f32_16x16x4_f32) so a member trains with fp32 numerics on the GPU instead of
falling back to per-member PyTorch eager.

Structure (per member row, all members packed along N as in the bf16 engine):
  v2 (``_building_block_v2``, resnet_model.py:171-212): the pre-activation BN+ReLU of each conv is applied while
     its operand is gathered (MODE 1), the conv epilogue produces the next BN's statistics (and adds the residual);
     backward: data gradients with the ReLU mask + BN-backward sums in the epilogue, the BN-backward transform
     A dz + B h + C applied while gathering (MODE 2), weight gradients split over pixel chunks.
  v1 (``_building_block_v1``, :127-168): conv -> BN (statistics epilogue) -> ReLU applied by the consumer's gather,
     the block output relu(BN2(h2) + shortcut) by one elementwise pass; backward masks by the block input's ReLU in
     the conv1 data-gradient epilogue.
BN coefficients come from the shared ``cg_bn_final`` kernel (convg_aux.hip, TF moving averages included), the
optimizer is the fused multi-optimizer kernel on the same fp32 state rows.  The step is captured in one HIP graph.
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, List

import torch

from .. import ops
from ..data.datasets import IndexBatch, batch_len
from .hip_imagenet import BnFinArgs, _register as _register_cg
from .hip_resnet import advance_steps, note_step_advanced, run_captured, same_batches, upload_hyper

c_void_p, c_int, c_long = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
CMAX = 64
TP = {16: 256, 32: 128, 64: 64}  # output pixels per conv workgroup by channel tile (f32conv.hip f_tp)
WG_CHUNK = 2048   # pixels per weight-gradient work item
BAND_WGRAD = os.environ.get("DTF_F32_BAND_WGRAD", "1") == "1"  # stride-1 3x3 wgrad on the LDS row-band kernel
BAND_WG_TARGET = int(os.environ.get("DTF_F32_BAND_WG", "768"))  # workgroups per band-wgrad launch
BAND_CONV = os.environ.get("DTF_F32_BAND_CONV", "1") == "1"  # stride-1 3x3 fwd / dgrad on the row-band kernel
BAND_CONV_WG_TARGET = int(os.environ.get("DTF_F32_BAND_CONV_WG", "1024"))


class F32Args(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("x2", c_void_p), ("dy", c_void_p), ("dy2", c_void_p), ("w", c_void_p),
        ("w_mstride", c_long), ("w_off", c_long), ("y", c_void_p), ("res", c_void_p), ("xm", c_void_p),
        ("grads", c_void_p), ("g_mstride", c_long), ("g_off", c_long), ("c_in", c_void_p), ("c_dy", c_void_p),
        ("c_ep", c_void_p), ("st_out", c_void_p), ("work", c_void_p),
        ("Hi", c_int), ("Wi", c_int), ("Ci", c_int), ("Ho", c_int), ("Wo", c_int), ("Co", c_int),
        ("kh", c_int), ("kw", c_int), ("stride", c_int), ("pad", c_int), ("cmax", c_int), ("log2ci", c_int),
        ("wci", c_int), ("wrows", c_int),
    ]


class F32Ew(ctypes.Structure):
    _fields_ = [("dz", c_void_p), ("h", c_void_p), ("add", c_void_p), ("out", c_void_p), ("coef", c_void_p),
                ("coef2", c_void_p), ("img_slot", c_void_p), ("hw", c_long), ("C", c_int), ("cmax", c_int),
                ("nimg", c_long)]


class F32Sum(ctypes.Structure):
    _fields_ = [("dz", c_void_p), ("h", c_void_p), ("h2", c_void_p), ("fc", c_void_p), ("fc2", c_void_p),
                ("sums", c_void_p), ("sums2", c_void_p), ("img_slot", c_void_p), ("hw", c_int), ("C", c_int),
                ("cmax", c_int), ("pad", c_int)]


class F32Head(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("coef", c_void_p), ("img_slot", c_void_p), ("labels", c_void_p),
                ("state", c_void_p), ("s_mstride", c_long), ("w_off", c_int), ("b_off", c_int), ("feat", c_void_p),
                ("dlog", c_void_p), ("dfeat", c_void_p), ("cnt", c_void_p), ("loss", c_void_p),
                ("correct", c_void_p), ("sums", c_void_p), ("bcoef", c_void_p), ("gout", c_void_p),
                ("hw", c_int), ("C", c_int), ("ncls", c_int), ("cmax", c_int), ("train", c_int), ("pad", c_int)]


_REGISTERED = False


def _register():
    global _REGISTERED
    if _REGISTERED:
        return
    _register_cg()  # dtf_cg_bn_final
    P = ctypes.POINTER
    reg = ops.register
    reg("dtf_f32_conv", [P(F32Args), c_int, c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_f32_wgrad", [P(F32Args), c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_f32_wgrad_band", [P(F32Args), c_int, c_int, c_int, c_void_p])
    reg("dtf_f32_wgrad_band_ok", [c_int, c_int])
    reg("dtf_f32_conv_band", [P(F32Args), c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_f32_conv_band_rows", [c_int])
    reg("dtf_f32_ew", [P(F32Ew), c_int, c_void_p])
    reg("dtf_f32_bwd_sums", [P(F32Sum), c_int, c_void_p])
    reg("dtf_f32_head", [P(F32Head), c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_long, c_void_p])
    reg("dtf_f32_prep_input", [c_void_p, c_void_p, c_long, c_void_p])
    for n in ("dtf_f32_args_size", "dtf_f32_ew_size", "dtf_f32_sum_size", "dtf_f32_head_size"):
        reg(n, [])
    L = ops.lib()
    for name, args in ops._SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes = args
            fn.restype = c_int
    for st, fn in ((F32Args, "dtf_f32_args_size"), (F32Ew, "dtf_f32_ew_size"), (F32Sum, "dtf_f32_sum_size"),
                   (F32Head, "dtf_f32_head_size")):
        assert getattr(L, fn)() == ctypes.sizeof(st), "%s ABI mismatch" % st.__name__
    _REGISTERED = True


def _p(t):
    return None if t is None else t.data_ptr()


def _xcd_order(items, ng):
    """XCD-aware work order (engine/hip_imagenet.py xcd_order; DTF_CG_XCD)."""
    from .hip_imagenet import xcd_order
    return xcd_order(items, ng)


def _log2(n):
    assert n > 0 and n & (n - 1) == 0, n
    return n.bit_length() - 1


def supports(arch) -> bool:
    cfg = getattr(arch, "cfg", None)
    return (cfg is not None and cfg.image_size == 32 and not cfg.bottleneck and cfg.version in (1, 2)
            and cfg.num_classes <= 64 and cfg.final_size <= 256)


class HipResNetF32Backend:
    name = "hip"
    accepts_index_batches = False

    def __init__(self, engine):
        _register()
        if not supports(engine.arch):
            raise ValueError("the fp32 HIP backend runs CIFAR-shape building-block ResNets")
        self.e = engine
        self.dev = engine.device
        self.prog = engine.arch.prog
        self.cfg = self.prog.cfg
        cap = engine.capacity
        nb = len(self.prog.bns)
        # deterministic build (--deterministic --dtype fp32): every cross-workgroup sum -- BN statistics, BN-backward
        # sums, weight gradients, the loss -- accumulates as int64 fixed point with integer atomics (common.h
        # DTF_FIXED_ACC, as the ImageNet step): order-free, so a replay is bitwise identical; cg_det_finish folds
        # the gradient / loss accumulators into the fp32 rows before the optimizer
        self.det = bool(ops.lib().dtf_fixed_acc())
        self.acc_dtype = torch.int64 if self.det else torch.float32
        self.sums = torch.zeros(2, nb, cap, 2, CMAX, dtype=self.acc_dtype, device=self.dev)  # [fwd|bwd]
        self.gacc = torch.zeros(cap, engine.Pp, dtype=torch.int64, device=self.dev) if self.det else None
        self.loss64 = torch.zeros(cap, dtype=torch.int64, device=self.dev) if self.det else None
        self.coef = torch.zeros(2, nb, cap, 4, CMAX, dtype=torch.float32, device=self.dev)
        self.loss = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.correct = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.ident = torch.zeros(cap, 4, CMAX, dtype=torch.float32, device=self.dev)  # v1 ReLU mask (x > 0)
        self.ident[:, 0].fill_(1.0)
        self.ident[:, 3].fill_(1.0)
        self._plans: Dict[tuple, "_F32Plan"] = {}
        self.use_graph = (os.environ.get("DTF_HIP_GRAPH", "1") == "1" and os.environ.get("DTF_DEBUG", "0") != "1")

    def on_params_changed(self, slots):
        pass  # the kernels read the fp32 master rows directly

    def shadow_weights(self):
        return None

    def plan(self, slots, sizes):
        key = (tuple(slots), tuple(sizes))
        p = self._plans.get(key)
        if p is None:
            if len(self._plans) > 4:
                self._plans.clear()
            p = _F32Plan(self, list(slots), list(sizes))
            self._plans[key] = p
        return p

    def train_step(self, slots, batches, hparams, lrs):
        e = self.e
        batches = [b.materialize() if isinstance(b, IndexBatch) else b for b in batches]
        sizes = [batch_len(b) for b in batches]
        p = self.plan(slots, sizes)
        upload_hyper(e, slots, hparams, lrs)
        p.load_batch(batches)
        run_captured(p)
        note_step_advanced(e, slots)
        return p.loss_sel.clone()

    def forward_backward(self, slots, batches):
        raise RuntimeError("HipResNetF32Backend runs whole steps: use train_step")

    def train_correct(self, slots):
        return self.correct[torch.as_tensor(list(slots), dtype=torch.long, device=self.dev)]

    def eval_plan(self, slots, m):
        key = (tuple(slots), int(m))
        plans = self.__dict__.setdefault("_eval_plans", {})
        p = plans.get(key)
        if p is None:
            if len(plans) >= 4:
                plans.pop(next(iter(plans)))
            p = _F32Plan(self, list(slots), [int(m)] * len(slots), eval_mode=True)
            plans[key] = p
        return p

    @torch.no_grad()
    def infer(self, slot, x):
        p = self.eval_plan([slot], int(x.shape[0]))
        p.want_logits = True
        p.load_eval(x, torch.zeros(x.shape[0], dtype=torch.int32, device=x.device))
        p.run_eval()
        return p.logits_of(slot)

    @torch.no_grad()
    def evaluate_population(self, slots, x, y, chunk=None):
        n = int(x.shape[0])
        if n == 0 or not slots:
            return {s: 0.0 for s in slots}
        chunk = min(n, int(chunk or os.environ.get("DTF_EVAL_CHUNK", "2000")))
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


class _F32Plan:
    def __init__(self, be: HipResNetF32Backend, slots: List[int], sizes: List[int], eval_mode: bool = False):
        self.be, self.e = be, be.e
        self.eval = bool(eval_mode)
        e, dev, prog, cfg = be.e, be.dev, be.prog, be.cfg
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
        self.first_t = torch.tensor([self.first[s] for s in slots], dtype=torch.int32, device=dev)
        self.loss_sel = torch.zeros(len(slots), dtype=torch.float32, device=dev)
        H = cfg.image_size
        self.H = H
        f32 = torch.float32
        self.x_in = torch.zeros(N, H, H, cfg.in_channels, dtype=f32, device=dev)
        self.xin4 = torch.zeros(N, H, H, 4, dtype=f32, device=dev)
        self.labels = torch.zeros(N, dtype=torch.int32, device=dev)
        self.v1 = cfg.version == 1

        def act(hw_, c_):
            return torch.empty(N, hw_, hw_, c_, dtype=f32, device=dev)

        # activations: xs[i] block inputs (v2: pre-BN residual stream; v1: ReLU outputs), h1 = conv_a output,
        # h2 = conv_b output (v1 only: BN2 input), sc = projection output
        self.y0 = act(H, cfg.num_filters) if self.v1 else None
        self.xs, self.h1, self.h2, self.sc, self.geo = [act(H, cfg.num_filters)], [], [], [], []
        hw, cin = H, cfg.num_filters
        for blk in prog.blocks:
            ca = prog.convs[blk.convs[0]]
            ho = hw // blk.stride
            self.h1.append(act(ho, ca.cout))
            self.h2.append(act(ho, ca.cout) if self.v1 else None)
            self.sc.append(act(ho, ca.cout) if blk.proj is not None else None)
            self.xs.append(act(ho, ca.cout))
            self.geo.append((hw, ho, cin, ca.cout))
            hw, cin = ho, ca.cout
        self.HL, self.CL = hw, cin
        self.feat = torch.zeros(N, cin, dtype=f32, device=dev)
        self.dlog = torch.zeros(N, cfg.num_classes, dtype=f32, device=dev)
        self.dfeat = torch.zeros(N, cin, dtype=f32, device=dev)
        self._tmp: Dict[tuple, torch.Tensor] = {}
        self._keep = []
        self.launches = []
        self.graph = None
        if self.eval:
            nb = len(prog.bns)
            self.ev_coef = torch.zeros(nb, e.capacity, 4, CMAX, dtype=f32, device=dev)
            self.ev_sink = torch.zeros(e.capacity, 2, CMAX, dtype=be.acc_dtype, device=dev)
            self.ev_acc = torch.zeros(2, e.capacity, dtype=f32, device=dev)
            self.ev_loss = torch.zeros(e.capacity, dtype=be.acc_dtype, device=dev)  # summed CE (accumulator words)
            self._build_eval()
        else:
            self._build()

    # ------------------------------------------------------------------------------------------------ helpers
    def tmp(self, name, hw, c):
        key = (name, hw, c)
        t = self._tmp.get(key)
        if t is None:
            t = torch.empty(self.N, hw, hw, c, dtype=torch.float32, device=self.be.dev)
            self._tmp[key] = t
        return t

    def _add(self, fn, *args):
        self.launches.append((fn, args))

    def _hold(self, o):
        self._keep.append(o)
        return o

    def cf(self, bn):
        return self.ev_coef[bn] if self.eval else self.be.coef[0, bn]

    def cb(self, bn):
        return self.be.coef[1, bn]

    def sf(self, bn):
        return self.be.sums[0, bn]

    def sb(self, bn):
        return self.be.sums[1, bn]

    def _args(self):
        e = self.e
        a = F32Args()
        a.w, a.w_mstride = _p(e.state), e.S
        a.grads, a.g_mstride = _p(e.grads), e.Pp
        a.cmax = CMAX
        return a

    def conv(self, ci, src, out, hw_in, mode=0, c_in=None, x2=None, epi=0, res=None, xm=None, c_ep=None, st=None,
             dgrad=False):
        """Forward conv ``ci`` (src at hw_in) or its data gradient (src = dy at hw_in, the conv's output size)."""
        c = self.be.prog.convs[ci]
        stem = ci == self.be.prog.stem
        a = self._args()
        a.x, a.x2, a.y, a.res, a.xm = _p(src), _p(x2), _p(out), _p(res), _p(xm)
        a.w_off = c.off
        a.c_in, a.c_ep, a.st_out = _p(c_in), _p(c_ep), _p(st)
        a.kh = a.kw = c.k
        a.stride, a.pad = c.stride, (c.k - 1) // 2
        if not dgrad:
            a.Hi = a.Wi = hw_in
            a.Ci = 4 if stem else c.cin
            a.wci = c.cin
            a.Ho = a.Wo = hw_in // c.stride
            a.Co = c.cout
        else:
            a.Hi = a.Wi = hw_in
            a.Ci = c.cout
            a.wci = c.cout
            a.Ho = a.Wo = hw_in * c.stride
            a.Co = c.cin
        a.log2ci = _log2(a.Ci)
        L = ops.lib()
        if (BAND_CONV and not stem and c.k == 3 and c.stride == 1 and c.cin == c.cout
                and L.dtf_f32_wgrad_band_ok(c.cin, hw_in)):
            # LDS row-band kernel: weights staged once per workgroup, the operand band once for all 9 taps
            self._add_band(a, c.cin, hw_in, BAND_CONV_WG_TARGET, L.dtf_f32_conv_band_rows(c.cin),
                           L.dtf_f32_conv_band, mode, epi, int(dgrad))
            return
        tc = min(64, a.Co)
        items = []
        hwo = a.Ho * a.Wo
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            tp = TP[tc]
            for p0 in range(f * hwo, (f + n) * hwo, tp):
                for o0 in range(0, a.Co, tc):
                    items.append([s, p0, min(p0 + tp, (f + n) * hwo), o0])
        items = _xcd_order(items, -(-a.Co // tc))
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_f32_conv, ctypes.byref(a), tc, mode, epi, int(dgrad), work.shape[0])

    def _add_band(self, a, C, hw, target, rows, fn, *mode_args):
        """Work items (slot, first band, end band, tile) of a row-band kernel: bands of R = min(hw, 128 / hw) output
        rows, ``tile`` = output-row offset (conv: multiples of ``rows``) or 16-channel tile index (wgrad: rows = 1,
        C / 16 tiles); bands per item chosen for about ``target`` workgroups."""
        R = min(hw, 128 // hw)
        bpi = hw // R
        tiles = list(range(0, C, rows)) if rows > 1 else list(range(C // 16))
        total = sum(self.sizes) * bpi * len(tiles)
        chunk = max(1, int(round(total / float(target))))
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for b0 in range(f * bpi, (f + n) * bpi, chunk):
                for t in tiles:
                    items.append([s, b0, min(b0 + chunk, (f + n) * bpi), t])
        items = _xcd_order(items, len(tiles))
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(fn, ctypes.byref(a), *mode_args, work.shape[0])

    def wgrad(self, ci, x, dy, hw_in, mode_x=0, c_x=None, mode_dy=0, c_dy=None, dy2=None):
        c = self.be.prog.convs[ci]
        stem = ci == self.be.prog.stem
        a = self._args()
        a.x, a.dy, a.dy2, a.c_in, a.c_dy = _p(x), _p(dy), _p(dy2), _p(c_x), _p(c_dy)
        a.g_off = c.off
        a.Hi = a.Wi = hw_in
        a.Ci = 4 if stem else c.cin
        a.wci = c.cin
        a.Ho = a.Wo = hw_in // c.stride
        a.Co = c.cout
        a.kh = a.kw = c.k
        a.stride, a.pad = c.stride, (c.k - 1) // 2
        a.log2ci = _log2(a.Ci)
        if self.be.det:  # weight gradients into the int64 accumulator rows (folded by cg_det_finish)
            a.grads = _p(self.be.gacc)
        L = ops.lib()
        if (BAND_WGRAD and not stem and c.k == 3 and c.stride == 1 and c.cin == c.cout
                and L.dtf_f32_wgrad_band_ok(c.cin, hw_in)):
            # LDS row-band kernel: x / dy staged once per band, all 9 taps from the same tile
            self._add_band(a, c.cin, hw_in, BAND_WG_TARGET, 1, L.dtf_f32_wgrad_band, mode_x, mode_dy)
            return
        K = c.k * c.k * a.Ci
        tc = min(64, c.cout)
        items = []
        hwo = a.Ho * a.Wo
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for p0 in range(f * hwo, (f + n) * hwo, WG_CHUNK):
                for o0 in range(0, c.cout, tc):
                    for n0 in range(0, K, 64):
                        items.append([s, p0, min(p0 + WG_CHUNK, (f + n) * hwo), o0 | ((n0 // 16) << 16)])
        items = _xcd_order(items, -(-c.cout // tc) * -(-K // 64))
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_f32_wgrad, ctypes.byref(a), tc, mode_x, mode_dy, work.shape[0])

    def bn_final(self, bn, hw, backward):
        e = self.e
        b = self.be.prog.bns[bn]
        a = BnFinArgs()
        a.state, a.s_mstride = _p(e.state), e.S
        a.sums = _p(self.sb(bn) if backward == 1 else self.sf(bn))
        a.coef = _p(self.cb(bn) if backward == 1 else self.cf(bn))
        a.fcoef = _p(self.cf(bn))
        a.grads, a.g_mstride = _p(e.grads), e.Pp
        a.slots, a.cnt = _p(self.slots_t), _p(self.cnt)
        a.gamma_off, a.beta_off, a.run_off = b.gamma_off, b.beta_off, 3 * e.Pp + b.run_off
        a.C, a.hw, a.cmax = b.c, hw * hw, CMAX
        self._hold(a)
        self._add(ops.lib().dtf_cg_bn_final, ctypes.byref(a), int(backward), len(self.slots))

    def ew(self, which, h, out, coef, hw, C, dz=None, add=None, coef2=None):
        """which 0: out = A dz + B h + C (+ add); 1: relu(h s + t); 2: relu(BN(h) + BN2(add) | add)."""
        a = F32Ew()
        a.dz, a.h, a.add, a.out, a.coef, a.coef2 = _p(dz), _p(h), _p(add), _p(out), _p(coef), _p(coef2)
        a.img_slot, a.hw, a.C, a.cmax, a.nimg = _p(self.img_slot), hw * hw, C, CMAX, self.N
        self._hold(a)
        self._add(ops.lib().dtf_f32_ew, ctypes.byref(a), which)

    def bwd_sums(self, dz, h, bn, hw, C, h2=None, bn2=None):
        a = F32Sum()
        a.dz, a.h, a.h2 = _p(dz), _p(h), _p(h2)
        a.fc, a.sums = _p(self.cf(bn)), _p(self.sb(bn))
        if bn2 is not None:
            a.fc2, a.sums2 = _p(self.cf(bn2)), _p(self.sb(bn2))
        a.img_slot, a.hw, a.C, a.cmax = _p(self.img_slot), hw * hw, C, CMAX
        self._hold(a)
        self._add(ops.lib().dtf_f32_bwd_sums, ctypes.byref(a), self.N)

    def _head_args(self, train):
        e, prog, cfg = self.e, self.be.prog, self.be.cfg
        h = F32Head()
        h.x, h.img_slot, h.labels = _p(self.xs[-1]), _p(self.img_slot), _p(self.labels)
        h.coef = None if self.v1 else _p(self.cf(prog.final_bn))
        h.state, h.s_mstride, h.w_off, h.b_off = _p(e.state), e.S, prog.dense_w_off, prog.dense_b_off
        h.feat, h.dlog, h.dfeat, h.cnt = _p(self.feat), _p(self.dlog), _p(self.dfeat), _p(self.cnt)
        if train:
            h.loss = _p(self.be.loss64 if self.be.det else self.be.loss)
            h.correct = _p(self.be.correct)
        else:
            h.loss, h.correct = _p(self.ev_loss), _p(self.ev_acc[0])
        if not self.v1 and train:
            h.sums, h.bcoef = _p(self.sb(prog.final_bn)), _p(self.cb(prog.final_bn))
        h.hw, h.C, h.ncls, h.cmax, h.train = self.HL * self.HL, self.CL, cfg.num_classes, CMAX, int(train)
        return self._hold(h)

    def head(self, h, which, gout=None):
        if gout is not None:
            h2 = F32Head()
            ctypes.memmove(ctypes.addressof(h2), ctypes.addressof(h), ctypes.sizeof(F32Head))
            h2.gout = _p(gout)
            h = self._hold(h2)
        e = self.e
        self._add(ops.lib().dtf_f32_head, ctypes.byref(h), which, self.N, _p(self.slots_t), _p(self.first_t),
                  len(self.slots), _p(e.grads), e.Pp)

    # ------------------------------------------------------------------------------------------------ program
    def _forward(self, train):
        be, prog, cfg = self.be, self.be.prog, self.be.cfg
        H = self.H
        sink = None if train else self.ev_sink
        self._add(ops.lib().dtf_f32_prep_input, _p(self.x_in), _p(self.xin4), self.N * H * H)
        nblk = len(prog.blocks)
        if self.v1:
            sbn = prog.stem_bn
            self.conv(prog.stem, self.xin4, self.y0, H, epi=4, st=self.sf(sbn) if train else sink)
            if train:
                self.bn_final(sbn, H, False)
            self.ew(1, self.y0, self.xs[0], self.cf(sbn), H, cfg.num_filters)
            for i, blk in enumerate(prog.blocks):
                hi, ho, cin, c = self.geo[i]
                b1, b2 = blk.bns
                ca, cbv = blk.convs
                x = self.xs[i]
                if blk.proj is not None:
                    self.conv(blk.proj, x, self.sc[i], hi, epi=4, st=self.sf(blk.proj_bn) if train else sink)
                self.conv(ca, x, self.h1[i], hi, epi=4, st=self.sf(b1) if train else sink)
                if train:
                    self.bn_final(b1, ho, False)
                self.conv(cbv, self.h1[i], self.h2[i], ho, mode=1, c_in=self.cf(b1), epi=4,
                          st=self.sf(b2) if train else sink)
                if train:
                    self.bn_final(b2, ho, False)
                    if blk.proj is not None:
                        self.bn_final(blk.proj_bn, ho, False)
                if blk.proj is not None:
                    self.ew(2, self.h2[i], self.xs[i + 1], self.cf(b2), ho, c, add=self.sc[i],
                            coef2=self.cf(blk.proj_bn))
                else:
                    self.ew(2, self.h2[i], self.xs[i + 1], self.cf(b2), ho, c, add=x)
            return
        first_bn = prog.blocks[0].bns[0]
        self.conv(prog.stem, self.xin4, self.xs[0], H, epi=4, st=self.sf(first_bn) if train else sink)
        for i, blk in enumerate(prog.blocks):
            hi, ho, cin, c = self.geo[i]
            b1, b2 = blk.bns
            ca, cbv = blk.convs
            x = self.xs[i]
            nxt = prog.blocks[i + 1].bns[0] if i + 1 < nblk else prog.final_bn
            if train:
                self.bn_final(b1, hi, False)
            if blk.proj is not None:
                self.conv(blk.proj, x, self.sc[i], hi, mode=1, c_in=self.cf(b1), epi=0)
            self.conv(ca, x, self.h1[i], hi, mode=1, c_in=self.cf(b1), epi=4, st=self.sf(b2) if train else sink)
            if train:
                self.bn_final(b2, ho, False)
            self.conv(cbv, self.h1[i], self.xs[i + 1], ho, mode=1, c_in=self.cf(b2), epi=5,
                      res=self.sc[i] if blk.proj is not None else x, st=self.sf(nxt) if train else sink)
        if train:
            self.bn_final(prog.final_bn, self.HL, False)

    def _build(self):
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        self._add("zero", be.sums)
        self._add("zero", be.loss)
        self._add("zero", be.correct)
        self._forward(True)
        H, HL, CL = self.H, self.HL, self.CL
        hd = self._head_args(True)
        self.head(hd, 0)
        self.head(hd, 1)
        g = self.tmp("gA" if len(prog.blocks) % 2 == 0 else "gB", HL, CL)
        if not self.v1:
            self.head(hd, 2)
            self.bn_final(prog.final_bn, HL, True)
        self.head(hd, 3, gout=g)  # v2: final BN backward; v1: masked by the last block's ReLU
        for i in range(len(prog.blocks) - 1, -1, -1):
            blk = prog.blocks[i]
            hi, ho, cin, c = self.geo[i]
            b1, b2 = blk.bns
            ca, cbv = blk.convs
            x, h1 = self.xs[i], self.h1[i]
            gnext = self.tmp("gA" if i % 2 == 0 else "gB", hi, cin)
            if self.v1:
                # g = dL/d(BN2(h2) + shortcut), already ReLU-masked
                h2, pbn = self.h2[i], blk.proj_bn
                self.bwd_sums(g, h2, b2, ho, c, h2=self.sc[i] if pbn is not None else None, bn2=pbn)
                self.bn_final(b2, ho, True)
                if pbn is not None:
                    self.bn_final(pbn, ho, True)
                dz1 = self.tmp("dz1", ho, c)
                self.conv(cbv, g, dz1, ho, mode=2, x2=h2, c_in=self.cb(b2), epi=6, xm=h1, c_ep=self.cf(b1),
                          st=self.sb(b1), dgrad=True)
                self.wgrad(cbv, h1, g, ho, mode_x=1, c_x=self.cf(b1), mode_dy=2, c_dy=self.cb(b2), dy2=h2)
                self.bn_final(b1, ho, True)
                res = g
                if blk.proj is not None:
                    res = self.tmp("pd", hi, cin)
                    self.conv(blk.proj, g, res, ho, mode=2, x2=self.sc[i], c_in=self.cb(pbn), epi=0, dgrad=True)
                    self.wgrad(blk.proj, x, g, hi, mode_dy=2, c_dy=self.cb(pbn), dy2=self.sc[i])
                # conv_a data gradient + shortcut gradient, masked by the block input's ReLU
                self.conv(ca, dz1, gnext, ho, mode=2, x2=h1, c_in=self.cb(b1), epi=3, res=res, xm=x,
                          c_ep=be.ident, dgrad=True)
                self.wgrad(ca, x, dz1, hi, mode_dy=2, c_dy=self.cb(b1), dy2=h1)
            else:
                # g = dL/dxs[i + 1]
                dz2 = self.tmp("dz2", ho, c)
                self.conv(cbv, g, dz2, ho, epi=6, xm=h1, c_ep=self.cf(b2), st=self.sb(b2), dgrad=True)
                self.bn_final(b2, ho, True)
                self.wgrad(cbv, h1, g, ho, mode_x=1, c_x=self.cf(b2))
                pd = None
                if blk.proj is not None:
                    pd = self.tmp("pd", hi, cin)
                    self.conv(blk.proj, g, pd, ho, epi=0, dgrad=True)
                    self.wgrad(blk.proj, x, g, hi, mode_x=1, c_x=self.cf(b1))
                dz1 = self.tmp("dz1", hi, cin)
                self.conv(ca, dz2, dz1, ho, mode=2, x2=h1, c_in=self.cb(b2), epi=7 if pd is not None else 6,
                          res=pd, xm=x, c_ep=self.cf(b1), st=self.sb(b1), dgrad=True)
                self.wgrad(ca, x, dz2, hi, mode_x=1, c_x=self.cf(b1), mode_dy=2, c_dy=self.cb(b2), dy2=h1)
                self.bn_final(b1, hi, True)
                self.ew(0, x, gnext, self.cb(b1), hi, cin, dz=dz1, add=g if blk.proj is None else None)
            g = gnext
        if self.v1:
            sbn = prog.stem_bn
            self.bwd_sums(g, self.y0, sbn, H, cfg.num_filters)
            self.bn_final(sbn, H, True)
            dy0 = self.tmp("dy0", H, cfg.num_filters)
            self.ew(0, self.y0, dy0, self.cb(sbn), H, cfg.num_filters, dz=g)
            g = dy0
        self.wgrad(prog.stem, self.xin4, g, H)
        if be.det:
            from .hip_imagenet import _register as _reg_cg
            _reg_cg()  # dtf_cg_det_finish signature
            self._add(ops.lib().dtf_cg_det_finish, _p(be.gacc), _p(e.grads), e.Pp, e.Pp, _p(self.slots_t),
                      len(self.slots), _p(be.loss64), _p(be.loss))
        self._add("optim", None)
        self._add("step", None)

    def _build_eval(self):
        prog = self.be.prog
        for b in range(len(prog.bns)):
            self.bn_final(b, 1, 2)
        self._forward(False)
        self.head(self._head_args(False), 0)

    # ------------------------------------------------------------------------------------------------ execution
    def load_batch(self, batches):
        if same_batches(self, batches):
            return
        off = 0
        for (x, y) in batches:
            n = x.shape[0]
            self.x_in[off:off + n].copy_(x.reshape(n, *self.x_in.shape[1:]), non_blocking=True)
            self.labels[off:off + n].copy_(y, non_blocking=True)
            off += n

    def load_eval(self, x, y):
        m, k = x.shape[0], len(self.slots)
        shp = tuple(self.x_in.shape[1:])
        self.x_in.view(k, m, *shp).copy_(x.reshape(1, m, *shp).expand(k, *([-1] * (len(shp) + 1))))
        self.labels.view(k, m).copy_(y.reshape(1, m).expand(k, -1))

    def logits_of(self, slot):
        """Eval logits of ``slot``'s images from the head's features (dense on the host side of the graph)."""
        e, prog, cfg = self.e, self.be.prog, self.be.cfg
        i0, n = self.first[slot], self.sizes[self.slots.index(slot)]
        W = e.state[slot, prog.dense_w_off:prog.dense_w_off + cfg.num_classes * self.CL].view(cfg.num_classes,
                                                                                               self.CL)
        b = e.state[slot, prog.dense_b_off:prog.dense_b_off + cfg.num_classes]
        return self.feat[i0:i0 + n] @ W.t() + b

    def run_eval(self):
        self._run_eager()

    def _run_eager(self):
        e = self.e
        st = ops.stream()
        for fn, args in self.launches:
            if fn == "zero":
                args[0].zero_()
            elif fn == "optim":
                e.dp_sync_grads(self.slots)
                ops.fused_optimizer(e.state, e.grads, e.hyper, e.Pp, e.P, e.n_reg, shadow=None, zero_grads=True)
            elif fn == "step":
                advance_steps(e, self.slots_long, self.slots_t, self.be.loss, self.loss_sel)
            else:
                err = fn(*args, st)
                if err != 0:
                    raise RuntimeError("kernel launch %s failed with %d" % (getattr(fn, "__name__", fn), err))
