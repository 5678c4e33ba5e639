"""Population-batched fp32 ImageNet-shape bottleneck ResNet (v1 / v2) training step: ``--dtype fp32 --model imagenet``.

The reference trains in fp32 by default (``resnet/official/utils/flags/_performance.py:30-33``); the bf16 step
(engine/hip_imagenet.py) is the throughput path.  This one runs the SAME program -- ``_ImageNetPlan``'s v1 / v2
forward and backward launch lists (reference ``resnet_model.py:215-320, 504-525``) -- with every tensor, weight and
accumulation in fp32, by overriding the plan's kernel vocabulary:

  convolutions       f32conv.hip generic kernels (v_mfma_f32_16x16x4_f32): 7x7/2 stem on the 4-channel padded
                     input, 1x1 / 3x3 / strided forward with BN-statistic epilogues, transposed-gather data
                     gradients with ReLU-mask + BN-backward-sum epilogues, split-K weight gradients
  dense layer        the same kernels as a 1x1 conv over the GAP features, the class dimension padded to 1024
                     (F32Args.wrows keeps the padding off the 1001-row weight matrix)
  BN apply / sums    f32conv.hip f32_ew (relu(BN), BN-backward apply, v1 relu(BN + shortcut)), f32_bwd_sums
  max-pool, GAP,     f32net.hip (fp32 twins of convg_aux.hip's kernels)
  softmax CE
  BN finalize        convg_aux.hip cg_bn_final (already fp32), the fused optimizer on the fp32 rows (no shadow)

The deterministic build accumulates every cross-workgroup sum as int64 fixed point (common.h DTF_FIXED_ACC), as
the bf16 step does.  The step is captured in one HIP graph per batch composition.
"""

from __future__ import annotations

import ctypes
import os

import torch

from .. import ops
from .hip_f32 import F32Args, F32Ew, F32Sum, TP, WG_CHUNK, _register as _register_f32
from .hip_imagenet import (CMAX, NPAD_CLS, GapArgs, HipImageNetBackend, _ImageNetPlan, _log2,
                           _register as _register_cg)

c_void_p, c_int, c_long = ctypes.c_void_p, ctypes.c_int, ctypes.c_long

_REGISTERED = False


def _register():
    global _REGISTERED
    if _REGISTERED:
        return
    _register_cg()
    _register_f32()
    P = ctypes.POINTER
    ops.register("dtf_f32_maxpool", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                     c_int, c_int, c_int, c_void_p])
    ops.register("dtf_f32_gap", [P(GapArgs), c_int, c_int, c_void_p])
    ops.register("dtf_f32_softmax_ce", [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p,
                                        c_long, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p])
    ops.register("dtf_f32_gap_args_size", [])
    L = ops.lib()
    for name, args in ops._SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes = args
            fn.restype = c_int
    assert L.dtf_f32_gap_args_size() == ctypes.sizeof(GapArgs), "F32GapArgs ABI mismatch"
    _REGISTERED = True


def _p(t):
    return None if t is None else t.data_ptr()


def supports(arch) -> bool:
    cfg = getattr(arch, "cfg", None)
    return (cfg is not None and cfg.bottleneck and cfg.version in (1, 2) and cfg.in_channels == 3
            and cfg.first_pool_size == 3 and cfg.first_pool_stride == 2 and cfg.kernel_size == 7
            and cfg.conv_stride == 2 and cfg.image_size % 32 == 0 and cfg.num_classes <= NPAD_CLS)


class HipImageNetF32Backend(HipImageNetBackend):
    """fp32 bottleneck-ResNet step: the bf16 backend's drivers (train_step, eval, infer) over fp32 plans."""

    def __init__(self, engine):
        _register()
        if not supports(engine.arch):
            raise ValueError("the fp32 HIP ImageNet backend runs the v1 / v2 bottleneck ImageNet configurations")
        self.e = engine
        self.dev = engine.device
        prog = engine.arch.prog
        self.prog, self.cfg = prog, prog.cfg
        cap = engine.capacity
        self.shadow = None  # every kernel reads the fp32 master rows
        self.ncls = self.cfg.num_classes
        nb = len(prog.bns)
        self.det = bool(ops.lib().dtf_fixed_acc())
        self.half = False
        self.loss_scale = 1.0
        self.acc_dtype = torch.int64 if self.det else torch.float32
        self.sums = torch.zeros(2, nb, cap, 2, CMAX, dtype=self.acc_dtype, device=self.dev)   # [fwd|bwd]
        self.coef = torch.zeros(2, nb, cap, 4, CMAX, dtype=torch.float32, device=self.dev)   # [fwd|bwd]
        self.loss = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.correct = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        if self.det:
            self.gacc = torch.zeros(cap, engine.Pp, dtype=torch.int64, device=self.dev)
            self.loss64 = torch.zeros(cap, dtype=torch.int64, device=self.dev)
        self.acc_grads = self.gacc if self.det else engine.grads
        self.acc_loss = self.loss64 if self.det else self.loss
        self.v1 = self.cfg.version == 1
        self.s2d = False  # the fp32 stem runs the 7x7/2 gather on the 4-channel padded input
        # identity coefficients (scale 1, shift 0, mean 0, inv 1): the v1 ReLU mask by the block input, and the
        # forward statistics of the pooled stem output through f32_bwd_sums (dz = h = x)
        self.ident = torch.zeros(cap, 4, CMAX, dtype=torch.float32, device=self.dev)
        self.ident[:, 0].fill_(1.0)
        self.ident[:, 3].fill_(1.0)
        self._plans = {}
        self.use_graph = (os.environ.get("DTF_HIP_GRAPH", "1") == "1" and os.environ.get("DTF_DEBUG", "0") != "1")

    def on_params_changed(self, slots):
        pass

    def shadow_weights(self):
        return None


class _ImageNetF32Plan(_ImageNetPlan):
    FOLD1_OK = False  # (the fp32 conv kernels are not exercised with the read-once BN1 fold)
    COMPACT_PD_OK = False  # (nor with the compact stride-2 projection gradient: f32conv has no EPI bit 8)
    GFOLD_OK = False  # (nor with the block-input gradient applied by conv3's data gradient: no f32conv MODE 3)

    def _act_dtype(self):
        return torch.float32

    def _stem_input_shape(self, N, H):
        return (N, H, H, 4)  # f32conv gathers 4-channel chunks: the 3-channel input padded to 4

    # ---------------------------------------------------------------------------------------- convolutions
    def _f32args(self, w_off, Hi, Ci, wci, Ho, Co, k, stride, pad):
        e = self.e
        a = F32Args()
        a.w, a.w_mstride, a.w_off = _p(e.state), e.S, w_off
        a.grads, a.g_mstride, a.g_off = _p(self.be.acc_grads), e.Pp, w_off
        a.Hi = a.Wi = Hi
        a.Ho = a.Wo = Ho
        a.Ci, a.wci, a.Co = Ci, wci, Co
        a.kh = a.kw = k
        a.stride, a.pad = stride, pad
        a.cmax = CMAX
        a.log2ci = _log2(Ci)
        assert Ci >= 4 and Co % 4 == 0, (Ci, Co)
        return a

    def _conv_launch(self, a, src, out, mode, epi, dgrad):
        N = self.N
        assert src.numel() == N * a.Hi * a.Wi * a.Ci and out.numel() == N * a.Ho * a.Wo * a.Co, \
            (tuple(src.shape), tuple(out.shape), a.Hi, a.Ci, a.Ho, a.Co)
        a.x, a.y = _p(src), _p(out)
        tc = min(64, a.Co)
        assert a.Co % tc == 0
        hwo = a.Ho * a.Wo
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for p0 in range(f * hwo, (f + n) * hwo, TP[tc]):
                for o0 in range(0, a.Co, tc):
                    items.append([s, p0, min(p0 + TP[tc], (f + n) * hwo), o0])
        items = self._xcd_order(items, a.Co // tc)
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_f32_conv, ctypes.byref(a), tc, mode, epi, int(dgrad), work.shape[0])

    def conv(self, ci, src, out, hw_in, mode=0, c_in=None, x2=None, epi=0, res=None, xm=None, c_ep=None, st=None,
             dgrad=False, compact=False):
        assert not compact and not (epi & 8), "the fp32 plan keeps the full-resolution projection gradient"
        be = self.be
        c = be.prog.convs[ci]
        stem = ci == be.prog.stem
        pad = (c.k - 1) // 2  # f32conv takes the FORWARD geometry for both directions
        if not dgrad:
            a = self._f32args(c.off, hw_in, 4 if stem else c.cin, c.cin, (hw_in + c.stride - 1) // c.stride, c.cout,
                              c.k, c.stride, pad)
        else:
            a = self._f32args(c.off, hw_in, c.cout, c.cout, hw_in * c.stride, c.cin, c.k, c.stride, pad)
        a.x2, a.res, a.xm = _p(x2), _p(res), _p(xm)
        a.c_in, a.c_ep, a.st_out = _p(c_in), _p(c_ep), _p(st)
        self._conv_launch(a, src, out, mode, epi, dgrad)

    def wgrad(self, ci, x, dy, hw_in, mode_x=0, c_x=None, mode_dy=0, c_dy=None, dy2=None):
        be = self.be
        c = be.prog.convs[ci]
        stem = ci == be.prog.stem
        hw_out = (hw_in + c.stride - 1) // c.stride
        a = self._f32args(c.off, hw_in, 4 if stem else c.cin, c.cin, hw_out, c.cout, c.k, c.stride, (c.k - 1) // 2)
        a.dy, a.dy2, a.c_in, a.c_dy = _p(dy), _p(dy2), _p(c_x), _p(c_dy)
        self._wgrad_launch(a, x, mode_x, mode_dy)

    def _wgrad_launch(self, a, x, mode_x, mode_dy):
        N = self.N
        assert x.numel() == N * a.Hi * a.Wi * a.Ci
        a.x = _p(x)
        K = a.kh * a.kw * a.Ci
        tc = min(64, a.Co)
        hwo = a.Ho * a.Wo
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for p0 in range(f * hwo, (f + n) * hwo, WG_CHUNK):
                for o0 in range(0, a.Co, tc):
                    for n0 in range(0, K, 64):
                        items.append([s, p0, min(p0 + WG_CHUNK, (f + n) * hwo), o0 | ((n0 // 16) << 16)])
        items = self._xcd_order(items, (a.Co // tc) * -(-K // 64))
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_f32_wgrad, ctypes.byref(a), tc, mode_x, mode_dy, work.shape[0])

    # ---------------------------------------------------------------------------------------- elementwise
    def ew(self, fn, h, out, coef, hw, C, dz=None, add=None):
        """fn: the bf16 program's dtf_cg_bn_relu_apply (-> f32_ew 1: relu(h s + t)) or dtf_cg_bn_bwd_apply
        (-> f32_ew 0: A dz + B h + C [+ add])."""
        which = 1 if "relu" in getattr(fn, "__name__", "") else 0
        self._ew(which, h, out, coef, hw, C, dz=dz, add=add)

    def _ew(self, which, h, out, coef, hw, C, dz=None, add=None, coef2=None):
        a = F32Ew()
        a.dz, a.h, a.add, a.out, a.coef, a.coef2 = _p(dz), _p(h), _p(add), _p(out), _p(coef), _p(coef2)
        a.img_slot, a.hw, a.C, a.cmax, a.nimg = _p(self.img_slot), hw * hw, C, CMAX, self.N
        self._hold(a)
        self._add(ops.lib().dtf_f32_ew, ctypes.byref(a), which)

    def bn_add_relu(self, h, s, out, coef_h, coef_s, hw, C):
        self._ew(2, h, out, coef_h, hw, C, add=s, coef2=coef_s)

    def bwd_sums(self, dz, h, bn, hw, C, h2=None, bn2=None):
        a = F32Sum()
        a.dz, a.h, a.h2 = _p(dz), _p(h), _p(h2)
        a.fc, a.sums = _p(self.cf(bn)), _p(self.sb(bn))
        if bn2 is not None:
            a.fc2, a.sums2 = _p(self.cf(bn2)), _p(self.sb(bn2))
        a.img_slot, a.hw, a.C, a.cmax = _p(self.img_slot), hw * hw, C, CMAX
        self._hold(a)
        self._add(ops.lib().dtf_f32_bwd_sums, ctypes.byref(a), self.N)

    # ---------------------------------------------------------------------------------------- vocabulary
    def prep_weights(self):
        pass  # no padded / bf16 copies: the convs read the fp32 rows

    def prep_input(self):
        assert self.be.cfg.in_channels == 3
        self._add(ops.lib().dtf_f32_prep_input, _p(self.x_in), _p(self.xin8), self.N * self.H * self.H)

    def maxpool(self, x, y, H1, H2):
        self._add(ops.lib().dtf_f32_maxpool, _p(x), _p(y), _p(self.am0), None, None, self.N, H1, H1, H2, H2,
                  self.be.cfg.num_filters, 0)

    def maxpool_bwd(self, g, dx, H1, H2):
        self._add(ops.lib().dtf_f32_maxpool, None, None, _p(self.am0), _p(g), _p(dx), self.N, H1, H1, H2, H2,
                  self.be.cfg.num_filters, 1)

    def chan_stats(self, x, sums, hw, C):
        """Forward statistics (sum x, sum x^2) of a tensor no conv produced: f32_bwd_sums with dz = h = x, identity
        coefficients, statistics scale (pad = 1)."""
        a = F32Sum()
        a.dz, a.h, a.h2 = _p(x), _p(x), None
        a.fc, a.sums = _p(self.be.ident), _p(sums)
        a.img_slot, a.hw, a.C, a.cmax, a.pad = _p(self.img_slot), hw, C, CMAX, 1
        self._hold(a)
        self._add(ops.lib().dtf_f32_bwd_sums, ctypes.byref(a), self.N)

    def gap(self, g, which):
        self._add(ops.lib().dtf_f32_gap, ctypes.byref(g), which, self.N)

    def dense_head(self, train):
        """logits = feat W^T as a 1x1 conv (classes padded to NPAD_CLS; wrows = the real class count), softmax CE;
        training: dfeat = dlogits W (1x1 data gradient), dW += dlogits^T feat (1x1 weight gradient)."""
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        L = ops.lib()
        C = cfg.final_size
        a = self._f32args(prog.dense_w_off, 1, C, C, 1, NPAD_CLS, 1, 1, 0)
        a.wrows = be.ncls
        self._conv_launch(a, self.feat, self.logits, 0, 0, False)
        if not train:
            self._add(L.dtf_f32_softmax_ce, _p(self.logits), NPAD_CLS, be.ncls, _p(self.labels), _p(self.img_slot),
                      _p(e.state), e.S, prog.dense_b_off, None, e.Pp, _p(self.cnt), _p(self.ev_loss),
                      _p(self.ev_acc[0]), None, self.N)
            return
        self._add(L.dtf_f32_softmax_ce, _p(self.logits), NPAD_CLS, be.ncls, _p(self.labels), _p(self.img_slot),
                  _p(e.state), e.S, prog.dense_b_off, _p(be.acc_grads), e.Pp, _p(self.cnt), _p(be.acc_loss),
                  _p(be.correct), _p(self.dlog), self.N)
        d = self._f32args(prog.dense_w_off, 1, NPAD_CLS, NPAD_CLS, 1, C, 1, 1, 0)
        d.wrows = be.ncls
        self._conv_launch(d, self.dlog, self.dfeat, 0, 0, True)
        w = self._f32args(prog.dense_w_off, 1, C, C, 1, NPAD_CLS, 1, 1, 0)
        w.wrows = be.ncls
        w.dy = _p(self.dlog)
        self._wgrad_launch(w, self.feat, 0, 0)


HipImageNetF32Backend._plan_cls = _ImageNetF32Plan
