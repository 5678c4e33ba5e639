"""Population-batched ImageNet-shape ResNet (v2 bottleneck) training step on hand-written gfx950 kernels.

Architecture (SURVEY.md C12'; reference block ``_bottleneck_block_v2``, ``resnet/resnet_model.py:267-320``):
7x7/2 stem (3 -> 64, no BN in v2), 3x3/2 'SAME' max-pool, bottleneck stages [3, 4, 6, 3] with strides
[1, 2, 2, 2] (BN1+ReLU -> 1x1 -> BN2+ReLU -> 3x3/s -> BN3+ReLU -> 1x1, + shortcut; the first block of a
stage projects the PRE-ACTIVATED input with a 1x1/s conv), final BN+ReLU, global average pool, dense.

Every conv is one ``convg`` launch (ops/csrc/convg.hip): the producing BN+ReLU is applied while the gathered
operand is staged (forward), the BN statistics of the output are reduced in the epilogue, and the residual is
added there.  Backward: the data gradient runs the same kernel on flipped/transposed weights (stride 2:
transposed gather), with the next BN's backward transform on load and ReLU-mask + BN-backward reductions in
the epilogue; weight gradients are split-K implicit GEMMs (k = pixels) with atomics into the member's row.
Per-member BN coefficients (forward scale/shift/mean/inv, backward A/B/C) are finalised by tiny kernels
between the convs (``convg_aux.hip``), which also update the running statistics / accumulate dgamma, dbeta.
The dense layer is the grouped bf16 GEMM (gemm.hip) with softmax-CE in between.  The whole step is captured
into one HIP graph per batch composition.  Eval (``evaluate_population``) runs the same forward kernels for every
member at once with BN coefficients from the moving statistics.
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, List

import torch

from .. import ops
from ..data.datasets import IndexBatch, batch_len
from .hip_resnet import advance_steps, run_captured, note_step_advanced, same_batches, upload_hyper

c_void_p, c_int, c_long, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
CMAX = 2048
NPAD_CLS = 1024
# k depth per LDS stage of the convg forward / data-gradient kernel (32 or 64)
_CG_BK = 32  # K depth of one LDS stage of the forward / dgrad tiles
# weight gradient: pixels per k-step (32 or 64), target items per launch, minimum pixels per split-K chunk
_CG_WPK = 32
_CG_WO64 = True
_CG_WIDE = True  # wide-column 3x3 weight-gradient tiles
_CG_WIDE128 = os.environ.get("DTF_CG_WIDE128", "1") == "1"  # 128-row wide wgrad tiles (0: 64-row: twice the items, half the splits)
_CG_WIDE7 = True  # one 64 x 416 tile for the 7x7 stem
_CG_WIDE1 = True  # the wide tiles for 1x1 convs with Ci % 256 == 0
_CG_TP256_128 = os.environ.get("DTF_CG_TP256_128", "1") == "1"  # 128 x 256 tiles (2 x 2 waves of 64 x 128)
_CG_TP256 = True  # 256-pixel forward / dgrad tiles for 64-channel outputs
# v_mfma_f32_32x32x16_bf16 tiles for the plain-A forward convolutions with 128-channel tiles (1x1 / strided / 7x7-stage
# convs with C_out >= 128): 32 x 32 MFMA tiles of each wave's 64 x 128 block (convg_fwd_kernel M32)
_CG_M32 = os.environ.get("DTF_CG_M32", "0") == "1"
# space-to-depth stem: the 7x7/2 conv over the 3-channel image as a 4x4/1 conv over 2x2 pixel blocks (12 of 16
# channels real): K = 256 instead of 7 x 7 x 8 = 392 padded, stride 1, half the input bytes (cg_prep_input_s2d,
# cg_weight_prep s2d rows, convg_wgrad_wide cin_real = -3 remaps the weight gradient onto the 7x7x3 kernel)
_CG_S2D = os.environ.get("DTF_CG_S2D", "1") == "1"
# stride-1 3x3 weight gradients from LDS-resident row bands (convg_wgrad_t3_kernel): image width -> rows per band;
# items per launch (each adds one 64 x 288 fp32 tile into the gradient row)
_CG_WGT3 = {56: 4, 28: 7, 14: 14} if os.environ.get("DTF_CG_WGT3", "1") == "1" else {}
_CG_WGT3_TARGET = int(os.environ.get("DTF_CG_WGT3_TARGET", "512"))
# the s2d stem forward from 2-row bands (convg_stem_s2d_kernel) at 224 x 224; workgroups per launch
_CG_STEM_BAND = os.environ.get("DTF_CG_STEM_BAND", "1") == "1"
_CG_STEM_WG = int(os.environ.get("DTF_CG_STEM_WG", "2048"))
_CG_WPK_WO64 = 32  # pixels per k-step of the 64-row tiles
# stride-1 3x3 forward / data gradient with LDS-resident input rows (convg_t3_kernel): image width -> rows per tile
_CG_T3 = {56: 8, 28: 7, 14: 14}  # must match dtf_convg_t3 (rows divide the image height)
# convg_t3 forward: bit 0 = LDS-staged weights (the pre-round-4 form) instead of direct fragment loads (A/B switch)
# Folded forward (v2 training): every BN+ReLU is applied while the consuming convolution -- and, in the backward, its
# weight gradient -- stages its input (convg MODE 1, convg_t3 XF, convg_wgrad_wide MX 1), so no relu(BN(.)) tensor
# (ax / a1 / a2) is materialised: 3 elementwise passes per block fewer
CG_FOLD = os.environ.get("DTF_CG_FOLD", "0") == "1"
# selective fold: only BN2 + ReLU (conv1 output -> the 3x3 conv2) is applied by its consumers -- conv2's forward
# (convg_t3 XF / convg MODE 1 when strided) and weight gradient (row-band MX 1 / wide MX 1) -- so the a1 = relu(BN2(h1))
# tensor is never written (each element is transformed once per 32-channel chunk and output tile)
CG_FOLD2 = os.environ.get("DTF_CG_FOLD2", "0") == "1"  # measured +2.7 ms: profiles/r5_imagenet_fold2_ab.log
# read-once fold: BN1 + ReLU applied by conv1 (the 1x1 reduce) only where that consumer transforms each input element
# exactly once -- blocks without a projection (the block input's only forward consumer is conv1) whose conv1 runs a
# single output-channel tile (Co <= 128: every workgroup holds all output channels of its pixels) -- and by conv1's
# weight gradient (wide 1x1 tiles, MX 1), so relu(BN1(x)) is never written for those blocks
# ... up to this conv1 width (128: one output-channel tile; 256 / 512 re-transform each element 2 / 4 times).  With the
# wide wgrad's coefficients read once per kernel, 256 measured 70.2 vs 70.7 ms (128) and 70.4 ms (512)
# (profiles/r6_imagenet_fold_xcol_ab.log)
CG_FOLD1_MAXC = int(os.environ.get("DTF_CG_FOLD1_MAXC", "256"))
# stride-2 projection data gradient computed / stored compact at the dy resolution (3/4 of its full-resolution
# tensor is zeros) and added by conv1's epilogue at even pixels
CG_COMPACT_PD = os.environ.get("DTF_CG_COMPACT_PD", "1") == "1"
CG_CLASS_LPT = os.environ.get("DTF_CG_CLASS_LPT", "0") == "1"  # stride-2 3x3 data gradient: heavy parity class first
CG_FOLD1 = os.environ.get("DTF_CG_FOLD1", "1") == "1"  # 73.24 -> 72.87 ms at pop 8 (profiles/r6_imagenet_fold1_ab.log)
# backward fold of the block-input gradient: g = BN1-backward(dz1, x) [+ g of the next block] is computed by its first
# consumer -- the previous block's conv3 data gradient (a stride-1 1x1 over g with one output-channel tile when that
# block's width f <= this: convg MODE 3) -- while it stages g, and stored from there (xout), instead of a standalone
# apply pass that conv3's data gradient then re-reads (0: off).  Numerics and det replay pass (bitwise the same
# values as the standalone pass), but 64 / 128 measured +0.2 / +0.5 ms: the conv's one-ahead pipeline streams the
# three extra operands slower than the apply pass does (profiles/r6_imagenet_gfold_ab.log)
CG_GFOLD_MAXF = int(os.environ.get("DTF_CG_GFOLD_MAXF", "0"))
# BN3 + ReLU applied by conv3 (the 1x1 expand, its only forward consumer) and by conv3's weight gradient in the blocks
# whose conv3 has at most this many output channels (each a2 element is transformed once per 128-channel tile), so
# a2 = relu(BN3(h2)) is never written for them (0: off; 256 / 512 / 1024 / 2048 measured -0.1 / +0.0 / +0.3 / +0.4 ms,
# within box noise at 256: profiles/r6_imagenet_fold3_ab.log)
CG_FOLD3_MAXC = int(os.environ.get("DTF_CG_FOLD3_MAXC", "0"))
# XCD-aware work order (_xcd_order): 0 off, 1 operand-sharing runs on one XCD, 2 additionally every member on its own
# XCD when the population is a multiple of 8 with equal work per member, 3 (default) also members on XCD subsets when
# the population divides 8 (pop 4: 39.73 -> 38.95 ms).  ResNet-50 pop 8 x 128:
# 76.7 (0) -> 75.0 (1) -> 73.8 ms (2) (profiles/r5_xcd_order_ab.log)
_CG_XCD = int(os.environ.get("DTF_CG_XCD", "3"))
# generic forward / dgrad launches with fewer 256-pixel workgroups than this take 128-pixel tiles (conv())
_CG_SMALL = int(os.environ.get("DTF_CG_SMALL", "0"))
# ... and so do the 1x1 launches whose GEMM depth (Ci of the gathered operand) is at most this (memory-bound: more,
# smaller workgroups in flight)
_CG_SHORTK = int(os.environ.get("DTF_CG_SHORTK", "0"))
T3_FLAGS = int(os.environ.get("DTF_T3_FLAGS", "1"))  # direct: 81.61 vs staged 80.92 ms (profiles/r4_imagenet_t3_ab.log)
_CG_WG_TARGET = int(os.environ.get("DTF_CG_WG_TARGET", "512"))
# generic forward / dgrad launches whose images are at most this wide take 64-channel output tiles (more, smaller
# workgroups for the 7x7 stage's few-round launches; 0: off -- 7 / 14 measured +1.0 / +3.1 ms, profiles/r6_imagenet_tc64_ab.log)
_CG_TC64_HW = int(os.environ.get("DTF_CG_TC64_HW", "0"))
_CG_WG_MINCHUNK = int(os.environ.get("DTF_CG_WG_MINCHUNK", "2048"))
_CG_WG_BALANCED = os.environ.get("DTF_CG_WG_BALANCED", "0") == "1"


class CgArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("x2", c_void_p), ("dy", c_void_p), ("dy2", c_void_p), ("w", c_void_p),
        ("w_mstride", c_long), ("w_off", c_long), ("y", c_void_p), ("res", c_void_p), ("xm", c_void_p),
        ("grads", c_void_p), ("g_mstride", c_long), ("g_off", c_long), ("c_in", c_void_p), ("c_dy", c_void_p),
        ("c_ep", c_void_p), ("st_out", c_void_p), ("work", c_void_p),
        ("Hi", c_int), ("Wi", c_int), ("Ci", c_int), ("Ho", c_int), ("Wo", c_int), ("Co", c_int),
        ("kh", c_int), ("kw", c_int), ("stride", c_int), ("pad", c_int), ("cmax", c_int), ("log2ci", c_int),
        ("cin_real", c_int), ("flags", c_int), ("x3", c_void_p), ("xout", c_void_p),
    ]


class BnFinArgs(ctypes.Structure):
    _fields_ = [
        ("state", c_void_p), ("s_mstride", c_long), ("sums", c_void_p), ("coef", c_void_p), ("fcoef", c_void_p),
        ("grads", c_void_p), ("g_mstride", c_long), ("slots", c_void_p), ("cnt", c_void_p),
        ("gamma_off", c_int), ("beta_off", c_int), ("run_off", c_int), ("C", c_int), ("hw", c_int), ("cmax", c_int),
    ]


class EwArgs(ctypes.Structure):
    _fields_ = [("dz", c_void_p), ("h", c_void_p), ("add", c_void_p), ("out", c_void_p), ("coef", c_void_p),
                ("img_slot", c_void_p), ("hw", c_long), ("C", c_int), ("cmax", c_int), ("nimg", c_long)]


class GapArgs(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("coef", c_void_p), ("img_slot", c_void_p), ("feat", c_void_p),
                ("dfeat", c_void_p), ("sums", c_void_p), ("bcoef", c_void_p), ("out", c_void_p),
                ("hw", c_int), ("C", c_int), ("cmax", c_int)]


class BnAddArgs(ctypes.Structure):
    _fields_ = [("h", c_void_p), ("s", c_void_p), ("out", c_void_p), ("coef_h", c_void_p), ("coef_s", c_void_p),
                ("img_slot", c_void_p), ("hw", c_long), ("C", c_int), ("cmax", c_int), ("nimg", c_long)]


class BnSumArgs(ctypes.Structure):
    _fields_ = [("dz", c_void_p), ("h", c_void_p), ("h2", c_void_p), ("fc", c_void_p), ("fc2", c_void_p),
                ("sums", c_void_p), ("sums2", c_void_p), ("img_slot", c_void_p), ("hw", c_int), ("C", c_int),
                ("cmax", c_int), ("pad", c_int)]


_REGISTERED = False


def xcd_order(items, ng):
    """XCD-aware dispatch order: consecutive runs of ``ng`` items share an operand tile (the co-tiles of one
    pixel tile; the dW tiles of one pixel chunk).  Workgroup k runs on XCD k % 8, each XCD with its own L2, so
    the run is spread over positions 8 apart -- every item of a run lands on the same XCD, dispatched close in
    time, and the shared tile is fetched into one L2 instead of ng of them."""
    if not _CG_XCD:
        return items
    # items are member-major (slot order); with a multiple of 8 members of equal work, member m's items all go
    # to XCD m % 8 (its weights and activations then live in one L2; positions 8 apart, runs kept adjacent)
    nm = len(items) and len({it[0] for it in items})
    if _CG_XCD >= 2 and nm and (nm % 8 == 0 or (_CG_XCD >= 3 and 8 % nm == 0)) and len(items) % nm == 0:
        per = len(items) // nm
        mem = [items[m * per:(m + 1) * per] for m in range(nm)]
        if all(len({it[0] for it in blk}) == 1 for blk in mem):
            # mode 3, nm | 8 (pop 1 / 2 / 4 per GPU): member m owns XCDs m, m + nm, ..;
            # its own items run-ordered over those
            # 8 / nm XCDs (position j * nm + m of the launch holds its j-th item)
            q = 8 // nm if 8 % nm == 0 else 1
            if q > 1:
                mem = [_run_order(blk, ng, q) for blk in mem]
            out = []
            g = min(nm, 8)
            for g0 in range(0, nm, g):
                grp = mem[g0:g0 + g]
                for j in range(per):
                    out.extend(blk[j] for blk in grp)
            return out
    return _run_order(items, ng, 8)


def _run_order(items, ng, lanes):
    """Runs of ``ng`` consecutive items spread ``lanes`` apart (one dispatch lane = one XCD of the sub-machine)."""
    if ng <= 1 or len(items) % ng:
        return items
    runs = [items[i:i + ng] for i in range(0, len(items), ng)]
    out = []
    for b in range(0, len(runs), lanes):
        blk = runs[b:b + lanes]
        for c in range(ng):
            out.extend(r[c] for r in blk)
    return out


def _register():
    global _REGISTERED
    if _REGISTERED:
        return
    from . import hip_mnist
    hip_mnist._register()  # grouped GEMM signatures
    P = ctypes.POINTER
    reg = ops.register
    reg("dtf_convg_fwd", [P(CgArgs), c_int, c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_convg_t3", [P(CgArgs), c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_convg_wgrad", [P(CgArgs), c_int, c_int, c_int, c_void_p])
    reg("dtf_convg_wgrad_wide", [P(CgArgs), c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_convg_wgrad_t3", [P(CgArgs), c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_convg_stem_s2d", [P(CgArgs), c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_cg_weight_prep", [c_void_p, c_long, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_long,
                               c_void_p])
    reg("dtf_cg_dense_prep", [c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_long,
                              c_void_p])
    reg("dtf_cg_bn_final", [P(BnFinArgs), c_int, c_int, c_void_p])
    reg("dtf_cg_bn_bwd_apply", [P(EwArgs), c_void_p])
    reg("dtf_cg_bn_relu_apply", [P(EwArgs), c_void_p])
    reg("dtf_cg_prep_input", [c_void_p, c_void_p, c_long, c_int, c_void_p])
    reg("dtf_cg_prep_input_s2d", [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_cg_maxpool", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                           c_int, c_int, c_void_p])
    reg("dtf_cg_gap", [P(GapArgs), c_int, c_int, c_void_p])
    reg("dtf_cg_softmax_ce", [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_long, c_int, c_void_p, c_long,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_float, c_void_p])
    reg("dtf_cg_chan_stats", [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p])
    reg("dtf_cg_bn_add_relu", [P(BnAddArgs), c_void_p])
    reg("dtf_cg_bn_bwd_sums", [P(BnSumArgs), c_int, c_void_p])
    reg("dtf_cg_det_finish", [c_void_p, c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_void_p, c_void_p])
    reg("dtf_fixed_acc", [])
    for n in ("dtf_cg_args_size", "dtf_bnfin_args_size", "dtf_ew_args_size", "dtf_gap_args_size",
              "dtf_bnadd_args_size", "dtf_bnsum_args_size"):
        reg(n, [])
    L = ops.lib()
    for name, args in ops._SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes = args
            fn.restype = c_int
    for st, fn in ((CgArgs, "dtf_cg_args_size"), (BnFinArgs, "dtf_bnfin_args_size"), (EwArgs, "dtf_ew_args_size"),
                   (GapArgs, "dtf_gap_args_size"), (BnAddArgs, "dtf_bnadd_args_size"),
                   (BnSumArgs, "dtf_bnsum_args_size")):
        assert getattr(L, fn)() == ctypes.sizeof(st), "%s ABI mismatch" % st.__name__
    _REGISTERED = True


def _p(t):
    return None if t is None else t.data_ptr()


def _log2(n):
    assert n > 0 and n & (n - 1) == 0, n
    return n.bit_length() - 1


class HipImageNetBackend:
    name = "hip"
    accepts_index_batches = False
    _plan_cls = None  # _ImageNetPlan (set below); the fp32 backend: engine/hip_imagenet_f32.py

    def __init__(self, engine):
        _register()
        self.e = engine
        self.dev = engine.device
        prog = engine.arch.prog
        cfg = prog.cfg
        if not (cfg.bottleneck and cfg.version in (1, 2) and cfg.first_pool_size == 3 and cfg.first_pool_stride == 2
                and cfg.kernel_size == 7 and cfg.conv_stride == 2):
            raise ValueError("HIP ImageNet backend supports the v1 / v2 bottleneck ImageNet configurations")
        if cfg.image_size % 32:
            raise ValueError("image size must be a multiple of 32")
        self.prog, self.cfg = prog, cfg
        cap = engine.capacity
        # bf16 weights: the fused optimizer writes a bf16 shadow of every member row in the same pass as the
        # update; every conv (forward [o][tap][i] rows, and the data gradient reading the same layout k-major)
        # reads it in place.  Only the stem needs a channel-padded (3 -> 8) copy.
        for c in prog.convs:
            assert c.off % 8 == 0, "conv weights must be 16-byte aligned in the shadow row"
        self.shadow = torch.zeros(cap, engine.Pp, dtype=ops.act_dtype(), device=self.dev)
        st = prog.convs[prog.stem]
        self.s2d = (_CG_S2D and st.cin == 3 and st.k == 7 and st.stride == 2 and cfg.image_size % 4 == 0)
        if self.s2d:
            self.wtot = (st.cout * 16 * 16 + 63) // 64 * 64
            row = [st.off, st.cout, st.cin, st.k, 16, 0, -1, 1]
        else:
            self.wtot = (st.cout * st.k * st.k * 8 + 63) // 64 * 64
            row = [st.off, st.cout, st.cin, st.k, 8, 0, -1, 0]
        self.w = torch.zeros(cap, self.wtot, dtype=ops.act_dtype(), device=self.dev)  # padded / s2d stem
        self.conv_table = torch.tensor([row], dtype=torch.int32, device=self.dev)
        self.ncls = cfg.num_classes
        assert self.ncls <= NPAD_CLS and cfg.final_size % 32 == 0
        self.dense = torch.zeros(cap, NPAD_CLS * cfg.final_size, dtype=ops.act_dtype(), device=self.dev)
        nb = len(prog.bns)
        # deterministic build (common.h DTF_FIXED_ACC): every cross-workgroup sum -- BN statistics, BN-backward sums,
        # conv weight gradients, dense bias gradient, loss -- accumulates as int64 fixed point (order-free integer
        # atomics); cg_det_finish folds the gradient / loss accumulators into the fp32 rows before the optimizer
        self.det = bool(ops.lib().dtf_fixed_acc())
        # fp16 (half build): static loss scaling (resnet_run_loop.py:284-294): softmax-CE differentiates
        # loss_scale * loss, the fused optimizer unscales
        self.half = ops.build_half()
        assert self.half == (engine.compute_dtype == torch.float16), \
            "the loaded kernel library does not match compute dtype %s: fp16 needs DTF_HALF=1" % engine.compute_dtype
        self.loss_scale = float(engine.loss_scale) if self.half else 1.0
        self.acc_dtype = torch.int64 if self.det else torch.float32
        self.sums = torch.zeros(2, nb, cap, 2, CMAX, dtype=self.acc_dtype, device=self.dev)   # [fwd|bwd]
        self.coef = torch.zeros(2, nb, cap, 4, CMAX, dtype=torch.float32, device=self.dev)   # [fwd|bwd]
        self.loss = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        self.correct = torch.zeros(cap, dtype=torch.float32, device=self.dev)
        if self.det:
            self.gacc = torch.zeros(cap, engine.Pp, dtype=torch.int64, device=self.dev)
            self.loss64 = torch.zeros(cap, dtype=torch.int64, device=self.dev)
        self.acc_grads = self.gacc if self.det else engine.grads  # where the convg / softmax kernels accumulate
        self.acc_loss = self.loss64 if self.det else self.loss
        self.v1 = cfg.version == 1
        if self.v1:
            # identity "BN" coefficients (scale 1, shift 0): the convg epilogue's ReLU mask by BN(xm) > 0 then masks by
            # xm > 0 -- the v1 block input is a ReLU output
            self.ident = torch.zeros(cap, 4, CMAX, dtype=torch.float32, device=self.dev)
            self.ident[:, 0].fill_(1.0)
            self.ident[:, 3].fill_(1.0)
        self._plans: Dict[tuple, "_ImageNetPlan"] = {}
        self.use_graph = (os.environ.get("DTF_HIP_GRAPH", "1") == "1" and os.environ.get("DTF_DEBUG", "0") != "1")

    def on_params_changed(self, slots):
        slots = list(slots)
        if slots:  # rows changed outside the optimizer (init, exploit import): refresh their bf16 shadow
            e = self.e
            self._rows = ops.shadow_refresh(e.state, self.shadow, slots, e.Pp, e.P)

    def shadow_weights(self):
        return self.shadow

    def plan(self, slots, sizes):
        key = (tuple(slots), tuple(sizes))
        p = self._plans.get(key)
        if p is None:
            if len(self._plans) > 4:
                self._plans.clear()
            p = self._plan_cls(self, list(slots), list(sizes))
            self._plans[key] = p
        return p

    def train_step(self, slots, batches, hparams, lrs):
        e = self.e
        batches = [b.materialize() if isinstance(b, IndexBatch) else b for b in batches]
        sizes = [batch_len(b) for b in batches]
        p = self.plan(slots, sizes)
        upload_hyper(e, slots, hparams, lrs)
        p.load_batch(batches)
        p.run()
        note_step_advanced(e, slots)
        return p.loss_sel.clone()  # gathered inside the step graph

    def forward_backward(self, slots, batches):
        raise RuntimeError("HipImageNetBackend runs whole steps: use train_step")

    def train_correct(self, slots):
        """Correct predictions of each member's last training batch (softmax-CE kernel count; device tensor)."""
        return self.correct[torch.as_tensor(list(slots), dtype=torch.long, device=self.dev)]

    def eval_plan(self, slots, m):
        """Eval plans live in their own bounded cache: an eval pass never evicts the captured training graph."""
        key = (tuple(slots), int(m))
        plans = self.__dict__.setdefault("_eval_plans", {})
        p = plans.get(key)
        if p is None:
            if len(plans) >= 4:
                plans.pop(next(iter(plans)))  # oldest first
            p = self._plan_cls(self, list(slots), [int(m)] * len(slots), eval_mode=True)
            plans[key] = p
        return p

    @torch.no_grad()
    def infer(self, slot, x):
        """Eval-mode logits of one member on the HIP forward kernels (moving BN statistics)."""
        p = self.eval_plan([slot], int(x.shape[0]))
        p.load_eval(x, torch.zeros(x.shape[0], dtype=torch.int32, device=x.device))
        p.run_eval()
        e = self.e
        b = e.state[slot, self.prog.dense_b_off:self.prog.dense_b_off + self.ncls]
        return p.logits[:, :self.ncls] + b

    @torch.no_grad()
    def evaluate_population(self, slots, x, y, chunk=None):
        """Eval accuracy of every member in ``slots``: one population-batched forward per chunk of the eval set
        (BN with moving statistics, the same convg / GAP / dense kernels as training); one host sync."""
        n = int(x.shape[0])
        if n == 0 or not slots:
            return {s: 0.0 for s in slots}
        chunk = min(n, int(chunk or os.environ.get("DTF_EVAL_CHUNK_IMAGENET", "64")))
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


class _ImageNetPlan:
    def __init__(self, be: HipImageNetBackend, slots: List[int], sizes: List[int], eval_mode: bool = False):
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
        self.loss_sel = torch.zeros(len(slots), dtype=be.loss.dtype, device=dev)
        bf = self._act_dtype()
        H = cfg.image_size
        self.H = H
        self.x_in = torch.zeros(N, H, H, cfg.in_channels, dtype=torch.float32, device=dev)
        self.labels = torch.zeros(N, dtype=torch.int32, device=dev)
        self.xin8 = torch.zeros(*self._stem_input_shape(N, H), dtype=bf, device=dev)  # stem input (padded / s2d)
        H1 = H // 2
        H2 = (H1 + 1) // 2
        pool = {}

        def act(kind, hw_, c_, i_=0, dtype=bf):
            """Activation buffer; eval plans save nothing for a backward, so buffers are shared per shape (the
            residual stream ping-pongs between two)."""
            if not self.eval:
                return torch.empty(N, hw_, hw_, c_, dtype=dtype, device=dev)
            key = (kind, hw_, c_, i_ % 2 if kind == "x" else 0)
            if key not in pool:
                pool[key] = torch.empty(N, hw_, hw_, c_, dtype=dtype, device=dev)
            return pool[key]

        self.y0 = torch.empty(N, H1, H1, cfg.num_filters, dtype=bf, device=dev)
        self.am0 = torch.empty(N, H2, H2, cfg.num_filters, dtype=torch.uint8, device=dev)
        self.xs, self.h1, self.h2, self.sc = [act("x", H2, cfg.num_filters, 0)], [], [], []
        # materialised BN+ReLU outputs (the operands every consumer conv stages as-is, and the weight-gradient
        # inputs): ax = relu(BN1(x)), a1 = relu(BN2(h1)), a2 = relu(BN3(h2)).  (Applying BN+ReLU while each consumer
        # stages its operand measured slower, 114.7 -> 135.7 ms/step at pop 8 x 128: the transform is repeated for
        # every output-channel tile and its coefficient LDS costs occupancy; profiles/r2_imagenet_fold_ab.log)
        self.ax, self.a1, self.a2 = [], [], []
        # folded forward (CG_FOLD): v2 training plans keep no relu(BN(.)) tensors
        self.fold = CG_FOLD and not self.eval and not be.v1
        self.fold2 = CG_FOLD2 and not self.fold and not self.eval and not be.v1
        self.fold1 = CG_FOLD1 and not self.fold and not self.eval and not be.v1 and self.FOLD1_OK
        self.fold3 = CG_FOLD3_MAXC > 0 and not self.fold and not self.eval and not be.v1 and self.FOLD1_OK
        # v1 (post-activation): h3 = conv3 output (BN3 input), sc = raw projection output (BN_p input), a0 = the
        # stem's relu(BN(y0)); no ax (the block input IS a ReLU output)
        self.v1 = be.v1
        self.h3 = []
        self.a0 = torch.empty(N, H1, H1, cfg.num_filters, dtype=bf, device=dev) if self.v1 else None
        hw, cin = H2, cfg.num_filters
        self.geo = []  # per block: (H_in, H_out, cin, f, fout)
        for bi, blk in enumerate(prog.blocks):
            c1, c2, c3 = (prog.convs[i] for i in blk.convs)
            ho = hw // blk.stride
            self.h1.append(act("h1", hw, c1.cout))
            self.h2.append(act("h2", ho, c2.cout))
            self.ax.append(act("ax", hw, cin) if not (self.v1 or self.fold) else None)
            self.h3.append(act("h3", ho, c3.cout) if self.v1 else None)
            self.a1.append(act("a1", hw, c1.cout) if not (self.fold or self.fold2) else None)
            self.a2.append(act("a2", ho, c2.cout) if not (self.fold or self._fold3(bi)) else None)
            self.sc.append(act("sc", ho, c3.cout) if blk.proj is not None else None)
            self.xs.append(act("x", ho, c3.cout, bi + 1))
            self.geo.append((hw, ho, cin, c1.cout, c3.cout))
            hw, cin = ho, c3.cout
        self.HL = hw
        self.feat = torch.empty(N, cfg.final_size, dtype=bf, device=dev)
        self.logits = torch.empty(N, NPAD_CLS, dtype=torch.float32, device=dev)
        self.dlog = torch.zeros(N, NPAD_CLS, dtype=bf, device=dev)
        self.dfeat = torch.empty(N, cfg.final_size, dtype=torch.float32, device=dev)
        self._tmp: Dict[tuple, torch.Tensor] = {}
        self._keep = []
        self.launches = []
        if self.eval:
            nb = len(prog.bns)
            self.ev_coef = torch.zeros(nb, e.capacity, 4, CMAX, dtype=torch.float32, device=dev)
            self.ev_sink = torch.zeros(e.capacity, 2, CMAX, dtype=be.acc_dtype, device=dev)  # conv-epilogue stats
            self.ev_acc = torch.zeros(2, e.capacity, dtype=torch.float32, device=dev)  # [correct, summed CE]
            self.ev_loss = torch.zeros(e.capacity, dtype=be.acc_dtype, device=dev)  # summed CE (accumulator words)
            self._build_eval_v1() if self.v1 else self._build_eval()
        else:
            self._build_v1() if self.v1 else self._build()
        self.graph = None

    # ----------------------------------------------------------------------------------------- helpers
    def _act_dtype(self):
        return ops.act_dtype()  # bf16 (fp16 in the half build)

    def _stem_input_shape(self, N, H):
        """Space-to-depth [N, H/2, H/2, 16] (12 real channels), else the 3 channels padded to the stem's 8-channel
        gather chunks."""
        return (N, H // 2, H // 2, 16) if self.be.s2d else (N, H, H, 8)

    def tmp(self, name, hw, c):
        key = (name, hw, c)
        t = self._tmp.get(key)
        if t is None:
            t = torch.empty(self.N, hw, hw, c, dtype=self._act_dtype(), device=self.be.dev)
            self._tmp[key] = t
        return t

    def _add(self, fn, *args):
        self.launches.append((fn, args))

    def _hold(self, obj):
        self._keep.append(obj)
        return obj

    @staticmethod
    def _xcd_order(items, ng):
        return xcd_order(items, ng)

    def _pix_work(self, hw_grid, co, tc, classes=(0,), tp=128):
        """(slot, p0, p1, o0 | class << 16) tiles of 128 grid pixels x tc output channels per member; a
        transposed (stride-2) dgrad runs every parity class (py*2 + px) over the dy-resolution grid."""
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            p_end = (f + n) * hw_grid * hw_grid
            for cls in classes:
                for p0 in range(f * hw_grid * hw_grid, p_end, tp):
                    for o0 in range(0, co, tc):
                        items.append([s, p0, min(p0 + tp, p_end), o0 | (cls << 16)])
        items = self._xcd_order(items, -(-co // tc))
        return self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))

    def _band_work(self, hw, rows, co, tc):
        """(slot, p0, p1, o0) tiles of `rows` whole image rows x tc output channels (convg_t3_kernel)."""
        items = []
        for s, n in zip(self.slots, self.sizes):
            for img in range(self.first[s], self.first[s] + n):
                for y0 in range(0, hw, rows):
                    p0 = (img * hw + y0) * hw
                    for o0 in range(0, co, tc):
                        items.append([s, p0, p0 + min(rows, hw - y0) * hw, o0])
        items = self._xcd_order(items, -(-co // tc))
        return self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))

    def _wgrad_work(self, hw_out, co, K, wo=128, wt=128):
        """(slot, p0, p1, o0 | n0/8 << 16) split-K items of the weight gradient: 128 x 128 dW tiles per member, the
        member's pixels split into chunks so that the launch has about ``_CG_WG_TARGET`` items.  Every item
        atomically adds its full fp32 tile into the member's gradient row, so the split count is a trade: more
        items fill the chip, but each split adds 64 KB of atomic traffic per tile (the chip absorbs about 1.3 TB/s
        of atomic adds).  The former 4096-item target moved ~14 GB of atomics per pop-8 ResNet-50 step; with the
        wide-column tiles 512 items measured best (85.3 ms/step vs 87.2 at 1024, 93.5 at 256;
        profiles/r2_s3_imagenet_wg_target_ab.log)."""
        tiles = -(-co // wo) * -(-K // wt)
        per_member = max(1, -(-_CG_WG_TARGET // max(1, len(self.slots) * tiles)))
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            p_beg, p_end = f * hw_out * hw_out, (f + n) * hw_out * hw_out
            if _CG_WG_BALANCED:  # equal splits (the rounded chunk could leave a short last one)
                nsplit = max(1, min(per_member, (p_end - p_beg) // _CG_WG_MINCHUNK))
                chunk = (-(-(p_end - p_beg) // nsplit) + 63) // 64 * 64
            else:
                chunk = max(_CG_WG_MINCHUNK, -(-(p_end - p_beg) // per_member))
                chunk = (chunk + 63) // 64 * 64
            for p0 in range(p_beg, p_end, chunk):
                for o0 in range(0, co, wo):
                    for n0 in range(0, K, wt):
                        items.append([s, p0, min(p0 + chunk, p_end), o0 | ((n0 // 8) << 16)])
        items = self._xcd_order(items, -(-co // wo) * -(-K // wt))
        return self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))

    def _args(self):
        be, e = self.be, self.e
        a = CgArgs()
        a.w_mstride = e.Pp
        a.grads, a.g_mstride = _p(be.acc_grads), e.Pp
        a.cmax = CMAX
        a.flags = T3_FLAGS
        return a

    def cf(self, bn):  # forward coefficients of BN `bn` (eval: from the moving statistics, the plan's own buffer)
        return self.ev_coef[bn] if self.eval else self.be.coef[0, bn]

    def cb(self, bn):  # backward coefficients
        return self.be.coef[1, bn]

    def sf(self, bn):
        return self.be.sums[0, bn]

    def sb(self, bn):
        return self.be.sums[1, bn]

    def conv(self, ci, src, out, hw_in, mode=0, c_in=None, x2=None, epi=0, res=None, xm=None, c_ep=None, st=None,
             dgrad=False, compact=False, x3=None, xout=None):
        """Forward conv (dgrad=False) or data gradient (dgrad=True) of conv `ci` through convg_fwd.  ``compact``
        (the data gradient of a stride-2 1x1 conv): only the even output rows / columns are nonzero, so the gradient
        is computed and stored at the dy resolution, [N, hw_in, hw_in, cin] -- a plain 1x1 GEMM with no zero-filled
        parity classes; its consumer reads it with convg EPI bit 8."""
        be = self.be
        c = self.be.prog.convs[ci]
        k = c.k
        pad = (k - 1) // 2
        a = self._args()
        a.x, a.x2, a.y, a.res, a.xm = _p(src), _p(x2), _p(out), _p(res), _p(xm)
        a.w, a.w_off = _p(be.shadow), c.off
        if ci == be.prog.stem:
            a.w, a.w_mstride, a.w_off = _p(be.w), be.wtot, 0
        a.c_in, a.c_ep, a.st_out = _p(c_in), _p(c_ep), _p(st)
        a.x3, a.xout = _p(x3), _p(xout)
        assert mode != 3 or (dgrad and k == 1 and c.stride == 1 and xout is not None), "MODE 3: 1x1 data gradient"
        a.kh = a.kw = k
        if not dgrad:
            cin = 8 if ci == be.prog.stem else c.cin
            hw_out = (hw_in + c.stride - 1) // c.stride
            a.Hi = a.Wi = hw_in
            a.Ci, a.Co = cin, c.cout
            a.Ho = a.Wo = hw_out
            a.stride, a.pad = c.stride, pad
            trans = 0
        elif compact:
            assert k == 1 and c.stride == 2 and pad == 0, (ci, k, c.stride)
            hw_out = hw_in
            a.Hi = a.Wi = a.Ho = a.Wo = hw_in
            a.Ci, a.Co = c.cout, c.cin
            a.stride, a.pad = 1, 0
            trans = 2
        else:
            # gathered = dy at the conv's output resolution; output = dx at its input resolution
            hw_out = hw_in * c.stride
            a.Hi = a.Wi = hw_in
            a.Ci, a.Co = c.cout, c.cin
            a.Ho = a.Wo = hw_out
            a.stride, a.pad = c.stride, k - 1 - pad
            trans = (1 if c.stride > 1 else 0) | 2  # | 2: A operand k-major from the forward layout
        if ci == be.prog.stem and be.s2d:
            assert not dgrad
            a.Hi = a.Wi = a.Ho = a.Wo = hw_in // 2  # 4x4/1 over 2x2 blocks (pad 2 before, 1 after)
            a.Ci, a.kh, a.kw, a.stride, a.pad = 16, 4, 4, 1, 2
            if _CG_STEM_BAND and a.Hi == 112 and mode == 0 and epi in (0, 4) and c.cout == 64:
                a.log2ci = 4
                bpi = a.Hi // 2
                total = self.N * bpi
                chunk = max(1, -(-total // _CG_STEM_WG))
                items = []
                for s_, n_ in zip(self.slots, self.sizes):
                    f_ = self.first[s_]
                    for b in range(f_ * bpi, (f_ + n_) * bpi, chunk):
                        items.append([s_, b, min(b + chunk, (f_ + n_) * bpi), 0])
                items = self._xcd_order(items, 1)
                work = self._hold(torch.tensor(items, dtype=torch.int32, device=be.dev))
                a.work = _p(work)
                self._hold(a)
                self._add(ops.lib().dtf_convg_stem_s2d, ctypes.byref(a), a.Hi, 2, epi, work.shape[0])
                return
        a.log2ci = _log2(a.Ci)
        tc = 128 if a.Co >= 128 and max(hw_in, hw_out) > _CG_TC64_HW else 64
        if (k == 3 and c.stride == 1 and (mode == 0 or (mode == 1 and not dgrad)) and hw_in in _CG_T3
                and ci != be.prog.stem and epi == (6 if dgrad else 4) and a.Ci % 32 == 0 and a.Ci <= 512):
            rows = _CG_T3[hw_in]
            tc = 64 if hw_in == 56 else 128  # must match dtf_convg_t3's instantiations
            work = self._band_work(hw_in, rows, a.Co, tc)
            a.work = _p(work)
            self._hold(a)
            self._add(ops.lib().dtf_convg_t3, ctypes.byref(a), tc, epi, int(dgrad), hw_in, work.shape[0], mode)
            return
        # (a 256-row tile, 128 x 64 per wave, measured slower: 111.7 -> 123.4 ms/step at pop 8 x 128,
        # profiles/r2_imagenet_tc256_ab.log -- removed)
        tp = 128
        # small launches (one member's 14x14 / 7x7 layers: 100-200 workgroups of 256 pixels on 256 CUs) take the
        # 128-pixel tiles -- twice the workgroups
        grid_px = (hw_in * hw_in) if trans & 1 else (hw_out * hw_out)
        n256 = -(-(self.N * grid_px * (4 if trans & 1 else 1)) // 256) * -(-a.Co // tc)
        small = n256 < _CG_SMALL or (k == 1 and a.Ci <= _CG_SHORTK)
        if not small and ((tc == 64 and _CG_TP256) or (tc == 128 and _CG_TP256_128)):
            trans |= 8  # 256-pixel tiles (BK = 32): 1 x 4 waves of 64 x 64, or 2 x 2 of 64 x 128 for tc 128
            tp = 256
            if _CG_M32 and tc == 128 and not dgrad:
                trans |= 16  # 32x32x16 MFMA tiles
        elif _CG_BK == 64 and (not trans or a.Ci >= 64):
            trans |= 4  # k depth 64 per LDS stage
        # parity classes of a stride-2 data gradient carry 1 / 2 / 2 / 4 taps (3x3, pad 1): CG_CLASS_LPT dispatches the
        # 4-tap class first (longest-processing-time order) so the launch does not end on a round of its heaviest items
        cls = (3, 1, 2, 0) if (CG_CLASS_LPT and k == 3) else (0, 1, 2, 3)
        work = (self._pix_work(hw_in, a.Co, tc, classes=cls, tp=tp) if trans & 1
                else self._pix_work(hw_out, a.Co, tc, tp=tp))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_convg_fwd, ctypes.byref(a), tc, mode, epi, trans, work.shape[0])

    def wgrad(self, ci, x, dy, hw_in, mode_x=0, c_x=None, mode_dy=0, c_dy=None, dy2=None):
        be = self.be
        c = be.prog.convs[ci]
        a = self._args()
        cin = 8 if ci == be.prog.stem else c.cin
        hw_out = (hw_in + c.stride - 1) // c.stride
        a.x, a.dy, a.dy2 = _p(x), _p(dy), _p(dy2)
        a.c_in, a.c_dy = _p(c_x), _p(c_dy)
        a.g_off = c.off
        a.Hi = a.Wi = hw_in
        a.Ci, a.Co = cin, c.cout
        a.Ho = a.Wo = hw_out
        a.kh = a.kw = c.k
        a.stride, a.pad = c.stride, (c.k - 1) // 2
        a.log2ci = _log2(cin)
        a.cin_real = c.cin
        K = c.k * c.k * cin
        s2d = ci == be.prog.stem and be.s2d
        if s2d:  # 4x4/1 over the 2x2-block input; the writer maps (tap', block channel) onto the 7x7x3 kernel
            a.Hi = a.Wi = a.Ho = a.Wo = hw_out
            a.Ci, a.kh, a.kw, a.stride, a.pad = 16, 4, 4, 1, 2
            a.log2ci, a.cin_real = 4, -3
            K = 256
        if (c.k == 3 and c.stride == 1 and not s2d and hw_in in _CG_WGT3 and mode_x in (0, 1) and mode_dy == 0
                and cin % 32 == 0 and c.cout % 8 == 0):
            self._wgrad_t3(a, hw_in, cin, c.cout, mode_x=mode_x)
            return
        if s2d and _CG_WGT3 and hw_out == 112 and mode_x == 0 and mode_dy == 0:  # the stem: 2-row bands of 112
            self._wgrad_t3(a, hw_out, 16, c.cout, R=2, bkc=16)
            return
        wide3 = c.k == 3 and cin % 64 == 0
        wide1 = c.k == 1 and cin % 256 == 0 and _CG_WIDE1
        wide7 = ci == be.prog.stem and c.k == 7 and cin == 8 and c.cout == 64 and _CG_WIDE7 and not s2d
        if (_CG_WIDE and (wide3 or wide1 or wide7 or s2d) and mode_x in (0, 1) and mode_dy == 0
                and not ((wide7 or s2d) and mode_x)):
            # 64 / 128 x 288 (3x3), x 256 (1x1, and the 4x4 x 16 s2d stem) or 64 x 416 (7x7 stem) tiles: 18 / 36,
            # 16 / 32, 26 MFMAs per wave and 32-pixel k-step (convg_wgrad_wide_kernel)
            wo = 128 if c.cout % 128 == 0 and _CG_WIDE128 else 64
            wt = 288 if wide3 else (256 if (wide1 or s2d) else 416)
            work = self._wgrad_work(hw_out, c.cout, K, wo, wt)
            a.work = _p(work)
            self._hold(a)
            self._add(ops.lib().dtf_convg_wgrad_wide, ctypes.byref(a), wo, wt, work.shape[0], mode_x)
            return
        wo = 64 if (c.cout % 128 != 0 and _CG_WO64) else 128  # 64-row tiles: no padded half for Co = 64
        work = self._wgrad_work(hw_out, c.cout, c.k * c.k * cin, wo)
        a.work = _p(work)
        self._hold(a)
        flags = (4 if (_CG_WPK_WO64 if wo == 64 else _CG_WPK) == 64 else 0) | (8 if wo == 64 else 0)
        self._add(ops.lib().dtf_convg_wgrad, ctypes.byref(a), mode_x, mode_dy | flags, work.shape[0])

    def _wgrad_t3(self, a, hw, cin, cout, R=None, bkc=32, mode_x=0):
        """Row-band weight gradient (3x3, or the 4x4 space-to-depth stem with R = 2, bkc = 16): items (slot, first
        band, end band, o0 | ci chunk << 16) -- per member, per 64-row output tile and bkc-channel input chunk, the
        member's bands split into about _CG_WGT3_TARGET items."""
        R = R or _CG_WGT3[hw]
        bpi = hw // R
        tiles = [(o0, cc) for o0 in range(0, cout, 64) for cc in range(cin // bkc)]
        total = sum(self.sizes) * bpi * len(tiles)
        chunk = max(1, -(-total // _CG_WGT3_TARGET))
        items = []
        for s, n in zip(self.slots, self.sizes):
            f = self.first[s]
            for b in range(f * bpi, (f + n) * bpi, chunk):
                for (o0, cc) in tiles:
                    items.append([s, b, min(b + chunk, (f + n) * bpi), o0 | (cc << 16)])
        items = self._xcd_order(items, len(tiles))
        work = self._hold(torch.tensor(items, dtype=torch.int32, device=self.be.dev))
        a.work = _p(work)
        self._hold(a)
        self._add(ops.lib().dtf_convg_wgrad_t3, ctypes.byref(a), hw, R, work.shape[0], mode_x)

    def bn_final(self, bn, hw, backward):
        be, e = self.be, self.e
        b = be.prog.bns[bn]
        a = BnFinArgs()
        a.state, a.s_mstride = _p(e.state), e.S
        a.sums = _p(self.sb(bn) if backward == 1 else self.sf(bn))
        a.coef = _p(self.cb(bn) if backward == 1 else self.cf(bn))  # backward 2: eval (moving statistics)
        a.fcoef = _p(self.cf(bn))
        a.grads, a.g_mstride = _p(e.grads), e.Pp
        a.slots, a.cnt = _p(self.slots_t), _p(self.cnt)
        a.gamma_off, a.beta_off, a.run_off = b.gamma_off, b.beta_off, 3 * e.Pp + b.run_off
        a.C, a.hw, a.cmax = b.c, hw * hw, CMAX
        self._hold(a)
        self._add(ops.lib().dtf_cg_bn_final, ctypes.byref(a), int(backward), len(self.slots))

    def ew(self, fn, h, out, coef, hw, C, dz=None, add=None):
        """Elementwise BN apply: fn = dtf_cg_bn_relu_apply (out = relu(BN(h))) or dtf_cg_bn_bwd_apply
        (out = A dz + B h + C [+ add])."""
        a = EwArgs()
        a.dz, a.h, a.add, a.out = _p(dz), _p(h), _p(add), _p(out)
        a.coef, a.img_slot, a.hw, a.C, a.cmax, a.nimg = _p(coef), _p(self.img_slot), hw * hw, C, CMAX, self.N
        self._hold(a)
        self._add(fn, ctypes.byref(a))

    def det_finish(self):
        be, e = self.be, self.e
        if be.det:
            self._add(ops.lib().dtf_cg_det_finish, _p(be.gacc), _p(e.grads), e.Pp, e.Pp, _p(self.slots_t),
                      len(self.slots), _p(be.loss64), _p(be.loss))

    # ------------------------------------------------------------------------- kernel vocabulary (non-conv ops)
    # The fp32 plan (engine/hip_imagenet_f32.py) runs the same program with fp32 kernels by overriding these, conv,
    # wgrad, ew, bn_add_relu and bwd_sums.
    def prep_weights(self):
        """Padded stem copy and the [NPAD_CLS][C] bf16 dense operand of every member of the plan (every other conv
        reads the optimizer's bf16 shadow)."""
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        L, ns = ops.lib(), len(self.slots)
        self._add(L.dtf_cg_weight_prep, _p(e.state), e.S, _p(be.conv_table), 1, _p(self.slots_t), ns,
                  _p(be.w), _p(be.w), be.wtot)
        self._add(L.dtf_cg_dense_prep, _p(e.state), e.S, prog.dense_w_off, be.ncls, NPAD_CLS, cfg.final_size,
                  _p(self.slots_t), ns, _p(be.dense), NPAD_CLS * cfg.final_size)

    def prep_input(self):
        if self.be.s2d:
            self._add(ops.lib().dtf_cg_prep_input_s2d, _p(self.x_in), _p(self.xin8), self.N, self.H, self.H,
                      self.be.cfg.in_channels)
            return
        self._add(ops.lib().dtf_cg_prep_input, _p(self.x_in), _p(self.xin8), self.N * self.H * self.H,
                  self.be.cfg.in_channels)

    def maxpool(self, x, y, H1, H2):
        self._add(ops.lib().dtf_cg_maxpool, _p(x), _p(y), _p(self.am0), None, None, self.N, H1, H1, H2, H2,
                  self.be.cfg.num_filters, 0)

    def maxpool_bwd(self, g, dx, H1, H2):
        self._add(ops.lib().dtf_cg_maxpool, None, None, _p(self.am0), _p(g), _p(dx), self.N, H1, H1, H2, H2,
                  self.be.cfg.num_filters, 1)

    def chan_stats(self, x, sums, hw, C):
        self._add(ops.lib().dtf_cg_chan_stats, _p(x), _p(self.img_slot), _p(sums), self.N, hw, C, CMAX)

    def gap(self, g, which):
        self._add(ops.lib().dtf_cg_gap, ctypes.byref(g), which, self.N)

    def dense_head(self, train):
        """Dense layer + softmax CE on the GAP features: the grouped bf16 GEMM (padded to NPAD_CLS classes) per
        member, cg_softmax_ce (bias, loss, correct count, dlogits, dbias); training adds dfeat = dlogits W and
        dW += dlogits^T feat."""
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        L = ops.lib()
        from .hip_mnist import GEMM_OUT_ACC, GEMM_OUT_F32, GroupedGemm
        C = cfg.final_size
        Dstride = NPAD_CLS * C
        fwd, dgr, wgr = [], [], []
        for s, n in zip(self.slots, self.sizes):
            f0 = self.first[s]
            fwd.append((f0 * C, s * Dstride, f0 * NPAD_CLS, n, NPAD_CLS, C))
            dgr.append((f0 * NPAD_CLS, s * Dstride, f0 * C, n, C, NPAD_CLS))
            wgr.append((f0 * NPAD_CLS, f0 * C, s * e.Pp + prog.dense_w_off, NPAD_CLS, C, n, be.ncls))
        dev = be.dev
        self.g_fwd = GroupedGemm(self.feat, be.dense, self.logits, C, C, NPAD_CLS, fwd, False, False, GEMM_OUT_F32, dev)
        self._add("gemm", self.g_fwd)
        if not train:
            self._add(L.dtf_cg_softmax_ce, _p(self.logits), NPAD_CLS, be.ncls, _p(self.labels), _p(self.img_slot),
                      _p(e.state), e.S, prog.dense_b_off, None, e.Pp, _p(self.cnt), _p(self.ev_loss),
                      _p(self.ev_acc[0]), None, self.N, 1.0)
            return
        self.g_dgr = GroupedGemm(self.dlog, be.dense, self.dfeat, NPAD_CLS, C, C, dgr, False, True, GEMM_OUT_F32, dev)
        self.g_wgr = GroupedGemm(self.dlog, self.feat, e.grads, NPAD_CLS, C, C, wgr, True, True, GEMM_OUT_ACC, dev)
        self._add(L.dtf_cg_softmax_ce, _p(self.logits), NPAD_CLS, be.ncls, _p(self.labels), _p(self.img_slot),
                  _p(e.state), e.S, prog.dense_b_off, _p(be.acc_grads), e.Pp, _p(self.cnt), _p(be.acc_loss),
                  _p(be.correct), _p(self.dlog), self.N, be.loss_scale)
        self._add("gemm", self.g_dgr)
        self._add("gemm", self.g_wgr)

    FOLD1_OK = True  # the fp32 plan (hip_imagenet_f32.py) keeps the materialised relu(BN1(x))
    GFOLD_OK = True  # ... and the standalone block-input gradient apply
    COMPACT_PD_OK = True  # ... and the full-resolution projection data gradient

    def _fold3(self, i):
        """Block i's BN3 + ReLU is applied by conv3 (forward, MODE 1) and its weight gradient (CG_FOLD3_MAXC)."""
        if not getattr(self, "fold3", False):
            return False
        return self.be.prog.convs[self.be.prog.blocks[i].convs[2]].cout <= CG_FOLD3_MAXC

    def _gfold(self, i):
        """Block i's input gradient g is applied by block i - 1's conv3 data gradient (MODE 3, CG_GFOLD_MAXF)."""
        if not (self.GFOLD_OK and CG_GFOLD_MAXF > 0 and i > 0 and not self.eval and not self.be.v1):
            return False
        prog = self.be.prog
        c3 = prog.convs[prog.blocks[i - 1].convs[2]]
        return c3.k == 1 and c3.stride == 1 and c3.cin <= min(CG_GFOLD_MAXF, 128)

    def _fold1(self, i):
        """Block i's BN1 + ReLU is applied by conv1 itself (CG_FOLD1: no projection, one output-channel tile)."""
        if not getattr(self, "fold1", False):
            return False
        blk = self.be.prog.blocks[i]
        return blk.proj is None and self.be.prog.convs[blk.convs[0]].cout <= CG_FOLD1_MAXC

    # ------------------------------------------------------------------------------------------ program
    def _build(self):
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        L = ops.lib()
        N, H = self.N, self.H
        ns = len(self.slots)
        self.prep_weights()
        self._add("zero", be.sums)
        self._add("zero", be.loss)
        self._add("zero", be.correct)
        self.prep_input()
        # ---- stem: conv 7x7/2 (no BN in v2) -> max-pool 3x3/2
        H1, H2 = H // 2, self.xs[0].shape[1]
        self.conv(prog.stem, self.xin8, self.y0, H, mode=0, epi=0)
        self.maxpool(self.y0, self.xs[0], H1, H2)
        self.chan_stats(self.xs[0], self.sf(prog.blocks[0].bns[0]), H2 * H2, cfg.num_filters)
        nblk = len(prog.blocks)
        for i, blk in enumerate(prog.blocks):
            hi, ho, cin, f, fout = self.geo[i]
            b1, b2, b3 = blk.bns
            c1, c2, c3 = blk.convs
            x = self.xs[i]
            relu = L.dtf_cg_bn_relu_apply
            nxt = prog.blocks[i + 1].bns[0] if i + 1 < nblk else prog.final_bn
            res = self.sc[i] if blk.proj is not None else x
            self.bn_final(b1, hi, False)
            if self.fold:
                if blk.proj is not None:
                    self.conv(blk.proj, x, self.sc[i], hi, mode=1, c_in=self.cf(b1), epi=0)
                self.conv(c1, x, self.h1[i], hi, mode=1, c_in=self.cf(b1), epi=4, st=self.sf(b2))
                self.bn_final(b2, hi, False)
                self.conv(c2, self.h1[i], self.h2[i], hi, mode=1, c_in=self.cf(b2), epi=4, st=self.sf(b3))
                self.bn_final(b3, ho, False)
                self.conv(c3, self.h2[i], self.xs[i + 1], ho, mode=1, c_in=self.cf(b3), epi=5, res=res,
                          st=self.sf(nxt))
                continue
            if self._fold1(i):
                self.conv(c1, x, self.h1[i], hi, mode=1, c_in=self.cf(b1), epi=4, st=self.sf(b2))
            else:
                self.ew(relu, x, self.ax[i], self.cf(b1), hi, cin)
            if blk.proj is not None:
                self.conv(blk.proj, self.ax[i], self.sc[i], hi, mode=0, epi=0)
            if not self._fold1(i):
                self.conv(c1, self.ax[i], self.h1[i], hi, mode=0, epi=4, st=self.sf(b2))
            self.bn_final(b2, hi, False)
            if self.fold2:
                self.conv(c2, self.h1[i], self.h2[i], hi, mode=1, c_in=self.cf(b2), epi=4, st=self.sf(b3))
            else:
                self.ew(relu, self.h1[i], self.a1[i], self.cf(b2), hi, f)
                self.conv(c2, self.a1[i], self.h2[i], hi, mode=0, epi=4, st=self.sf(b3))
            self.bn_final(b3, ho, False)
            if self._fold3(i):
                self.conv(c3, self.h2[i], self.xs[i + 1], ho, mode=1, c_in=self.cf(b3), epi=5, res=res,
                          st=self.sf(nxt))
                continue
            self.ew(relu, self.h2[i], self.a2[i], self.cf(b3), ho, f)
            self.conv(c3, self.a2[i], self.xs[i + 1], ho, mode=0, epi=5, res=res, st=self.sf(nxt))
        fb = prog.final_bn
        HL = self.HL
        self.bn_final(fb, HL, False)
        g = GapArgs()
        g.x, g.coef, g.img_slot, g.feat = _p(self.xs[-1]), _p(self.cf(fb)), _p(self.img_slot), _p(self.feat)
        g.dfeat, g.sums, g.bcoef = _p(self.dfeat), _p(self.sb(fb)), _p(self.cb(fb))
        g.hw, g.C, g.cmax = HL * HL, cfg.final_size, CMAX
        self._hold(g)
        self.gap(g, 0)
        # ---- dense + softmax CE
        self.dense_head(True)
        # ---- final BN backward -> gradient at the last block output
        self.gap(g, 1)
        self.bn_final(fb, HL, True)
        gcur = self.tmp("g0", HL, cfg.final_size)
        g2 = GapArgs()
        ctypes.memmove(ctypes.addressof(g2), ctypes.addressof(g), ctypes.sizeof(GapArgs))
        g2.out = _p(gcur)
        self._hold(g2)
        self.gap(g2, 2)
        # ---- blocks, reversed
        gpend = None  # a block-input gradient left to its consumer (CG_GFOLD_MAXF): (dz1, x, BN1 coefficients, add)
        for i in range(nblk - 1, -1, -1):
            blk = prog.blocks[i]
            hi, ho, cin, f, fout = self.geo[i]
            b1, b2, b3 = blk.bns
            c1, c2, c3 = blk.convs
            x, h1, h2 = self.xs[i], self.h1[i], self.h2[i]
            bwd = L.dtf_cg_bn_bwd_apply
            # conv3: dz3 = dgrad(g) masked by BN3(h2) (+ BN3 reductions); dh2 = BN3-backward(dz3, h2)
            dz3 = self.tmp("dz3", ho, f)
            if gpend is not None:  # g of block i + 1 computed (and stored into gcur) while this dgrad stages it
                pdz, px, pcb, padd = gpend
                self.conv(c3, pdz, dz3, ho, mode=3, c_in=pcb, x2=px, x3=padd, xout=gcur, epi=6, xm=h2,
                          c_ep=self.cf(b3), st=self.sb(b3), dgrad=True)
                gpend = None
            else:
                self.conv(c3, gcur, dz3, ho, mode=0, epi=6, xm=h2, c_ep=self.cf(b3), st=self.sb(b3), dgrad=True)
            self.bn_final(b3, ho, True)
            dh2 = self.tmp("dh2", ho, f)
            self.ew(bwd, h2, dh2, self.cb(b3), ho, f, dz=dz3)
            if self.fold or self._fold3(i):
                self.wgrad(c3, h2, gcur, ho, mode_x=1, c_x=self.cf(b3))
            else:
                self.wgrad(c3, self.a2[i], gcur, ho)
            # conv2 (3x3 / s): dz2 = dgrad(dh2) masked by BN2(h1); dh1 = BN2-backward(dz2, h1)
            dz2 = self.tmp("dz2", hi, f)
            self.conv(c2, dh2, dz2, ho, mode=0, epi=6, xm=h1, c_ep=self.cf(b2), st=self.sb(b2), dgrad=True)
            self.bn_final(b2, hi, True)
            dh1 = self.tmp("dh1", hi, f)
            self.ew(bwd, h1, dh1, self.cb(b2), hi, f, dz=dz2)
            if self.fold or self.fold2:
                self.wgrad(c2, h1, dh2, hi, mode_x=1, c_x=self.cf(b2))
            else:
                self.wgrad(c2, self.a1[i], dh2, hi)
            pd = None
            cpd = False
            if blk.proj is not None:
                pc = prog.convs[blk.proj]
                # a stride-2 projection's data gradient is zero at odd rows / columns: kept compact at the dy
                # resolution and added by conv1's epilogue at the even pixels (CG_COMPACT_PD)
                cpd = CG_COMPACT_PD and self.COMPACT_PD_OK and pc.stride == 2 and pc.k == 1
                pd = self.tmp("pdc" if cpd else "pd", ho if cpd else hi, cin)
                self.conv(blk.proj, gcur, pd, ho, mode=0, epi=0, dgrad=True, compact=cpd)
                if self.fold:
                    self.wgrad(blk.proj, x, gcur, hi, mode_x=1, c_x=self.cf(b1))
                else:
                    self.wgrad(blk.proj, self.ax[i], gcur, hi)
            # conv1: dz1 = (dgrad(dh1) [+ projection dgrad]) masked by BN1(x); g_in = BN1-backward(dz1, x) [+ g]
            dz1 = self.tmp("dz1", hi, cin)
            self.conv(c1, dh1, dz1, hi, mode=0, epi=6 | (1 if pd is not None else 0) | (8 if cpd else 0), res=pd,
                      xm=x, c_ep=self.cf(b1), st=self.sb(b1), dgrad=True)
            self.bn_final(b1, hi, True)
            if self.fold or self._fold1(i):
                self.wgrad(c1, x, dh1, hi, mode_x=1, c_x=self.cf(b1))
            else:
                self.wgrad(c1, self.ax[i], dh1, hi)
            gnext = self.tmp("gA" if (i % 2 == 0) else "gB", hi, cin)
            if self._gfold(i):
                gpend = (dz1, x, self.cb(b1), None if blk.proj is not None else gcur)
            else:
                self.ew(bwd, x, gnext, self.cb(b1), hi, cin, dz=dz1, add=None if blk.proj is not None else gcur)
            gcur = gnext
        # ---- stem: max-pool backward, stem wgrad (padded input, 3 real channels)
        dy0 = self.tmp("dy0", H1, cfg.num_filters)
        self.maxpool_bwd(gcur, dy0, H1, H2)
        self.wgrad(prog.stem, self.xin8, dy0, H, mode_x=0, mode_dy=0)
        self.det_finish()
        self._add("optim", None)
        self._add("step", None)

    def _build_eval(self):
        """Forward-only launch list of an eval chunk (resnet_run_loop.py:463-466): padded stem / dense weights of the
        evaluated members, BN coefficients from the moving statistics (cg_bn_final mode 2), the training forward
        kernels with their statistic epilogues drained into a sink, GAP, dense GEMM and a gradient-free
        softmax-CE that only counts loss / correct predictions."""
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        L = ops.lib()
        N, H = self.N, self.H
        ns = len(self.slots)
        sink = self.ev_sink
        self.prep_weights()
        for b in range(len(prog.bns)):
            hw = 1  # the eval coefficients do not depend on the spatial size
            self.bn_final(b, hw, 2)
        self.prep_input()
        H1, H2 = H // 2, self.xs[0].shape[1]
        self.conv(prog.stem, self.xin8, self.y0, H, mode=0, epi=0)
        self.maxpool(self.y0, self.xs[0], H1, H2)
        relu = L.dtf_cg_bn_relu_apply
        for i, blk in enumerate(prog.blocks):
            hi, ho, cin, f, fout = self.geo[i]
            b1, b2, b3 = blk.bns
            c1, c2, c3 = blk.convs
            x = self.xs[i]
            self.ew(relu, x, self.ax[i], self.cf(b1), hi, cin)
            if blk.proj is not None:
                self.conv(blk.proj, self.ax[i], self.sc[i], hi, mode=0, epi=0)
            self.conv(c1, self.ax[i], self.h1[i], hi, mode=0, epi=4, st=sink)
            self.ew(relu, self.h1[i], self.a1[i], self.cf(b2), hi, f)
            self.conv(c2, self.a1[i], self.h2[i], hi, mode=0, epi=4, st=sink)
            self.ew(relu, self.h2[i], self.a2[i], self.cf(b3), ho, f)
            res = self.sc[i] if blk.proj is not None else x
            self.conv(c3, self.a2[i], self.xs[i + 1], ho, mode=0, epi=5, res=res, st=sink)
        fb = prog.final_bn
        HL = self.HL
        g = GapArgs()
        g.x, g.coef, g.img_slot, g.feat = _p(self.xs[-1]), _p(self.cf(fb)), _p(self.img_slot), _p(self.feat)
        g.dfeat, g.sums, g.bcoef = _p(self.dfeat), _p(sink), _p(self.cf(fb))
        g.hw, g.C, g.cmax = HL * HL, cfg.final_size, CMAX
        self._hold(g)
        self.gap(g, 0)
        self.dense_head(False)

    # ------------------------------------------------------------------------------------ ResNet v1 program
    def bn_add_relu(self, h, s, out, coef_h, coef_s, hw, C):
        """v1 block output: out = relu(BN3(h) + (BN_p(s) if coef_s else s))."""
        a = BnAddArgs()
        a.h, a.s, a.out, a.coef_h, a.coef_s = _p(h), _p(s), _p(out), _p(coef_h), _p(coef_s)
        a.img_slot, a.hw, a.C, a.cmax, a.nimg = _p(self.img_slot), hw * hw, C, CMAX, self.N
        self._hold(a)
        self._add(ops.lib().dtf_cg_bn_add_relu, ctypes.byref(a))

    def bwd_sums(self, dz, h, bn, hw, C, h2=None, bn2=None):
        """sum dz, sum dz * xhat of the post-activation BN `bn` (input h) [and of `bn2` (input h2), same dz]."""
        a = BnSumArgs()
        a.dz, a.h, a.h2 = _p(dz), _p(h), _p(h2)
        a.fc, a.sums = _p(self.cf(bn)), _p(self.sb(bn))
        if bn2 is not None:
            a.fc2, a.sums2 = _p(self.cf(bn2)), _p(self.sb(bn2))
        a.img_slot, a.hw, a.C, a.cmax = _p(self.img_slot), hw * hw, C, CMAX
        self._hold(a)
        self._add(ops.lib().dtf_cg_bn_bwd_sums, ctypes.byref(a), self.N)

    def _forward_v1(self, sink=None):
        """Forward of the v1 bottleneck net (reference resnet_model.py:215-264, 504-510): stem conv -> BN -> ReLU ->
        max-pool; per block conv -> BN -> ReLU twice, conv -> BN, + shortcut (identity, or projection conv -> BN),
        ReLU; no final BN.  Training: statistics epilogues + bn_final per BN; eval (``sink``): every BN's
        coefficients come from the moving statistics (bn_final mode 2, issued by the caller)."""
        be, prog, cfg = self.be, self.be.prog, self.be.cfg
        L = ops.lib()
        N, H = self.N, self.H
        H1, H2 = H // 2, self.xs[0].shape[1]
        train = sink is None
        relu = L.dtf_cg_bn_relu_apply
        sb = prog.stem_bn
        self.conv(prog.stem, self.xin8, self.y0, H, mode=0, epi=4, st=self.sf(sb) if train else sink)
        if train:
            self.bn_final(sb, H1, False)
        self.ew(relu, self.y0, self.a0, self.cf(sb), H1, cfg.num_filters)
        self.maxpool(self.a0, self.xs[0], H1, H2)
        for i, blk in enumerate(prog.blocks):
            hi, ho, cin, f, fout = self.geo[i]
            b1, b2, b3 = blk.bns
            c1, c2, c3 = blk.convs
            x = self.xs[i]
            if blk.proj is not None:
                self.conv(blk.proj, x, self.sc[i], hi, mode=0, epi=4, st=self.sf(blk.proj_bn) if train else sink)
            self.conv(c1, x, self.h1[i], hi, mode=0, epi=4, st=self.sf(b1) if train else sink)
            if train:
                self.bn_final(b1, hi, False)
            self.ew(relu, self.h1[i], self.a1[i], self.cf(b1), hi, f)
            self.conv(c2, self.a1[i], self.h2[i], hi, mode=0, epi=4, st=self.sf(b2) if train else sink)
            if train:
                self.bn_final(b2, ho, False)
            self.ew(relu, self.h2[i], self.a2[i], self.cf(b2), ho, f)
            self.conv(c3, self.a2[i], self.h3[i], ho, mode=0, epi=4, st=self.sf(b3) if train else sink)
            if train:
                self.bn_final(b3, ho, False)
                if blk.proj is not None:
                    self.bn_final(blk.proj_bn, ho, False)
            if blk.proj is not None:
                self.bn_add_relu(self.h3[i], self.sc[i], self.xs[i + 1], self.cf(b3), self.cf(blk.proj_bn), ho, fout)
            else:
                self.bn_add_relu(self.h3[i], x, self.xs[i + 1], self.cf(b3), None, ho, fout)

    def _build_v1(self):
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        L = ops.lib()
        N, H = self.N, self.H
        ns = len(self.slots)
        self.prep_weights()
        self._add("zero", be.sums)
        self._add("zero", be.loss)
        self._add("zero", be.correct)
        self.prep_input()
        self._forward_v1()
        H1, H2, HL = H // 2, self.xs[0].shape[1], self.HL
        C = cfg.final_size
        # GAP of the last block output (already a ReLU output: no final BN in v1), dense, softmax CE
        g = GapArgs()
        g.x, g.coef, g.img_slot, g.feat = _p(self.xs[-1]), None, _p(self.img_slot), _p(self.feat)
        g.dfeat, g.sums, g.bcoef = _p(self.dfeat), None, None
        g.hw, g.C, g.cmax = HL * HL, C, CMAX
        self._hold(g)
        self.gap(g, 0)
        self.dense_head(True)
        # GAP backward: the gradient at the last block output, masked by its ReLU (cg_gap_bwd_apply, coef = null)
        gz = self.tmp("gA" if (len(prog.blocks) % 2 == 0) else "gB", HL, C)
        g2 = GapArgs()
        ctypes.memmove(ctypes.addressof(g2), ctypes.addressof(g), ctypes.sizeof(GapArgs))
        g2.out = _p(gz)
        self._hold(g2)
        self.gap(g2, 2)
        bwd = L.dtf_cg_bn_bwd_apply
        # ---- blocks, reversed.  gz = dL/d(BN3(h3) + shortcut), already ReLU-masked (by the GAP backward, or by the
        # next block's conv1 data-gradient epilogue)
        for i in range(len(prog.blocks) - 1, -1, -1):
            blk = prog.blocks[i]
            hi, ho, cin, f, fout = self.geo[i]
            b1, b2, b3 = blk.bns
            c1, c2, c3 = blk.convs
            x, h1, h2, h3 = self.xs[i], self.h1[i], self.h2[i], self.h3[i]
            pbn = blk.proj_bn
            # BN3 (and the projection BN: same dz) backward sums -> coefficients; dh3 = A3 gz + B3 h3 + C3
            self.bwd_sums(gz, h3, b3, ho, fout, h2=self.sc[i] if pbn is not None else None, bn2=pbn)
            self.bn_final(b3, ho, True)
            dh3 = self.tmp("dh3", ho, fout)
            self.ew(bwd, h3, dh3, self.cb(b3), ho, fout, dz=gz)
            ds = None
            if pbn is not None:
                self.bn_final(pbn, ho, True)
                ds = self.tmp("ds", ho, fout)
                self.ew(bwd, self.sc[i], ds, self.cb(pbn), ho, fout, dz=gz)
            # conv3: dz2 = dgrad(dh3) masked by relu(BN2(h2)) + BN2 backward sums
            dz2 = self.tmp("dz3", ho, f)
            self.conv(c3, dh3, dz2, ho, mode=0, epi=6, xm=h2, c_ep=self.cf(b2), st=self.sb(b2), dgrad=True)
            self.bn_final(b2, ho, True)
            dh2 = self.tmp("dh2", ho, f)
            self.ew(bwd, h2, dh2, self.cb(b2), ho, f, dz=dz2)
            self.wgrad(c3, self.a2[i], dh3, ho)
            # conv2 (3x3 / s): dz1 = dgrad(dh2) masked by relu(BN1(h1)) + BN1 sums
            dz1 = self.tmp("dz2", hi, f)
            self.conv(c2, dh2, dz1, ho, mode=0, epi=6, xm=h1, c_ep=self.cf(b1), st=self.sb(b1), dgrad=True)
            self.bn_final(b1, hi, True)
            dh1 = self.tmp("dh1", hi, f)
            self.ew(bwd, h1, dh1, self.cb(b1), hi, f, dz=dz1)
            self.wgrad(c2, self.a1[i], dh2, hi)
            res = gz
            if blk.proj is not None:
                res = self.tmp("pd", hi, cin)
                self.conv(blk.proj, ds, res, ho, mode=0, epi=0, dgrad=True)
                self.wgrad(blk.proj, x, ds, hi)
            # conv1: g = dgrad(dh1) + shortcut gradient, masked by the block input's ReLU (x > 0) -> the previous
            # block's gz (block 0: the pooled stem activation's)
            gnext = self.tmp("gA" if (i % 2 == 0) else "gB", hi, cin)
            self.conv(c1, dh1, gnext, hi, mode=0, epi=3, res=res, xm=x, c_ep=be.ident, dgrad=True)
            self.wgrad(c1, x, dh1, hi)
            gz = gnext
        # ---- stem: max-pool backward (gz is masked by the pooled ReLU output > 0), BN_stem backward, stem wgrad
        sbn = prog.stem_bn
        dz0 = self.tmp("dz0", H1, cfg.num_filters)
        self.maxpool_bwd(gz, dz0, H1, H2)
        self.bwd_sums(dz0, self.y0, sbn, H1, cfg.num_filters)
        self.bn_final(sbn, H1, True)
        dy0 = self.tmp("dy0", H1, cfg.num_filters)
        self.ew(bwd, self.y0, dy0, self.cb(sbn), H1, cfg.num_filters, dz=dz0)
        self.wgrad(prog.stem, self.xin8, dy0, H, mode_x=0, mode_dy=0)
        self.det_finish()
        self._add("optim", None)
        self._add("step", None)

    def _build_eval_v1(self):
        be, e, prog, cfg = self.be, self.e, self.be.prog, self.be.cfg
        L = ops.lib()
        N, H = self.N, self.H
        ns = len(self.slots)
        self.prep_weights()
        for b in range(len(prog.bns)):
            self.bn_final(b, 1, 2)
        self.prep_input()
        self._forward_v1(sink=self.ev_sink)
        HL, C = self.HL, cfg.final_size
        g = GapArgs()
        g.x, g.coef, g.img_slot, g.feat = _p(self.xs[-1]), None, _p(self.img_slot), _p(self.feat)
        g.hw, g.C, g.cmax = HL * HL, C, CMAX
        self._hold(g)
        self.gap(g, 0)
        self.dense_head(False)

    def load_eval(self, x, y):
        """The same eval images for every member: [m, H, W, C] fp32 -> this plan's [members * m] input."""
        m, k = x.shape[0], len(self.slots)
        assert all(n == m for n in self.sizes)
        shp = tuple(self.x_in.shape[1:])
        self.x_in.view(k, m, *shp).copy_(x.reshape(1, m, *shp).expand(k, *([-1] * (len(shp) + 1))))
        self.labels.view(k, m).copy_(y.reshape(1, m).expand(k, -1))

    def run_eval(self):
        assert self.eval
        self._run_eager()

    # ----------------------------------------------------------------------------------------- execution
    def load_batch(self, batches):
        if same_batches(self, batches):
            return
        off = 0
        for (x, y) in batches:
            n = x.shape[0]
            self.x_in[off:off + n].copy_(x.reshape(n, *self.x_in.shape[1:]), non_blocking=True)
            self.labels[off:off + n].copy_(y, non_blocking=True)
            off += n

    def _run_eager(self):
        e = self.e
        st = ops.stream()
        for fn, args in self.launches:
            if fn == "zero":
                args[0].zero_()
            elif fn == "gemm":
                args[0].launch(st)
            elif fn == "optim":
                e.dp_sync_grads(self.slots)  # data-parallel member groups only (no-op otherwise)
                ops.fused_optimizer(e.state, e.grads, e.hyper, e.Pp, e.P, e.n_reg, shadow=self.be.shadow,
                                    zero_grads=True, grad_scale=1.0 / self.be.loss_scale)
            elif fn == "step":
                # step counters + per-member losses gathered inside the step (graph): a replay leaves one copy
                advance_steps(e, self.slots_long, self.slots_t, self.be.loss, self.loss_sel)
            else:
                err = fn(*args, st)
                if err != 0:
                    raise RuntimeError("kernel launch %s failed with %d" % (getattr(fn, "__name__", fn), err))

    def run(self):
        run_captured(self)


HipImageNetBackend._plan_cls = _ImageNetPlan
