"""Population-batched ResNet v2 (CIFAR shape) training step on hand-written gfx950 kernels.

One optimizer step of EVERY resident member is a fixed sequence of ~200 kernel
launches over population-packed NHWC bf16 tensors (images of all members
concatenated along N, ``img_slot`` maps image -> member row):

  weight_prep  fp32 master rows -> bf16 OHWI (forward) + IHWO (dgrad) layouts
  memset       BN statistic accumulators, loss
  prep_input   fp32 NHWC images -> bf16, channels padded 3 -> 16
  stem         conv_fwd (no input BN)                           -> x0, stats(x0)
  per block    [proj conv_fwd 1x1 (BN1+ReLU prologue)]          -> sc
               conv_fwd 3x3 (BN1+ReLU prologue)                 -> h,  stats(h)
               conv_fwd 3x3 (BN2+ReLU prologue, + residual)     -> x', stats(x')
  head         final BN+ReLU, GAP, dense, softmax-CE, dense grads, BN-final reductions
  bn_running   moving averages of every BN of every member
  backward     head_bwd_apply -> g_L; per block (reverse): conv_b dgrad (+relu mask, BN2 reductions),
               conv_b wgrad, [proj dgrad + wgrad], conv_a dgrad (BN2-backward prologue, relu mask,
               BN1 reductions), conv_a wgrad, bn_bwd_apply (+ identity residual) -> g_{l}; stem wgrad
  optimizer    one fused launch over all members (engine/optim.py semantics), zeroes grads

The whole sequence is captured once per batch composition into a HIP graph
(``torch.cuda.CUDAGraph``) and replayed; the Python orchestration below runs
only at capture time.  BN statistics use 8 replicated accumulators per member
(see ops/csrc/conv.hip).
"""

from __future__ import annotations

import ctypes
import os
import weakref
from typing import Dict, List, Sequence, Tuple

import torch

from .. import ops
from ..data.datasets import IndexBatch, batch_len
from ..models.resnet import BN_EPS

def _nrep() -> int:
    """BN statistic replicas, as compiled into the loaded library (common.h DTF_NREP; 64 in the deterministic
    build)."""
    return ops.build_nrep()


DET_WG_PER_MEMBER = 64  # deterministic mode: statistic-producing launches use <= this many workgroups per member
# Work-split constants of the step plans (each the winner of an A/B in profiles/; the losing variants were deleted)
DUAL_MAX_POP = 2          # dual (dgrad | wgrad role) backward launches up to this many members per GPU ...
DUAL_CS = (32, 64)        # ... for these channel widths (C = 16 keeps the fused kernel)
DUAL_WG = {16: 128, 32: 128, 64: 64}  # wgrad-role workgroups per member of a dual launch
# small populations: every layer's wgrad deferred past the dgrad chain (1) or run by the dual launches (0: C = 32 / 64
# dual, C = 16 fused -- the round-2 form, kept as an A/B switch)
SMALL_DEFER = os.environ.get("DTF_SMALL_DEFER", "1") == "1"
FWD_ITERS_PER_WG = int(os.environ.get("DTF_FWD_ITERS", "4"))  # forward: (image, band) iterations per workgroup (>= FWD_MIN_WG workgroups kept;
# ... per channel width: C = 64 (the 8x8 stage: one band per image) at 2 -- pop 8 3.006 -> 2.989 ms, 512 workgroups of
# 2 images instead of 256 of 4 (1: +1.2 %; C = 32 at 2: +0.5 %; profiles/r6_fwd_iters_per_width_ab.log)
FWD_ITERS_C = {64: 2}
# ... and C = 16 (32x32, 4 bands per image) at no more than 512 workgroups: 8 iterations at pop 8 (3.020 -> 2.999 ms,
# ResNet-110 -0.4 %), unchanged at pop <= 4 (a flat 8 cost pop 4 +3 %: 256 workgroups; profiles/r6_fwd_iters16_ab.log)
FWD_WG_TARGET = {16: int(os.environ.get("DTF_FWD_WG16", "512"))}
FWD_ITERS_C.update({c: int(os.environ["DTF_FWD_ITERS%d" % c]) for c in (16, 32, 64) if "DTF_FWD_ITERS%d" % c in os.environ})
FWD_MIN_WG = 256          # 512 for up to DUAL_MAX_POP members: pop 1 1.059 -> 1.055, pop 2 1.427 -> 1.398 ms)
FWD_MIN_WG_SMALL = 512
FWD_RESIDENT = int(os.environ.get("DTF_FWD_RESIDENT", "0"))  # stride-1 forward: one round of resident workgroups
HEAD_ITEMS = 512          # head / GAP+dense+CE work items
WGRAD_WG_PER_MEMBER = 128  # standalone wgrad launches: workgroups per member (bounds the dW partial traffic)
DENSE_REDUCE_BLOCKS = 256  # slab_reduce_all, dense jobs: max 32-element blocks per job
# slab_reduce_all, conv slab jobs: at most this many 256-element blocks per (job, member) -- each loops over the
# job's chunks (0: one block per chunk, the round-5 form)
SLAB_X_BLOCKS = int(os.environ.get("DTF_SLAB_X_BLOCKS", "0"))  # 16 / 32 measured flat (profiles/r6_slab_xblocks_ab.log)
FUSED_SLAB_BYTES = {16: 16e6, 32: 16e6, 64: 48e6}  # fused backward: per-launch dW slab budget -> workgroup count
FUSED_MIN_WG = int(os.environ.get("DTF_FUSED_MIN_WG", "256"))  # ... at least this many workgroups (one member would leave CUs idle otherwise)
FUSED_MAX_WG = {32: 128}  # ... at most this many per member (C = 32: fewer, fuller workgroups)
# ... and at most this many per launch (C = 16 at pop 8: 512 workgroups of 8 bands, 3.111 -> 3.091 ms; a 64-per-
# member cap instead costs pop 4 +3.9 %: profiles/r4_fwd_wg_ab.txt)
# C = 32 at 8+ members: 256 (one workgroup of 8 bands per CU; half the dW slab bytes): pop 8 3.18 -> 3.11 ms;
# pop 4 keeps its 512 (256 there: +0.4 %)
FUSED_TOTAL_MAX = {16: int(os.environ.get("DTF_FUSED_TOTAL16", "512")),
                   32: int(os.environ.get("DTF_FUSED_TOTAL32", "256"))}
FUSED_TOTAL_MIN_POP = {16: 1, 32: 8}  # populations from which the per-launch cap applies
# ... and never a partial second round of workgroups: a count above the resident slots (CUs x WGs per CU of the
# kernel's occupancy) is rounded down to a multiple of them (pop 8, C = 16: 1024 -> 768 workgroups of 6 bands
# instead of 768 + a 256-workgroup tail at a third of the occupancy)
FUSED_RESIDENT = int(os.environ.get("DTF_FUSED_RESIDENT", "1"))
FUSED_ROUNDS = int(os.environ.get("DTF_FUSED_ROUNDS", "1"))  # > 0: at most this many rounds of resident workgroups
N_CU = None  # compute units: the device's (256 on MI355X; 256 without a GPU)


def _n_cu():
    global N_CU
    if N_CU is None:
        N_CU = 256
        if torch.cuda.is_available():
            N_CU = max(1, torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
    return N_CU


def _fused_wgs_per_cu(C, mode_dy):
    """Workgroups per CU of conv_bwd_fused_kernel<C, mode_dy> (conv.hip FUSED_WAVES, 4 waves per workgroup)."""
    if C <= 16:
        return _lib_knob("dtf_fused16_m2_waves") if mode_dy != 3 else _lib_knob("dtf_fused16_m3_waves")
    return 2 if C <= 32 else 1
_KNOBS = {}


def _lib_knob(name):
    """A compile-time knob of conv.hip as built into the loaded library (DTF_FUSED16_WLDS / DTF_FUSED16_M3_WAVES):
    the launch geometry (dynamic LDS, workgroups per CU) must follow the kernel that runs, not the environment."""
    if name not in _KNOBS:
        _KNOBS[name] = int(getattr(ops.lib(), name)())
    return _KNOBS[name]


PIGGYBACK_MAX_WG = 3000   # slab reductions ride on the next backward launch when they add <= this many workgroups
DEFER_WG = {16: 64, 32: 32, 64: 16}  # deferred wgrad (small populations): workgroups per member and layer
# deferred wgrad launches issued on a side stream (a parallel branch of the step graph) as soon as a stage's layers
# -- or OVERLAP_CHUNK of them -- are queued, so they run under the serial dgrad chain of the earlier stages instead
# of as a tail after it.  Off by default: the two-branch step graph measured SLOWER (pop 1: 1.051 -> 1.272 ms, stage
# chunks 1.394 ms; pop 2: 1.389 -> 1.577 ms; profiles/r4_wg_overlap_ab.log) -- the branch's cross-stream
# dependencies cost more than the idle CUs it fills
WG_OVERLAP = os.environ.get("DTF_WG_OVERLAP", "0") == "1"  # measured slower: profiles/r4_wg_overlap_ab.log
OVERLAP_CHUNK = int(os.environ.get("DTF_WG_OVERLAP_CHUNK", "0"))  # 0: stage boundaries only
DEFER_MID_POP = int(os.environ.get("DTF_DEFER_MID_POP", "4"))  # up to this many members: defer the wgrad of DEFER_MID_CS ...
DEFER_MID_CS = (32, 64)
DEFER_LARGE_CS = (64,)    # larger populations defer the wgrad of these channel widths only ...
DEFER_LARGE_WG = {16: 16, 32: int(os.environ.get("DTF_DEFER32_WG", "8")),
                  64: int(os.environ.get("DTF_DEFER64_WG", "8"))}  # ... with this many workgroups per member and layer
DEFER_ATOMIC = os.environ.get("DTF_DEFER_ATOMIC", "0") == "1"  # deferred wgrad jobs: fp32 atomics instead of dW slabs
DEFER_ATOMIC_CS = tuple(int(c) for c in os.environ.get("DTF_DEFER_ATOMIC_CS", "16,32,64").split(",") if c)
V1_CHAIN_BN = os.environ.get("DTF_V1_CHAIN_BN", "1") == "1"  # v1: BN_b backward sums in the next conv_a epilogue
# small populations: each stage's run of stride-1 forward convs in one persistent launch with a software grid
# barrier between layers instead of a kernel boundary (conv_fwd_s1_persist_kernel); up to PERSIST_MAX_POP members
PERSIST_FWD = os.environ.get("DTF_PERSIST_FWD", "0") == "1"
PERSIST_MAX_POP = int(os.environ.get("DTF_PERSIST_MAX_POP", "2"))
PERSIST_FENCE = int(os.environ.get("DTF_PERSIST_FENCE", "0"))  # conv.hip persist_barrier fence bits
HALF_BANDS_MAX_IMGS = 128  # C = 64 stage (8x8): 4-row half-image bands for the forward / dgrad launches up to this many
#                            images per step (one member: whole-image items left half the CUs idle; pop 2 and the
#                            C = 32 stage are slower with half bands: profiles/r3_half_bands_ab.log)
DG_ITERS_LARGE = int(os.environ.get("DTF_DG_ITERS", "2"))  # ... and (image, band) iterations per dgrad workgroup (the weights load once per workgroup)
DG_MIN_WG = 512           # ... keeping at least this many dgrad workgroups
c_void_p, c_int, c_long = ctypes.c_void_p, ctypes.c_int, ctypes.c_long


class ConvArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("x2", c_void_p), ("dy", c_void_p), ("dy2", c_void_p), ("y", c_void_p),
        ("res", c_void_p), ("xm", c_void_p), ("w", c_void_p), ("w_mstride", c_long), ("w_off", c_long),
        ("grads", c_void_p), ("g_mstride", c_long), ("g_off", c_long), ("img_slot", c_void_p), ("work", c_void_p),
        ("params", c_void_p), ("p_mstride", c_long),
        ("in_gamma", c_int), ("in_beta", c_int), ("ep_gamma", c_int), ("ep_beta", c_int),
        ("x_gamma", c_int), ("x_beta", c_int),
        ("st_in", c_void_p), ("st_in_b", c_void_p), ("st_ep", c_void_p), ("st_x", c_void_p), ("st_out", c_void_p),
        ("cnt", c_void_p), ("Hi", c_int), ("Wi", c_int), ("Ho", c_int), ("Wo", c_int), ("rows", c_int),
        ("cin_real", c_int), ("slab", c_void_p),
        ("x3", c_void_p), ("xout", c_void_p), ("rslab", c_void_p), ("rtab", c_void_p), ("r_goff", c_long),
        ("r_c", c_int), ("r_nblk", c_int), ("n_main", c_int),
        ("u_items", c_int), ("u_chunk", c_int), ("u_per", c_int), ("u_pad", c_int),
    ]


class SlabJob(ctypes.Structure):
    _fields_ = [("slab", c_void_p), ("red", c_void_p), ("g_off", c_long), ("nmem", c_int), ("pad", c_int)]


class WorkGenDesc(ctypes.Structure):
    _fields_ = [("dst", c_void_p), ("red", c_void_p), ("per", c_int), ("bands", c_int), ("min_chunk", c_int),
                ("split", c_int), ("prop", c_int), ("pad", c_int)]


# elastic work tables deal their rows out in proportion to the members' batch sizes (resnet_aux.hip work_gen_kernel,
# prop = 1) instead of `per` rows per member; the deterministic build keeps the fixed split (its replay caps the
# workgroups per member)
ELASTIC_PROP = os.environ.get("DTF_ELASTIC_PROP", "1") == "1"


def elastic_rows(totals, per, min_chunk, prop):
    """Host mirror of work_gen_kernel: [(first row, rows, chunk)] per member for these iteration totals."""
    M = len(totals)
    R = per * M
    if prop and R > M:
        chunk = max(min_chunk, -(-sum(totals) // (R - M)), 1)
        out, r0 = [], 0
        for k, t in enumerate(totals):
            n = max(1, -(-t // chunk)) if k + 1 < M else R - r0
            out.append((r0, n, chunk))
            r0 += n
        return out
    return [(k * per, per, max(min_chunk, -(-t // per), 1)) for k, t in enumerate(totals)]


class DenseJob(ctypes.Structure):
    _fields_ = [("slab", c_void_p), ("red", c_void_p), ("g_off", c_long), ("kel", c_int), ("nmem", c_int)]


class BnBwdArgs(ctypes.Structure):
    _fields_ = [
        ("dz", c_void_p), ("x", c_void_p), ("add", c_void_p), ("out", c_void_p), ("img_slot", c_void_p),
        ("params", c_void_p), ("p_mstride", c_long), ("gamma_off", c_int), ("st_f", c_void_p), ("st_b", c_void_p),
        ("cnt", c_void_p), ("hw", c_int), ("C", c_int), ("nimg", c_long),
    ]


class BnEwArgs(ctypes.Structure):
    _fields_ = [
        ("h1", c_void_p), ("h2", c_void_p), ("add", c_void_p), ("out", c_void_p), ("d", c_void_p),
        ("img_slot", c_void_p), ("params", c_void_p), ("p_mstride", c_long),
        ("g1", c_int), ("b1", c_int), ("g2", c_int), ("b2", c_int),
        ("st1", c_void_p), ("st2", c_void_p), ("sb1", c_void_p), ("sb2", c_void_p), ("cnt", c_void_p),
        ("hw", c_int), ("C", c_int), ("nimg", c_long), ("cap", c_int), ("pad_", c_int), ("slab", c_void_p),
    ]


class HeadArgs(ctypes.Structure):
    _fields_ = [
        ("x", c_void_p), ("labels", c_void_p), ("work", c_void_p), ("params", c_void_p), ("p_mstride", c_long),
        ("gamma_off", c_int), ("beta_off", c_int), ("dw_off", c_int), ("db_off", c_int), ("grads", c_void_p),
        ("g_mstride", c_long), ("st_f", c_void_p), ("st_b", c_void_p), ("cnt", c_void_p), ("dfeat", c_void_p),
        ("loss", c_void_p), ("correct", c_void_p), ("logits_out", c_void_p), ("hw", c_int), ("C", c_int),
        ("ncls", c_int), ("train", c_int), ("slab", c_void_p), ("slab_b", c_void_p), ("loss_scale", ctypes.c_float),
    ]


_REGISTERED = False


def _register():
    global _REGISTERED
    if _REGISTERED:
        return
    P = ctypes.POINTER
    ops.register("dtf_conv_fwd", [P(ConvArgs), c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_void_p])
    ops.register("dtf_conv_dgrad", [P(ConvArgs), c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_conv_wgrad", [P(ConvArgs), c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_conv_fwd_s1", [P(ConvArgs), c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_dw_slab_reduce", [c_void_p, c_void_p, c_int, c_void_p, c_long, c_long, c_int, c_void_p])
    ops.register("dtf_conv_bwd_fused", [P(ConvArgs), c_int, c_int, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_conv_bwd_dual", [P(ConvArgs), P(ConvArgs), c_int, c_int, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_conv_bwd_dg", [P(ConvArgs), c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_conv_wgrad_all", [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_conv_fwd_s1_persist", [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                             c_void_p, c_int, c_int, c_void_p])
    ops.register("dtf_slab_reduce_all", [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_long, c_void_p])
    ops.register("dtf_slab_job_size", [])
    ops.register("dtf_dense_job_size", [])
    ops.register("dtf_conv_args_size", [])
    ops.register("dtf_bnbwd_args_size", [])
    ops.register("dtf_head_args_size", [])
    ops.register("dtf_prep_input", [c_void_p, c_void_p, c_long, c_int, c_void_p])
    ops.register("dtf_weight_prep", [c_void_p, c_long, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_long,
                                     c_void_p, c_long, c_void_p])
    ops.register("dtf_bn_running_update", [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_long, c_void_p,
                                           c_int, c_void_p, c_void_p, c_long, c_void_p])
    ops.register("dtf_wpitch", [c_int])
    ops.register("dtf_cpad_fwd", [c_int])
    ops.register("dtf_conv_trans_multi", [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p])
    ops.register("dtf_work_gen", [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p])
    ops.register("dtf_workgen_desc_size", [])
    ops.register("dtf_bn_step_end", [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_void_p, c_long, c_void_p,
                                     c_int, c_void_p, c_void_p, c_long, c_void_p])
    ops.register("dtf_bn_eval_stats", [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_long, c_void_p, c_int,
                                       c_void_p, c_void_p])
    ops.register("dtf_bn_bwd_apply", [P(BnBwdArgs), c_void_p])
    ops.register("dtf_bn_add_relu", [P(BnEwArgs), c_void_p])
    ops.register("dtf_bn_bwd_reduce", [P(BnEwArgs), c_void_p])
    ops.register("dtf_bn_bwd_reduce_finish", [P(BnEwArgs), c_void_p, c_void_p, c_int, c_void_p])
    ops.register("dtf_bnew_args_size", [])
    ops.register("dtf_head", [P(HeadArgs), c_int, c_void_p])
    ops.register("dtf_head_bwd_apply", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int, c_int,
                                        c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p])
    L = ops.lib()
    # the library may have been loaded before these were registered: (re)bind signatures
    for name, args in ops._SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.argtypes = args
            fn.restype = c_int
    assert L.dtf_conv_args_size() == ctypes.sizeof(ConvArgs), "ConvArgs ABI mismatch"
    assert L.dtf_slab_job_size() == ctypes.sizeof(SlabJob), "SlabJob ABI mismatch"
    assert L.dtf_dense_job_size() == ctypes.sizeof(DenseJob), "DenseJob ABI mismatch"
    assert L.dtf_workgen_desc_size() == ctypes.sizeof(WorkGenDesc), "WorkGenDesc ABI mismatch"
    assert L.dtf_bnbwd_args_size() == ctypes.sizeof(BnBwdArgs), "BnBwdArgs ABI mismatch"
    assert L.dtf_head_args_size() == ctypes.sizeof(HeadArgs), "HeadArgs ABI mismatch"
    assert L.dtf_bnew_args_size() == ctypes.sizeof(BnEwArgs), "BnEwArgs ABI mismatch"
    _REGISTERED = True


def _cpad(c: int) -> int:
    """LDS pixel pitch (bf16 elements) of a C-channel tile: must match conv.hip ``cpad<C>()``."""
    return {16: 16, 32: 48, 64: 80}.get(c, c + 8)


_WPITCH = {}


def _wpitch(c: int) -> int:
    """LDS row pitch (pixels) of the stage kernels' C-channel tiles, as compiled into the loaded library."""
    if c not in _WPITCH:
        _WPITCH[c] = int(ops.lib().dtf_wpitch(c))
        assert _WPITCH[c] >= 512 // c + 2, ("unexpected LDS pitch", c, _WPITCH[c])
    return _WPITCH[c]


_CPAD_FWD = {}


def _cpad_fwd(c: int) -> int:
    """conv_fwd_s1 pitch (conv.hip ``cpad_fwd<C>()``), as compiled into the loaded library."""
    if c != 16:
        return _cpad(c)
    if c not in _CPAD_FWD:
        _CPAD_FWD[c] = int(ops.lib().dtf_cpad_fwd(c))
        assert _CPAD_FWD[c] >= c, ("unexpected LDS pitch", c, _CPAD_FWD[c])
    return _CPAD_FWD[c]


def _p(t):
    return None if t is None else t.data_ptr()


def _check(err, what):
    if err != 0:
        raise RuntimeError("%s: launch error %d (unsupported shape or HIP error)" % (what, err))


def _pick_rows(H, W, n_images, align, target_items=2048, max_rows=None):
    """Largest divisor R of H with R*W % align == 0 and n_images*(H/R) >= target (else smallest valid)."""
    cands = [r for r in range(1, H + 1) if H % r == 0 and (r * W) % align == 0]
    if max_rows:
        cands = [r for r in cands if r <= max_rows] or cands[:1]
    best = cands[0]
    for r in cands:
        if n_images * (H // r) >= target_items:
            best = r
    return best


class _Layout:
    """Static (per architecture) tables: conv / BN metadata and buffer offsets."""

    def __init__(self, engine):
        prog = engine.arch.prog
        cfg = prog.cfg
        if cfg.version not in (1, 2) or cfg.bottleneck or cfg.image_size != 32:
            raise ValueError("HIP ResNet backend supports CIFAR-shape v1/v2 building-block nets")
        self.prog = prog
        self.cfg = cfg
        convs = prog.convs
        # bf16 weight layouts: forward (OHWI, stem padded to 16 input channels) + dgrad (IHWO)
        self.fwd_off, self.dgr_off = {}, {}
        off = 0
        table = []
        for c in convs:
            cin_pad = 16 if c.idx == prog.stem else c.cin
            self.fwd_off[c.idx] = off
            off += c.cout * c.k * c.k * cin_pad
            if c.idx != prog.stem:
                self.dgr_off[c.idx] = off
                off += c.cout * c.k * c.k * c.cin
            table.append([c.off, c.cout, c.cin, c.k, cin_pad, self.fwd_off[c.idx], self.dgr_off.get(c.idx, -1), 0])
        self.wtot = (off + 63) // 64 * 64
        self.conv_table = table
        # spatial size of each BN's input
        self.bn_hw = {}
        hw = cfg.image_size
        if cfg.version == 1:
            self.bn_hw[prog.stem_bn] = hw * hw
        for blk in prog.blocks:
            hw_out = hw // blk.stride
            if cfg.version == 2:
                self.bn_hw[blk.bns[0]] = hw * hw
                self.bn_hw[blk.bns[1]] = hw_out * hw_out
            else:  # v1: every BN follows a conv at the block-output resolution
                for b in blk.bns + ([blk.proj_bn] if blk.proj_bn is not None else []):
                    self.bn_hw[b] = hw_out * hw_out
            hw = hw_out
        if cfg.version == 2:
            self.bn_hw[prog.final_bn] = hw * hw
        self.final_hw = hw * hw
        self.bn_table = [[b.run_off, b.c, self.bn_hw[b.idx], b.idx, b.gamma_off, b.beta_off, 0, 0] for b in prog.bns]


def upload_hyper(e, slots, hparams, lrs):
    """Per-member optimizer hyper rows -> device table, skipped when only the step counter moved (the lr
    schedule is piecewise constant).  The captured step advances the table's step column on the device
    (``advance_steps``) and ``e._hyper_dev`` mirrors what the device holds, so a skip is exact -- also after
    an exploit import changes a member's step."""
    from .optim import H_STEP, hyper_row
    rows = [(s, hyper_row(hp, lr, e.host_step[s] + 1, True)) for s, hp, lr in zip(slots, hparams, lrs)]
    dev = getattr(e, "_hyper_dev", None)
    if dev is not None and dev.get("slots") == tuple(slots) and all(dev.get(s) == r for s, r in rows):
        return
    hy = torch.zeros(e.capacity, 8, dtype=torch.float32)
    for s, r in rows:
        hy[s] = torch.tensor(r)
    e.hyper.copy_(hy.pin_memory() if e.device.type == "cuda" else hy, non_blocking=True)
    e._hyper_dev = {s: list(r) for s, r in rows}
    e._hyper_dev["slots"] = tuple(slots)


class PinnedStager:
    """Small per-step host->device uploads through one pinned staging buffer.

    A pageable ``non_blocking`` copy is staged synchronously and waits for the stream to drain, so the host
    cannot queue step k+1 while step k runs.  Here the host waits only for the previous upload from this stager
    (issued at the start of the previous step) before overwriting the staging buffer."""

    def __init__(self, n, dtype):
        self.host = torch.empty(n, dtype=dtype).pin_memory() if torch.cuda.is_available() else None
        self.evt = None

    def upload(self, dst, values):
        if dst.device.type != "cuda" or self.host is None:
            dst.copy_(torch.tensor(list(values), dtype=dst.dtype))
            return
        if self.evt is None:
            self.evt = torch.cuda.Event()
        else:
            self.evt.synchronize()
        for i, v in enumerate(values):
            self.host[i] = v
        dst.copy_(self.host[:len(values)], non_blocking=True)
        self.evt.record()


def note_step_advanced(e, slots):
    """Host mirror of ``advance_steps`` (call once per executed step)."""
    from .optim import H_STEP
    dev = getattr(e, "_hyper_dev", None)
    if dev is not None:
        for s in slots:
            if s in dev:
                dev[s][H_STEP] += 1.0


def advance_steps(e, slots_long, slots_i32=None, loss=None, loss_sel=None, ring=None):
    """Inside the captured step: per-member step counters (state column + hyper table) += 1 and, given
    ``loss``/``loss_sel``, the per-member losses gathered in slot-list order (one kernel when the int32 slot list is
    given).  ``ring`` = (rows [R, n] fp32, index int32 [1]): the losses go to the ring's next row instead of
    ``loss_sel`` (LossRing)."""
    from .optim import H_STEP
    if slots_i32 is not None and e.device.type == "cuda":
        rb, ri = (ring.rows, ring.idx) if ring is not None else (None, None)
        ops.check(ops.lib().dtf_step_end(_p(e.state), e.S, 3 * e.Pp + e.R, _p(e.hyper), H_STEP, _p(slots_i32),
                                         slots_i32.numel(), _p(loss), _p(loss_sel) if ring is None else None,
                                         _p(rb), _p(ri), rb.shape[0] if rb is not None else 0, ops.stream()),
                  "step_end")
        return
    one = torch.ones(slots_long.numel(), device=e.device)
    e.step_col().index_add_(0, slots_long, one)
    e.hyper[:, H_STEP].index_add_(0, slots_long, one)
    if loss_sel is not None:
        torch.index_select(loss, 0, slots_long, out=loss_sel)


class LossRing:
    """Per-step member losses without a per-step copy: the captured step's step_end kernel writes each replay's
    losses into the next row of a [rows, n] device ring (the row index lives on the device), and the host hands out
    a VIEW of that row.  A view stays valid for ``rows`` later steps; engine_model._train_cycle clones a member's
    last loss when the member leaves the active set (before its view can be overwritten)."""

    ROWS = 4096

    def __init__(self, n, device):
        self.rows = torch.zeros(self.ROWS, n, dtype=torch.float32, device=device)
        self.idx = torch.zeros(1, dtype=torch.int32, device=device)
        self.k = 0  # host mirror of idx: steps executed

    def advance(self):
        self.k += 1

    def last(self):
        assert self.k > 0
        return self.rows[(self.k - 1) % self.ROWS]


_LIVE_GRAPH_PLANS = weakref.WeakSet()  # plans holding a captured step graph (released before RCCL teardown)


def release_graphs() -> int:
    """Drop every captured step graph (they are re-captured on the next step).  A graph that recorded an RCCL
    collective keeps that communicator busy: ``destroy_process_group`` then blocks forever (measured with the
    data-parallel step on the GPU box), so ``parallel.comm.shutdown_distributed`` calls this first."""
    n = 0
    for plan in list(_LIVE_GRAPH_PLANS):
        if plan.graph is not None:
            plan.graph = None
            n += 1
    _LIVE_GRAPH_PLANS.clear()
    return n


def run_captured(plan) -> None:
    """Run one step of ``plan``: the first call executes it eagerly (allocator / lazy init warm-up) and then
    captures the launch list into a HIP graph; later calls replay the graph.  A data-parallel step captures its
    RCCL gradient all-reduce with the rest of the step; if this RCCL build refuses a collective inside a capture,
    the plan falls back to eager launches (the warm-up already ran this step)."""
    be = plan.be
    if be.use_graph and plan.graph is None and not getattr(plan, "_no_graph", False):
        plan._run_eager()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        ok = False
        try:
            with torch.cuda.stream(s):
                g.capture_begin(capture_error_mode="thread_local")
                try:
                    plan._run_eager()
                finally:
                    g.capture_end()
            ok = True
        except RuntimeError as err:
            if plan.e.dp is None:
                raise
            import sys
            import warnings
            msg = "step graph capture with the data-parallel all-reduce failed (%s): eager launches" % err
            warnings.warn(msg)
            print("DTF WARNING: " + msg, file=sys.stderr, flush=True)
            torch.cuda.synchronize()
            plan._no_graph = True
            be.graph_fallbacks = getattr(be, "graph_fallbacks", 0) + 1
        torch.cuda.current_stream().wait_stream(s)
        if ok:
            plan.graph = g
            be.graphs_captured = getattr(be, "graphs_captured", 0) + 1
            _LIVE_GRAPH_PLANS.add(plan)
        return
    if plan.graph is not None:
        plan.graph.replay()
    else:
        plan._run_eager()


def graph_state(be):
    """How a HIP backend's steps run: "captured" (HIP-graph replay), "eager_fallback" (a data-parallel capture was
    refused and at least one plan runs its launches eagerly -- slow, recorded in the bench JSON and metrics.jsonl),
    "disabled" (DTF_HIP_GRAPH=0 / debug), "none" (nothing captured yet), or None (not a HIP backend)."""
    if not hasattr(be, "use_graph"):
        return None
    if not be.use_graph:
        return "disabled"
    if getattr(be, "graph_fallbacks", 0):
        return "eager_fallback"
    return "captured" if getattr(be, "graphs_captured", 0) else "none"


def same_batches(plan, batches) -> bool:
    """True if ``batches`` are the very (x, y) storages staged last step and unmodified since (tensor version
    counters); a reference to them is held so their memory cannot be recycled into a different batch."""
    key = tuple((x.data_ptr(), x.shape, x.stride(), x._version, y.data_ptr(), y.shape, y._version)
                for x, y in batches)
    if getattr(plan, "_batch_key", None) == key:
        return True
    plan._batch_key = key
    plan._batch_ref = list(batches)
    return False


class HipResNetBackend:
    name = "hip"

    def __init__(self, engine):
        _register()
        self.e = engine
        self.dev = engine.device
        self.L = _Layout(engine)
        cap = engine.capacity
        self.wf = torch.zeros(cap, self.L.wtot, dtype=ops.act_dtype(), device=self.dev)
        self.wd = torch.zeros(cap, self.L.wtot, dtype=ops.act_dtype(), device=self.dev)
        nb = len(self.L.prog.bns)
        self.det = ops.build_deterministic()  # what the loaded library was compiled as
        # fp16 (the half build of the same kernels, ops.half_mode()): static loss scaling as the reference's fp16 mode
        # (resnet_run_loop.py:284-294) -- the head differentiates loss_scale * loss, the optimizer unscales
        self.half = ops.build_half()
        assert self.half == (engine.compute_dtype == torch.float16), \
            "the loaded kernel library (%s) does not match compute dtype %s: fp16 needs DTF_HALF=1" % (
                "fp16" if self.half else "bf16", engine.compute_dtype)
        self.loss_scale = float(engine.loss_scale) if self.half else 1.0
        NREP = self.nrep = _nrep()
        self.stats_bn_stride = cap * NREP * 128
        # [fwd | bwd] statistic accumulators: zeroed by ONE memset per step
        # [fwd | bwd] statistic accumulators + per-member loss / correct count: ONE buffer, zeroed by the step's
        # weight_prep launch
        nst = 2 * nb * cap * NREP * 128
        self.zbuf = torch.zeros(nst + 2 * cap, dtype=torch.float32, device=self.dev)
        self.stats = self.zbuf[:nst].view(2, nb, cap, NREP, 128)
        self.conv_table_t = torch.tensor(self.L.conv_table, dtype=torch.int32, device=self.dev)
        self.bn_table_t = torch.tensor(self.L.bn_table, dtype=torch.int32, device=self.dev)
        self.loss = self.zbuf[nst:nst + cap]
        self.correct = self.zbuf[nst + cap:]
        self._plans: Dict[tuple, "_StepPlan"] = {}
        self.use_graph = (os.environ.get("DTF_HIP_GRAPH", "1") == "1" and os.environ.get("DTF_DEBUG", "0") != "1")

    # --- engine hooks --------------------------------------------------------------
    def persist_failures(self) -> int:
        """Software grid barriers of the persistent forward segments that timed out (their step is wrong; 0 on a
        healthy run: every workgroup of such a launch is co-resident by construction).  Reads the device."""
        t = getattr(self, "persist_fail", None)
        return 0 if t is None else int(t.item())

    def on_params_changed(self, slots):
        pass  # weight_prep runs at the start of every step (inside the graph)

    def shadow_weights(self):
        return None

    def st_f(self, bn):
        return self.stats[0, bn]

    def st_b(self, bn):
        return self.stats[1, bn]

    # --- plans ------------------------------------------------------------------------
    accepts_index_batches = True

    def _elastic_cap(self, sizes, force=False):
        """Per-member capacity of an elastic plan for these batch sizes, or None for an exact plan.  Mixed batch
        sizes (PBT samples and perturbs them, constants.py:91-93) run on one capacity-keyed plan whose work tables
        are regenerated on the device every step (DTF_ELASTIC: "auto" = mixed sizes only (or ``force``: a
        shrinking active set), "1", "0")."""
        mode = os.environ.get("DTF_ELASTIC", "auto")
        cap = int(os.environ.get("DTF_ELASTIC_MAXB", "256"))
        if (mode == "0" or self.dev.type != "cuda" or self.e.dp is not None
                or max(sizes) > cap or (mode == "auto" and len(set(sizes)) == 1 and not force)):
            return None
        return cap

    def plan(self, slots: Sequence[int], sizes: Sequence[int], src=None) -> "_StepPlan":
        """The step plan (buffers + captured graph) for this batch composition.  Elastic plans are keyed on the
        capacity and the member set; a step of a SUBSET of an elastic plan's members (members that finished their
        epoch drop out of the active set: engine_model._train_cycle) replays that plan with zero images for the
        others -- their optimizer rows are inactive (hyper table), their step counters and BN moving statistics do
        not move (step_advance / bn_running_update) -- instead of building and capturing a new plan."""
        src_id = id(src) if src is not None else None
        shrink = self._covering_plan(slots, sizes, src_id)
        if shrink is not None:
            by = dict(zip(slots, sizes))
            shrink.set_sizes([by.get(s, 0) for s in shrink.slots])
            return shrink
        cap = self._elastic_cap(sizes) if sizes else None
        if cap is None and self._subset_of_known(slots, src_id):
            cap = self._elastic_cap(sizes, force=True)  # a shrinking active set: go elastic once, reuse after
        key = (tuple(slots), ("elastic", cap) if cap else tuple(sizes), src_id)
        p = self._plans.get(key)
        if p is None:
            if len(self._plans) > 16:
                self._plans.clear()
            p = _StepPlan(self, list(slots), list(sizes), src, elastic_cap=cap)
            self._plans[key] = p
        if cap:
            p.set_sizes(list(sizes))
        return p

    def _covering_plan(self, slots, sizes, src_id):
        """An elastic plan whose members strictly include ``slots`` (and whose capacity fits ``sizes``)."""
        want = set(slots)
        for key, p in self._plans.items():
            if (p.elastic and key[2] == src_id and want < set(p.slots) and sizes
                    and max(sizes) <= p.sizes[0]):
                return p
        return None

    def _subset_of_known(self, slots, src_id):
        want = set(slots)
        return any(key[2] == src_id and want < set(key[0]) for key in self._plans)

    def train_step(self, slots, batches, hparams, lrs):
        e = self.e
        src = None
        if all(isinstance(b, IndexBatch) for b in batches) and batches and all(b.ds is batches[0].ds
                                                                               for b in batches):
            src = batches[0].ds  # on-device gather + augmentation inside the step graph
        else:
            batches = [b.materialize() if isinstance(b, IndexBatch) else b for b in batches]
        sizes = [batch_len(b) for b in batches]
        p = self.plan(slots, sizes, src)
        upload_hyper(e, slots, hparams, lrs)
        if list(p.slots) != list(slots):  # a subset of an elastic plan's members (idle members: no images)
            by = dict(zip(slots, batches))
            p.load_batch([by[s] for s in p.slots if s in by], slots=list(slots))
        else:
            p.load_batch(batches)
        p.run(train=True)
        note_step_advanced(e, slots)
        if list(p.slots) != list(slots):
            return p.loss_view()[p.slot_index(slots)]
        return p.loss_view()

    def forward_backward(self, slots, batches):
        raise RuntimeError("HipResNetBackend runs whole steps: use train_step")

    def train_correct(self, slots):
        """Correct predictions of each member's last training batch (head kernel count; device tensor)."""
        return self.correct[torch.as_tensor(list(slots), dtype=torch.long, device=self.dev)]

    @torch.no_grad()
    def infer(self, slot, x):
        """Eval-mode logits of one member on the HIP forward kernels (moving BN statistics)."""
        p = self.eval_plan([slot], int(x.shape[0]))
        logits = p.want_logits()
        p.load_eval(x, torch.zeros(x.shape[0], dtype=torch.int32, device=x.device))
        p.run_eval()
        return logits.clone()

    def eval_plan(self, slots, m):
        key = (tuple(slots), int(m))
        plans = self.__dict__.setdefault("_eval_plans", {})
        p = plans.get(key)
        if p is None:
            if len(plans) > 8:
                plans.clear()
            p = _StepPlan(self, list(slots), [int(m)] * len(slots), None, eval_mode=True)
            plans[key] = p
        return p

    @torch.no_grad()
    def evaluate_population(self, slots, x, y, chunk=None):
        """Eval accuracy of every member in ``slots`` on (x, y) in one population-batched forward per chunk of
        ``chunk`` images (all members see the same chunk); one host sync at the end."""
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


class _StepPlan:
    """Buffers + prebuilt launch list for one batch composition (slots, per-member sizes)."""

    def __init__(self, be: HipResNetBackend, slots: List[int], sizes: List[int], src=None, eval_mode=False,
                 elastic_cap=None):
        self.be = be
        e = be.e
        self.e = e
        self.slots = slots
        # elastic plan: buffers / layout for elastic_cap images per member, the real sizes live in self.cnt and
        # the work tables are rebuilt from them on the device at the start of every step (work_gen_kernel)
        self.elastic = bool(elastic_cap) and not eval_mode
        self.real_sizes = list(sizes)
        if self.elastic:
            sizes = [int(elastic_cap)] * len(slots)
        self.sizes = sizes
        self._wgen = []
        self.eval = bool(eval_mode)
        self.persist_fwd = False  # (training plans of small populations may enable it below)
        dev = be.dev
        L = be.L
        prog = L.prog
        cfg = L.cfg
        N = sum(sizes)
        self.N = N
        img_slot = []
        self.first = {}
        for s, n in zip(slots, sizes):
            self.first[s] = len(img_slot)
            img_slot += [s] * n
        self.img_slot = torch.tensor(img_slot, dtype=torch.int32, device=dev)
        cnt = torch.zeros(e.capacity, dtype=torch.float32)
        for s, n in zip(slots, sizes):
            cnt[s] = float(n)
        self.cnt = cnt.to(dev)
        # uniform population: work items of the stage kernels computed from blockIdx (ConvArgs.u_items)
        self.uniform = (len(set(sizes)) == 1 and list(slots) == list(range(len(slots))) and not self.elastic
                        and not be.det)
        if self.elastic:
            for s, n in zip(slots, self.real_sizes):
                cnt[s] = float(n)
            self.cnt = cnt.to(dev)
            self.first_t = torch.tensor([self.first[s] for s in slots], dtype=torch.int32, device=dev)
            self._cnt_stage = None
        self.slots_t = torch.tensor(slots, dtype=torch.int32, device=dev)
        self.slots_long = torch.tensor(slots, dtype=torch.long, device=dev)
        self.loss_sel = torch.zeros(len(slots), dtype=be.loss.dtype, device=dev)
        self.ring = LossRing(len(slots), dev) if (dev.type == "cuda" and not eval_mode and len(slots) <= 1024) else None
        H = cfg.image_size
        self.x_in = torch.zeros(N, H, H, 3, dtype=torch.float32, device=dev)
        self.labels = torch.zeros(N, dtype=torch.int32, device=dev)
        self.xin16 = torch.zeros(N, H, H, 16, dtype=ops.act_dtype(), device=dev)
        self.src = src
        if src is not None:
            self.idx = torch.zeros(N, dtype=torch.long, device=dev)
            self.rng = torch.zeros(2, dtype=torch.int32, device=dev)
        self.v1 = cfg.version == 1
        # forward activations saved for backward (eval: nothing is saved -- per-resolution buffers are reused,
        # the residual stream ping-pongs between two)
        self.xs, self.hs, self.scs = [], [], []
        self.hb = []  # v1: conv_b outputs (pre-BN); hs = conv_a outputs, scs = projection outputs (pre-BN)
        self.h0 = torch.empty(N, H, H, cfg.num_filters, dtype=ops.act_dtype(), device=dev) if self.v1 else None
        pool = {}

        def act(kind, hw_, c_, i_=0):
            if not self.eval:
                return torch.empty(N, hw_, hw_, c_, dtype=ops.act_dtype(), device=dev)
            key = (kind, hw_, c_, i_ % 2 if kind == "x" else 0)
            if key not in pool:
                pool[key] = torch.empty(N, hw_, hw_, c_, dtype=ops.act_dtype(), device=dev)
            return pool[key]

        hw, c = H, cfg.num_filters
        self.xs.append(act("x", hw, c, 0))
        for bi, blk in enumerate(prog.blocks):
            ca = prog.convs[blk.convs[0]]
            hw_o = hw // blk.stride
            self.hs.append(act("h", hw_o, ca.cout))
            self.scs.append(act("sc", hw_o, ca.cout) if blk.proj is not None else None)
            self.xs.append(act("x", hw_o, ca.cout, bi + 1))
            if self.v1:
                self.hb.append(act("hb", hw_o, ca.cout))
            hw = hw_o
        if self.eval:
            nb = len(prog.bns)
            cap = e.capacity
            # moving statistics in accumulator form (bn_eval_stats) + a sink for the conv epilogues' statistics
            self.ev_stats = torch.zeros(nb, cap, be.nrep, 128, dtype=torch.float32, device=dev)
            self.ev_sink = torch.zeros(cap, be.nrep, 128, dtype=torch.float32, device=dev)
            self.ev_acc = torch.zeros(2, cap, dtype=torch.float32, device=dev)  # [correct, summed mean CE] per slot
            self.logits = None  # [N, ncls] fp32 when requested (tests)
            self._work_cache, self._uniform_geo = {}, {}
            self.launches = []
            self._pending_slab = None
            self._build_eval()
            self.graph = None
            return
        # backward temporaries, one set per resolution
        self.tmp = {}
        hw, c = H, cfg.num_filters
        for st in range(len(cfg.block_sizes)):
            if st > 0:
                hw //= 2
            cc = cfg.num_filters * (2 ** st)
            self.tmp[hw] = dict(g=[torch.empty(N, hw, hw, cc, dtype=ops.act_dtype(), device=dev) for _ in range(2)],
                                dz2=torch.empty(N, hw, hw, cc, dtype=ops.act_dtype(), device=dev),
                                dz1=torch.empty(N, hw, hw, cc, dtype=ops.act_dtype(), device=dev))
        self.pd = {}  # projection dgrad outputs at block-input resolution
        hw = H
        for blk in prog.blocks:
            if blk.proj is not None:
                ci = prog.convs[blk.proj].cin
                self.pd[id(blk)] = torch.empty(N, hw, hw, ci, dtype=ops.act_dtype(), device=dev)
            hw //= blk.stride
        self.dfeat = torch.zeros(N, cfg.final_size, dtype=torch.float32, device=dev)
        self._work_cache = {}
        self._uniform_geo = {}
        # Dual backward (small populations, <= DUAL_MAX_POP members): each stride-1 C = 32 / 64 conv's dgrad and wgrad
        # run as two workgroup roles of ONE launch (conv_bwd_dual_kernel); the layer costs max(dgrad, wgrad) instead
        # of their sum while the population leaves CUs idle (C = 16 keeps the fused kernel: its single-band work
        # items already fill the GPU; profiles/r2_dual_pop1_breakdown.txt)
        # (the deterministic build never switches kernel families with the population size: a member's reduction
        # order must not depend on how many members share its plan -- placement invariance, _work_iters)
        self.dual = dev.type == "cuda" and cfg.version == 2 and len(slots) <= DUAL_MAX_POP and not be.det
        # Deferred weight gradients (the same small populations): each stride-1 layer's backward launch runs only
        # its dgrad role -- the critical path, serialised by the BatchNorm statistics -- and the wgrad work of all
        # those layers runs afterwards in two wide launches (conv_wgrad_all_kernel: widths 64 + 32, width 16).
        # Their dY / x operands stay alive for the whole backward (per-block buffers instead of ping-pong ones).
        self.defer_wg = self.dual and SMALL_DEFER
        self.persist_fwd = (PERSIST_FWD and dev.type == "cuda" and len(slots) <= PERSIST_MAX_POP
                            and not self.be.det and not self.eval)
        self.overlap_wg = self.defer_wg and WG_OVERLAP and dev.type == "cuda"
        # channel widths whose stride-1 wgrad is deferred: every width at small populations; up to 4 members C = 32
        # and 64, at larger ones the C = 64 layers only (1 workgroup per CU of the fused kernel left the MFMA pipe
        # idle, and its 147 KB dW slab per workgroup cost more than re-reading dY / x once in the wide wgrad
        # launch; profiles/r3_defer_ab.log)
        v2gpu = dev.type == "cuda" and cfg.version == 2
        large = DEFER_MID_CS if (len(slots) <= DEFER_MID_POP and not be.det) else DEFER_LARGE_CS
        self.defer_cs = {16, 32, 64} if self.defer_wg else (set(large) if v2gpu and not self.dual else set())
        self._wg_jobs = {}  # (C, wgrad dY mode) -> [(ConvArgs, work table, grad offset)]
        self.launches = []
        self._pending_slab = None  # (slab ptr, reduce table, C, grad offset) of the last fused launch
        self._slab_flip = 0
        # C = 64 dW slabs reduced together by ONE launch after the backward (instead of 17 small reductions)
        self._deferred = []  # (slab, reduce table, grad offset, C): reduced by one launch per C after the backward
        # standalone wgrad launches (stem, projections, strided convs) write dense per-workgroup dW partials reduced
        # in one launch after the backward (no contended fp32 atomics; fixed order)
        self.wslab = dev.type == "cuda"
        self._deferred_dense = []
        self._build()
        assert self._pending_slab is None and not self._deferred and not self._deferred_dense, \
            "every dW slab must be reduced before the optimizer"
        if self.elastic:
            self._work_gen_launch()
        self.graph = None

    # -------------------------------------------------------------------- work lists
    def _work_iters(self, bands, n_wg, det_per=None):
        """(it0, nit, 0, slot) items over the flattened (image, band) iterations of each member.

        Deterministic build: ``n_wg`` is ignored -- every member gets exactly DET_WG_PER_MEMBER rows (empty ones,
        nit = 0, past its iterations), so a member's split into workgroups, the statistic replica each of its
        workgroups adds to (blockIdx % 64 = the row within the member) and the order its dW slabs are reduced in
        depend on its own batch size only: the step of a member is bitwise the same whichever members share its
        plan (a PBT run replays identically at any placement over ranks, tests/test_gpu_placement.py).
        ``det_per``: launches that produce no BatchNorm statistics (the deferred weight-gradient jobs) take that
        fixed number of rows per member instead (any population-independent count keeps the dW slab order a
        function of the member alone; 64 rows wrote 8x the slab bytes of the release plan at pop 8)."""
        det = self.be.det
        dper = (det_per or DET_WG_PER_MEMBER) if det else None
        key = ("it", bands, ("det", dper) if det else n_wg)
        w = self._work_cache.get(key)
        if w is None and self.elastic:
            per = dper if det else max(1, n_wg // max(1, len(self.slots)))
            w = self._elastic_table(per, bands, 1)
            self._work_cache[key] = w
        if w is None:
            items = []
            per_member = dper if det else max(1, n_wg // max(1, len(self.slots)))
            for s, n in zip(self.slots, self.sizes):
                total = n * bands
                f = self.first[s] * bands
                chunk = max(1, -(-total // per_member))
                for i in range(0, total, chunk):
                    items.append([f + i, min(chunk, total - i), 0, s])
                if det:  # pad to exactly per_member rows (empty rows point at the member's first iteration)
                    items += [[f, 0, 0, s]] * (per_member - -(-total // chunk))
                # uniform geometry (identical for every member when self.uniform): items, chunk, iterations
                geo = (-(-total // chunk), chunk, total)
            w = torch.tensor(items, dtype=torch.int32, device=self.be.dev)
            self._work_cache[key] = w
            self._uniform_geo[w.data_ptr()] = geo
        return w

    def _set_uniform(self, a, work):
        """Arithmetic work items (ConvArgs.u_*) for a _work_iters array when the population is uniform."""
        if self.uniform:
            a.u_items, a.u_chunk, a.u_per = self._uniform_geo[work.data_ptr()]
            assert a.u_items * len(self.slots) == work.shape[0]

    # ------------------------------------------------------------------ elastic plans
    def _elastic_table(self, per, bands, min_chunk, split=False):
        """A work table of `per` rows per member (x2 when split) filled on the device each step from the real batch
        sizes (work_gen_kernel; same split rule as _work_iters / _work_member, empty rows past a member's end)."""
        rows = 2 if split else 1
        host = []
        prop = int(ELASTIC_PROP and not self.be.det)
        layout = elastic_rows([n * bands for n in self.real_sizes], per, min_chunk, prop)
        for (s, n), (r0, nrows, chunk) in zip(zip(self.slots, self.real_sizes), layout):
            total, f = n * bands, self.first[s] * bands
            for j in range(nrows):
                st = j * chunk
                nit = min(chunk, total - st) if st < total else 0
                for z in range(rows):
                    host.append([f + st if nit > 0 else f, nit, z, s])
        assert len(host) == per * len(self.slots) * rows
        w = torch.tensor(host, dtype=torch.int32, device=self.be.dev)
        self._wgen.append((w, per, bands, min_chunk, int(split), prop))
        self.__dict__.setdefault("_wgen_params", {})[w.data_ptr()] = (per, bands, min_chunk)
        return w

    def _work_gen_launch(self):
        """First launch of an elastic step: regenerate every work table from the per-member sizes (self.cnt)."""
        descs = (WorkGenDesc * len(self._wgen))()
        red = getattr(self, "_elastic_red", {})
        for i, (w, per, bands, mc, sp, prop) in enumerate(self._wgen):
            # the slab-reduction table over this work table (one per member), rewritten with it every step
            descs[i] = WorkGenDesc(w.data_ptr(), _p(red.get(w.data_ptr())), per, bands, mc, sp, prop, 0)
        dt = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(self.be.dev)
        self._keep(dt)
        self.launches.insert(0, (ops.lib().dtf_work_gen, (_p(dt), len(self._wgen), _p(self.slots_t),
                                                          _p(self.first_t), len(self.slots), _p(self.cnt))))

    def set_sizes(self, sizes):
        """Elastic plan: the real per-member batch sizes of the next step (device cnt; read by the step graph)."""
        assert self.elastic and len(sizes) == len(self.slots) and max(sizes) <= self.sizes[0]
        if list(sizes) == self.real_sizes:
            return
        self.real_sizes = list(sizes)
        vals = [0.0] * self.e.capacity
        for s, n in zip(self.slots, sizes):
            vals[s] = float(n)
        if self._cnt_stage is None:
            self._cnt_stage = PinnedStager(self.e.capacity, torch.float32)
        self._cnt_stage.upload(self.cnt, vals)

    def _n_wg_iters(self, total_iters, per_wg=4, lo=256, hi=1024):
        """Enough (image, band) iterations per workgroup for the double-buffered pipeline,
        while keeping >= lo workgroups (fill 256 CUs) when the batch allows."""
        return self._det_cap(int(max(lo, min(hi, total_iters // per_wg))))

    def _det_cap(self, n_wg):
        """Deterministic mode: at most DET_WG_PER_MEMBER workgroups per member, so each statistic replica of a
        member receives at most one atomic add (onto zero) per launch."""
        if self.be.det:
            return min(n_wg, DET_WG_PER_MEMBER * len(self.slots))
        return n_wg

    def _head_work(self):
        """Head work items (img0, nimg, 0, slot).  Deterministic build: exactly DET_WG_PER_MEMBER items per member
        (empty ones past its images): each workgroup then adds its final-BN backward partial to its own statistic
        replica (the row within the member), its dense gradients go to its own slab (reduced in a fixed order),
        and its loss partial is rounded to 2^-16 (order-free sum) -- a member's head depends on its own batch only.
        (One workgroup per member serialised the pop-8 deterministic step: 627 us vs 34 us,
        profiles/r6_det_vs_release_kstats.txt.)"""
        if not self.be.det:
            return self._work_member(target_items=HEAD_ITEMS)
        if self.elastic:  # the device-generated table: `per` rows per member, empty ones past its images
            return self._work_member(target_items=DET_WG_PER_MEMBER * len(self.slots))
        key = ("head_det",)
        w = self._work_cache.get(key)
        if w is None:
            items = []
            per = DET_WG_PER_MEMBER
            for s, n in zip(self.slots, self.sizes):
                f = self.first[s]
                chunk = max(1, -(-n // per))
                rows = [[f + i, min(chunk, n - i), 0, s] for i in range(0, n, chunk)]
                items += rows + [[f, 0, 0, s]] * (per - len(rows))
            w = torch.tensor(items, dtype=torch.int32, device=self.be.dev)
            self._work_cache[key] = w
        return w

    def _work_member(self, target_items=256, min_chunk=1):
        key = ("m", target_items)
        w = self._work_cache.get(key)
        if w is None and self.elastic:
            w = self._elastic_table(max(1, target_items // max(1, len(self.slots))), 1, min_chunk)
            self._work_cache[key] = w
        if w is None:
            items = []
            per_member = max(1, target_items // max(1, len(self.slots)))
            for s, n in zip(self.slots, self.sizes):
                chunk = max(min_chunk, -(-n // per_member))
                f = self.first[s]
                for i in range(0, n, chunk):
                    items.append([f + i, min(chunk, n - i), 0, s])
            w = torch.tensor(items, dtype=torch.int32, device=self.be.dev)
            self._work_cache[key] = w
        return w

    # -------------------------------------------------------------------- launches
    def _base_args(self):
        be, e = self.be, self.e
        a = ConvArgs()
        a.img_slot = _p(self.img_slot)
        a.params = _p(e.state)
        a.p_mstride = e.S
        a.cnt = _p(self.cnt)
        a.w_mstride = be.L.wtot
        a.grads = _p(e.grads)
        a.g_mstride = e.Pp
        a.cin_real = 0
        return a

    def _bn(self, idx):
        b = self.be.L.prog.bns[idx]
        return b.gamma_off, b.beta_off

    def _add(self, fn, *args):
        if getattr(self, "_pseg", None):
            self._flush_pseg()  # a pending persistent forward segment precedes every other launch
        if getattr(self, "_grab", None) is not None:
            self._grab.append((fn, args))  # collected for a combined multi-role launch
            return
        self.launches.append((fn, args))

    def _pseg_add(self, a, cin, mode, resid, rows, nwg, lds):
        """Queue a conv_fwd_s1 launch into the pending persistent segment (same C / bands / workgroup count)."""
        seg = getattr(self, "_pseg", None)
        if seg and (seg[0][1], seg[0][4], seg[0][5]) != (cin, rows, nwg):
            self._flush_pseg()
            seg = None
        if not seg:
            self._pseg = seg = []
        seg.append((a, cin, mode, resid, rows, nwg, lds))

    def _flush_pseg(self):
        """Emit the pending segment: one persistent launch (2+ layers whose workgroups are all co-resident), else
        the ordinary per-layer launches."""
        seg, self._pseg = self._pseg, None
        lib = ops.lib()
        if not seg:
            return
        cin, rows, nwg = seg[0][1], seg[0][4], seg[0][5]
        lds = max(t[6] for t in seg)
        be = self.be
        if len(seg) >= 2:
            if getattr(be, "persist_fail", None) is None:
                be.persist_fail = torch.zeros(1, dtype=torch.int32, device=be.dev)
            # this segment's own arrival-flag words (conv.hip persist_barrier: [64 + b]): every launch of the segment
            # has the same workgroup count and barrier count, so its flags stay in lockstep across replays
            bar = torch.zeros(64 + 1024, dtype=torch.int32, device=be.dev)
            self._keep(bar)
            arr = (ConvArgs * len(seg))(*[t[0] for t in seg])
            tbl = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(be.dev)
            kinds = torch.tensor([0 if t[2] == 0 else (2 if t[3] else 1) for t in seg], dtype=torch.int32,
                                 device=be.dev)
            ok = lib.dtf_conv_fwd_s1_persist(_p(tbl), _p(kinds), len(seg), cin, rows, nwg, lds, _p(bar),
                                             _p(be.persist_fail), PERSIST_FENCE, 1, None)
            if ok == 1 and nwg <= 1024 and all(t[2] != 0 or rows == 8 for t in seg):
                self._keep(tbl)
                self._keep(kinds)
                self.launches.append((lib.dtf_conv_fwd_s1_persist,
                                      (_p(tbl), _p(kinds), len(seg), cin, rows, nwg, lds, _p(bar),
                                       _p(be.persist_fail), PERSIST_FENCE, 0)))
                self.persist_segments = getattr(self, "persist_segments", 0) + 1
                return
        for a, cin, mode, resid, rows, nwg, lds in seg:
            self.launches.append((lib.dtf_conv_fwd_s1, (ctypes.byref(a), cin, mode, int(resid), rows, nwg, lds)))

    def _conv_fwd(self, ci, x, y, stats_bn, in_bn, res=None):
        be, L = self.be, self.be.L
        c = L.prog.convs[ci]
        Hi = x.shape[1]
        Ho = Hi // c.stride
        cin = 16 if ci == L.prog.stem else c.cin
        P = (c.k - 1) // 2
        rows = None
        for r in range(min(8, Ho), 0, -1):
            rows_in = (r - 1) * c.stride + c.k
            if Ho % r == 0 and (r * Ho) % 16 == 0 and rows_in * (Hi + 2 * P) * (cin // 8) <= 4 * 256:
                rows = r
                break
        assert rows is not None, ("no valid band for conv", ci)
        s1 = c.k == 3 and c.stride == 1 and cin == c.cout and Hi == 512 // cin and stats_bn is not None
        if s1 and cin == 64 and self.N <= HALF_BANDS_MAX_IMGS and in_bn is not None and not be.det:
            rows = 4  # conv_fwd_s1_kernel<64, ., ., 4>
        bands = Ho // rows
        lo = FWD_MIN_WG_SMALL if len(self.slots) <= DUAL_MAX_POP else FWD_MIN_WG
        iters = FWD_ITERS_C.get(cin, FWD_ITERS_PER_WG)
        if cin in FWD_WG_TARGET:  # no more than this many workgroups: longer ones once the population allows
            iters = max(iters, min(8, self.N * bands // FWD_WG_TARGET[cin]))  # (16 at 256 workgroups: +2.4 %)
        n_wg = self._n_wg_iters(self.N * bands, per_wg=iters, lo=lo, hi=max(1024, self.N * bands // iters))
        if FWD_RESIDENT and s1 and len(self.slots) > DUAL_MAX_POP:
            # conv_fwd_s1_kernel occupancy: 4 WGs / CU (C <= 32), 3 (C = 64)
            n_wg = self._det_cap(min(self.N * bands, _n_cu() * (4 if cin <= 32 else 3)))
        work = self._work_iters(bands, n_wg)
        a = self._base_args()
        a.x, a.y, a.res = _p(x), _p(y), _p(res)
        a.w, a.w_off = _p(be.wf), L.fwd_off[ci]
        a.work = _p(work)
        if in_bn is not None:
            a.in_gamma, a.in_beta = self._bn(in_bn)
            a.st_in = _p(self._st_r(in_bn))
        if stats_bn is not None:
            a.st_out = _p(self._st_w(stats_bn))
        a.Hi, a.Wi, a.Ho, a.Wo, a.rows = Hi, Hi, Ho, Ho, rows
        rows_in = (rows - 1) * c.stride + c.k
        tsz = (rows_in * (Hi + 2 * P) * max(_cpad(cin), _cpad_fwd(cin)) + 8 + 63) // 64 * 64
        lds = 1280 + 2 * tsz * 2
        mode = 0 if in_bn is None else 1
        lib = ops.lib()
        if s1 and (rows == 8 or (rows == 4 and cin == 64)):
            # compile-time-geometry kernel of the CIFAR stages (conv_fwd_s1_kernel)
            self._set_uniform(a, work)
            a.cin_real = self._stamp_row("fwd", "fwd_s1 C=%d in=%d res=%d" % (cin, mode, res is not None))  # launch ordinal for DTF_STAMP diagnostic builds (unused otherwise)
            lds = 1280 + 2 * ((rows_in * _wpitch(cin) * _cpad_fwd(cin) + 8 + 63) // 64 * 64) * 2
            if self.persist_fwd and getattr(self, "_grab", None) is None:
                self._pseg_add(a, cin, mode, res is not None, rows, work.shape[0], lds)
            else:
                self._add(lib.dtf_conv_fwd_s1, ctypes.byref(a), cin, mode, int(res is not None), rows,
                          work.shape[0], lds)
        else:
            self._add(lib.dtf_conv_fwd, ctypes.byref(a), cin, c.cout, c.stride, c.k, mode, int(res is not None),
                      int(stats_bn is not None), work.shape[0], lds)
        self._keep(a)

    def _conv_dgrad(self, ci, dy, y, Hi, mode, epi, dy2=None, in_bn=None, res=None, xm=None, ep_bn=None):
        be, L = self.be, self.be.L
        c = L.prog.convs[ci]
        S, K = c.stride, c.k
        Ho = Hi // S
        rows = None
        for r in range(min(8, Hi), 0, -1):
            rows_t = r + K - 1 if S == 1 else (r + K + S - 2) // S + 1
            if Hi % r == 0 and (r * Hi) % 16 == 0 and rows_t * (Ho + 2) * (c.cout // 8) <= 4 * 256:
                rows = r
                break
        assert rows is not None, ("no valid band for dgrad", ci)
        if S == 2 and K == 3:  # conv.hip conv_dgrad_body PAR: parity-class tiles of 8-row bands, Wi = 512 / cin
            assert rows == 8 and Hi == 512 // c.cin, ("stride-2 dgrad geometry", ci, Hi, c.cin, rows)
        rows_t = rows + K - 1 if S == 1 else (rows + K + S - 2) // S + 1
        bands = Hi // rows
        n_wg = self._n_wg_iters(self.N * bands)
        work = self._work_iters(bands, n_wg)
        a = self._base_args()
        a.x, a.x2, a.y, a.res, a.xm = _p(dy), _p(dy2), _p(y), _p(res), _p(xm)
        a.w, a.w_off = _p(be.wd), L.dgr_off[ci]
        a.work = _p(work)
        if in_bn is not None:
            a.in_gamma, a.in_beta = self._bn(in_bn)
            a.st_in, a.st_in_b = _p(be.st_f(in_bn)), _p(be.st_b(in_bn))
        if ep_bn is not None:
            a.ep_gamma, a.ep_beta = self._bn(ep_bn)
            a.st_ep = _p(be.st_f(ep_bn))
            a.st_out = _p(be.st_b(ep_bn))
        a.Hi, a.Wi, a.Ho, a.Wo, a.rows = Hi, Hi, Ho, Ho, rows
        tsz = (rows_t * (Ho + 2) * _cpad(c.cout) + 63) // 64 * 64
        lds = 2304 + 2 * tsz * 2
        lib = ops.lib()
        self._add(lib.dtf_conv_dgrad, ctypes.byref(a), c.cin, c.cout, S, K, mode, epi, work.shape[0], lds)
        self._keep(a)

    @staticmethod
    def _trans_multi(ca_spec):
        """Combined stage-transition backward launch (conv_trans_multi_kernel) for the 3x3 / 2 conv_a of a projection
        block with 16->32 or 32->64 channels."""
        return ca_spec.stride == 2 and ca_spec.k == 3 and (ca_spec.cin, ca_spec.cout) in ((16, 32), (32, 64))

    def _add_trans_multi(self, grabbed, ca_spec):
        (f_c, args_c), (f_a, args_a), (f_b, args_b) = grabbed
        lib = ops.lib()
        # by name: the debug library hands out a fresh checked wrapper per attribute access
        assert [ops.launcher_name(f) for f in (f_c, f_a, f_b)] == ["dtf_conv_wgrad", "dtf_conv_dgrad", "dtf_conv_wgrad"]
        # (byref(args), cin, cout, S, K, mode.., mode.., nblocks, lds)
        assert args_c[1:6] == (ca_spec.cin, ca_spec.cout, 2, 3, 1) and args_c[6] == 2
        assert args_a[1:7] == (ca_spec.cin, ca_spec.cout, 2, 1, 0, 0)
        assert args_b[1:7] == (ca_spec.cin, ca_spec.cout, 2, 1, 1, 0)
        ac, aa, ab = args_c[0]._obj, args_a[0]._obj, args_b[0]._obj
        ac.n_main, aa.n_main, ab.n_main = args_c[7], args_a[7], args_b[7]
        nblocks = args_c[7] + args_a[7] + args_b[7]
        lds = max(args_c[8], args_a[8], args_b[8])
        self._add(lib.dtf_conv_trans_multi, ctypes.byref(ac), ctypes.byref(aa), ctypes.byref(ab), ca_spec.cin,
                  ca_spec.cout, nblocks, lds)

    def _conv_wgrad(self, ci, x, dy, mode_x, mode_dy, x_bn=None, dy_bn=None, dy2=None, cin_real=None):
        be, L, e = self.be, self.be.L, self.e
        c = L.prog.convs[ci]
        Hi = x.shape[1]
        Ho = Hi // c.stride
        cin = 16 if ci == L.prog.stem else c.cin
        P = (c.k - 1) // 2
        # band rows: R*Wo % 32 == 0, and the register-staged tiles fit 4 (x) / 2 (dy) chunks per thread
        rows = None
        for r in range(min(8, Ho), 0, -1):
            if Ho % r or (r * Ho) % 32:
                continue
            rows_in = (r - 1) * c.stride + c.k
            if rows_in * (Hi + 2 * P) * (cin // 8) <= 4 * 256 and r * Ho * (c.cout // 8) <= 2 * 256:
                rows = r
                break
        if rows is None:
            rows = _pick_rows(Ho, Ho, 1, 32, target_items=1, max_rows=8)
        # images per workgroup: bound the fp32 atomic traffic of the per-WG partial dW (~12 MB per launch)
        wn = c.cout * c.k * c.k * c.cin
        # bound fp32 atomic traffic (~12 MB / launch) and same-address contention (<= 128 WGs per member)
        n_wg = max(64, min(WGRAD_WG_PER_MEMBER * len(self.slots), int(12e6 / (4.0 * wn))))
        if self.be.det and not self.wslab:
            n_wg = len(self.slots)  # one workgroup per member: every dW element is added once (fixed order)
        work = self._work_iters(Ho // rows, n_wg)
        a = self._base_args()
        a.x, a.dy, a.dy2 = _p(x), _p(dy), _p(dy2)
        a.work = _p(work)
        a.g_off = c.off
        a.cin_real = c.cin if cin_real is None else cin_real
        if x_bn is not None:
            a.x_gamma, a.x_beta = self._bn(x_bn)
            a.st_x = _p(be.st_f(x_bn))
        if dy_bn is not None:
            a.in_gamma, a.in_beta = self._bn(dy_bn)
            a.st_in, a.st_in_b = _p(be.st_f(dy_bn)), _p(be.st_b(dy_bn))
        a.Hi, a.Wi, a.Ho, a.Wo, a.rows = Hi, Hi, Ho, Ho, rows
        rows_in = (rows - 1) * c.stride + c.k
        assert 32 % Ho == 0, "wgrad k-step addressing needs Wo | 32"
        xt = (rows_in * (Hi + 2 * P) * _cpad(cin) + 63) // 64 * 64
        dt = (rows * Ho * _cpad(c.cout) + 63) // 64 * 64
        lds = 1536 + 2 * (xt + dt) * 2  # double-buffered
        lib = ops.lib()
        if self.wslab:
            kel = c.cout * c.k * c.k * a.cin_real
            a.slab = _p(self._layer_slab(work.shape[0] * kel))
            self._deferred_dense.append((a.slab, self._slab_table(work), c.off, kel))
        self._add(lib.dtf_conv_wgrad, ctypes.byref(a), cin, c.cout, c.stride, c.k, mode_x, mode_dy, work.shape[0], lds)
        self._keep(a)

    def _conv_bwd_fused(self, ci, dy, dz_out, x, mode_dy, dy2=None, dy_bn=None, x_bn=None, res=None, ident_x=False,
                        dy3=None, dy_out=None, chain_bn=None, chain_h=None):
        """dgrad + wgrad of a stride-1 3x3 C->C conv in one launch (see conv_bwd_fused_kernel).

        ``mode_dy`` 3: dY = BN-backward(dy, dy2) + dy3 (the previous block's BN1 backward and the identity
        shortcut folded into the staging); ``dy_out`` materialises that dY (needed downstream).  The dW slabs
        of the PREVIOUS fused launch are reduced by trailing workgroups of this one when small enough
        (``_piggyback``); the rest by a standalone dw_slab_reduce.
        ``chain_bn`` / ``chain_h`` (v1 conv_a, identity mask): the epilogue also takes the backward sums of BN
        ``chain_bn`` whose input is ``chain_h`` -- sum(dz), sum(dz * x-hat) of the output gradient this launch
        produces (EPI bit 8), instead of a standalone bn_bwd_reduce pass over it."""
        be, L = self.be, self.be.L
        c = L.prog.convs[ci]
        assert c.stride == 1 and c.k == 3 and c.cin == c.cout
        assert (mode_dy == 3) == (dy3 is not None)
        C, H = c.cin, x.shape[1]
        rows = None
        for r in (8, 4, 2):
            if H % r == 0 and (r * H) % 32 == 0 and (r + 2) * (H + 2) * (C // 8) <= 4 * 256:
                rows = r
                break
        # the fused kernel's geometry is compile-time: W = H = 512 / C, 8-row bands
        assert rows == 8 and H == 512 // C and x.shape[2] == H, (C, H, rows)
        for t in (dy, dy2, dy3, dy_out, dz_out, x, res):
            assert t is None or tuple(t.shape) == (self.N, H, H, C), (t.shape, C, H)
        bands = H // rows
        if (self.dual and (C in DUAL_CS or self.defer_wg)) or C in self.defer_cs:
            # the dual / deferred launches have no epilogue for a chained BN's backward sums: a caller that marked
            # the previous block as chained (v1 _build_v1) would silently lose them
            assert chain_bn is None, "chain_bn needs the fused launch (dual / deferred paths are v2-only)"
            return self._conv_bwd_dual(ci, c, C, H, rows, bands, dy, dz_out, x, mode_dy, dy2, dy_bn, x_bn, res,
                                       ident_x, dy3, dy_out)
        n_wg = self._fused_nwg(C, bands, mode_dy)
        work = self._work_iters(bands, n_wg)
        a = self._base_args()
        a.x, a.x2, a.y, a.xm, a.res = _p(dy), _p(dy2), _p(dz_out), _p(x), _p(res)
        a.x3, a.xout = _p(dy3), _p(dy_out)
        a.w, a.w_off = _p(be.wd), L.dgr_off[ci]
        a.work = _p(work)
        a.g_off = c.off
        a.n_main = work.shape[0]
        self._set_uniform(a, work)
        if dy_bn is not None:
            a.in_gamma, a.in_beta = self._bn(dy_bn)
            a.st_in, a.st_in_b = _p(be.st_f(dy_bn)), _p(be.st_b(dy_bn))
        if not ident_x:
            a.ep_gamma, a.ep_beta = self._bn(x_bn)
            a.st_ep = _p(be.st_f(x_bn))
            a.st_out = _p(be.st_b(x_bn))
        if chain_bn is not None:
            assert ident_x and mode_dy == 2 and tuple(chain_h.shape) == (self.N, H, H, C)
            a.x3 = _p(chain_h)
            a.ep_gamma, a.ep_beta = self._bn(chain_bn)
            a.st_ep = _p(self._st_r(chain_bn))
            a.st_out = _p(be.st_b(chain_bn))
        a.Hi, a.Wi, a.Ho, a.Wo, a.rows = H, H, H, H, rows
        tsz = ((rows + 2) * _wpitch(C) * _cpad(C) + 8 + 63) // 64 * 64
        raw = C >= 64  # must match conv.hip RAWX
        nbuf = 4  # double-buffered size even when conv.hip single-buffers (SB): C = 16 still fits 3 WGs per CU
        lds = 2304 + (nbuf * tsz + (2 * rows * H * _cpad(C) if raw else 0)) * 2  # dY/X tiles [+ raw-x interiors]
        if C == 16 and _lib_knob("dtf_fused16_wlds"):
            lds += 16 * (32 * 5 + 8) * 2  # conv.hip DTF_FUSED16_WLDS: the dgrad weights in LDS
        lib = ops.lib()
        # dW partials: per-workgroup slabs.  C = 64: every layer its own slab, all reduced by ONE launch after the
        # backward; C = 16 / 32: ping-pong slab buffers, each reduced by trailing workgroups of the next launch
        n_red = 0
        pend = self._pending_slab
        if pend is not None and self._piggyback(pend):
            buf, red, rc, goff = pend
            a.rslab, a.rtab, a.r_c, a.r_goff = buf, _p(red), rc, goff
            a.r_nblk = self._reduce_wgs(rc)
            n_red = a.r_nblk * red.shape[0]
            self._pending_slab = None
        else:
            self._flush_slab()
        if C == 64:
            a.slab = _p(self._layer_slab(work.shape[0] * self._slab_elems(C)))
        else:
            a.slab = _p(self._slab(self._slab_floats())[self._slab_flip])
            self._slab_flip ^= 1
        epi = int(res is not None) | (2 if ident_x else 0) | (8 if chain_bn is not None else 0)
        a.cin_real = self._stamp_row("fused", "fused C=%d mdy=%d epi=%d" % (C, mode_dy, epi))
        self._add(lib.dtf_conv_bwd_fused, ctypes.byref(a), C, mode_dy, epi, work.shape[0] + n_red, lds)
        self._keep(a)
        red = self._slab_table(work)
        if C == 64:
            self._deferred.append((a.slab, red, c.off, 64))
        else:
            self._pending_slab = (a.slab, red, C, c.off)

    def _conv_bwd_dual(self, ci, c, C, H, rows, bands, dy, dz_out, x, mode_dy, dy2, dy_bn, x_bn, res, ident_x, dy3,
                       dy_out):
        """Dual backward of a stride-1 C->C conv (conv_bwd_dual_kernel): dgrad-role workgroups (one (image, band)
        iteration each by default: the critical path) and wgrad-role workgroups (DUAL_WG[C] per member, each
        over a run of iterations, writing a dW slab) in one launch; both stage the same transformed dY.  The
        slabs are reduced by the trailing workgroups of the next backward launch (or a standalone reduction)."""
        be, L = self.be, self.be.L
        lib = ops.lib()
        tsz = ((rows + 2) * _wpitch(C) * _cpad(C) + 8 + 63) // 64 * 64
        epi = int(res is not None) | (2 if ident_x else 0)
        # ---- dgrad role: one (image, band) iteration per workgroup (larger populations: DG_ITERS_LARGE); the
        # deferred-wgrad dgrad launch of the C = 64 stage takes half-image bands at small populations
        rows_dg = 4 if (C == 64 and C in self.defer_cs and self.N <= HALF_BANDS_MAX_IMGS and not be.det) else rows
        bands_dg = H // rows_dg
        n_dg = max(1, self.N * bands_dg)
        if not self.dual:
            n_dg = min(n_dg, max(DG_MIN_WG, -(-n_dg // DG_ITERS_LARGE)))
        work = self._work_iters(bands_dg, self._det_cap(n_dg))
        a = self._base_args()
        a.x, a.x2, a.y, a.xm, a.res = _p(dy), _p(dy2), _p(dz_out), _p(x), _p(res)
        a.x3, a.xout = _p(dy3), _p(dy_out if mode_dy >= 2 else None)
        a.w, a.w_off = _p(be.wd), L.dgr_off[ci]
        a.work = _p(work)
        a.g_off = c.off
        a.n_main = work.shape[0]
        self._set_uniform(a, work)
        if dy_bn is not None:
            a.in_gamma, a.in_beta = self._bn(dy_bn)
            a.st_in, a.st_in_b = _p(be.st_f(dy_bn)), _p(be.st_b(dy_bn))
        if not ident_x:
            a.ep_gamma, a.ep_beta = self._bn(x_bn)
            a.st_ep = _p(be.st_f(x_bn))
            a.st_out = _p(be.st_b(x_bn))
        a.Hi, a.Wi, a.Ho, a.Wo, a.rows = H, H, H, H, rows_dg
        a.cin_real = self._stamp_row("fused", "fused-dg C=%d mdy=%d epi=%d" % (C, mode_dy, epi))
        # ---- wgrad role (same staging of dY / X; own work split)
        wwork = self._work_iters(bands, max(1, min(self.N * bands, DUAL_WG[C] * len(self.slots))))
        b = self._base_args()
        b.x, b.x2, b.x3, b.xm = _p(dy), _p(dy2), _p(dy3), _p(x)
        b.work = _p(wwork)
        b.g_off = c.off
        b.n_main = wwork.shape[0]
        self._set_uniform(b, wwork)
        if dy_bn is not None:
            b.in_gamma, b.in_beta = self._bn(dy_bn)
            b.st_in, b.st_in_b = _p(be.st_f(dy_bn)), _p(be.st_b(dy_bn))
        if not ident_x:
            b.ep_gamma, b.ep_beta = self._bn(x_bn)
            b.st_ep = _p(be.st_f(x_bn))
        b.Hi, b.Wi, b.Ho, b.Wo, b.rows = H, H, H, H, rows
        b.cin_real = self._stamp_row("fused", "fused-wg C=%d mdy=%d epi=%d" % (C, mode_dy, epi))
        if C in self.defer_cs:
            return self._defer_wgrad(ci, c, C, H, rows, bands, a, b, dy, x, mode_dy, dy2, dy_bn, x_bn, dy_out,
                                     tsz, epi)
        b.slab = _p(self._layer_slab(wwork.shape[0] * self._slab_elems(C)))
        # ---- trailing reduction of the previous backward launch's slabs
        n_red = 0
        pend = self._pending_slab
        if pend is not None and self._piggyback(pend):
            buf, red, rc, goff = pend
            a.rslab, a.rtab, a.r_c, a.r_goff = buf, _p(red), rc, goff
            a.r_nblk = self._reduce_wgs(rc)
            n_red = a.r_nblk * red.shape[0]
            self._pending_slab = None
        else:
            self._flush_slab()
        self._keep(a)
        self._keep(b)
        lds = 2304 + 4 * tsz * 2  # the wgrad role's dY + X tiles (double-buffered); the dgrad role uses half
        self._add(lib.dtf_conv_bwd_dual, ctypes.byref(a), ctypes.byref(b), C, mode_dy, epi,
                  a.n_main + b.n_main + n_red, lds)
        if C == 64:
            self._deferred.append((b.slab, self._slab_table(wwork), c.off, 64))
        else:
            self._pending_slab = (b.slab, self._slab_table(wwork), C, c.off)

    def _defer_wgrad(self, ci, c, C, H, rows, bands, a, b, dy, x, mode_dy, dy2, dy_bn, x_bn, dy_out, tsz, epi):
        """Deferred-wgrad form of a dual launch: the launch holds the dgrad role only; the wgrad job (the role's
        arguments with its own work split) is queued for conv_wgrad_all_kernel.  Its dY operand: the dY the
        dgrad role materialises (``dy_out``) or the plain incoming gradient (mode 0), read as-is; else (conv_a)
        BN2-backward(dz2, h) recomputed while staging, as the dgrad role does."""
        lib = ops.lib()
        self._keep(a)
        tsz_dg = ((a.rows + 2) * _wpitch(C) * _cpad(C) + 8 + 63) // 64 * 64
        self._add(lib.dtf_conv_bwd_dg, ctypes.byref(a), C, mode_dy, epi, a.rows, a.n_main, 2304 + 2 * tsz_dg * 2)
        w = self._base_args()
        ctypes.memmove(ctypes.addressof(w), ctypes.addressof(b), ctypes.sizeof(ConvArgs))
        if dy_out is not None or mode_dy == 0:
            wmode = 0
            w.x, w.x2, w.x3 = _p(dy_out if dy_out is not None else dy), None, None
            w.in_gamma = w.in_beta = 0
            w.st_in = w.st_in_b = None
        else:
            wmode = 2
            assert mode_dy == 2 and dy2 is not None and dy_bn is not None
        per = DEFER_WG[C] if self.defer_wg else DEFER_LARGE_WG[C]
        wwork = self._work_iters(bands, max(1, min(self.N * bands, per * len(self.slots))), det_per=per)
        w.work = _p(wwork)
        w.n_main = wwork.shape[0]
        self._set_uniform(w, wwork)
        # DEFER_ATOMIC (release build): the job's workgroups add their dW partials straight into the gradient rows
        # (fp32 atomics, a handful of workgroups per address) instead of writing slabs for slab_reduce_all
        atomic = DEFER_ATOMIC and not self.be.det and C in DEFER_ATOMIC_CS
        w.slab = None if atomic else _p(self._layer_slab(wwork.shape[0] * self._slab_elems(C)))
        w.cin_real = -1
        self._wg_jobs.setdefault((C, wmode), []).append((w, wwork, c.off))

    def _emit_deferred_wgrad(self, only_c=None, side=False):
        """Every queued layer's wgrad job in two launches (conv_wgrad_all_kernel: widths 64 + 32 -- one wave per SIMD
        -- and width 16, kept apart at its higher occupancy); their slabs join the reduction of _flush_deferred.
        One launch per (C, dY mode) measured 18 us slower at pop 1 (profiles/r3_merged_launches_ab.log).
        ``only_c``: just the jobs of that width; ``side``: on the side stream (a parallel graph branch, joined before
        the slab reduction)."""
        lib = ops.lib()
        if side and any(C == only_c or only_c is None for (C, _) in self._wg_jobs):
            self._add("fork", None)
            self._forked = True
        for cset, widths in ((0, (64, 32)), (1, (16,))):  # must match dtf_conv_wgrad_all's instantiations
            arr_l, wmap, lds = [], [], 0
            for (C, wmode), jobs in sorted(self._wg_jobs.items(), key=lambda kv: (-kv[0][0], -kv[0][1])):
                if C not in widths or (only_c is not None and C != only_c):
                    continue
                tsz = ((8 + 2) * _wpitch(C) * _cpad(C) + 8 + 63) // 64 * 64
                lds = max(lds, 2304 + 4 * tsz * 2)
                for (w, work, goff) in jobs:
                    j = len(arr_l)
                    arr_l.append(w)
                    wmap += [(j, k, C, wmode) for k in range(w.n_main)]
                    if w.slab:  # (None: the job accumulates with atomics, DEFER_ATOMIC)
                        self._deferred.append((w.slab, self._slab_table(work), goff, C))
            if not arr_l:
                continue
            arr = (ConvArgs * len(arr_l))(*arr_l)
            jt = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.be.dev)
            mt = torch.tensor(wmap, dtype=torch.int32, device=self.be.dev)
            self._keep(jt)
            self._keep(mt)
            self._add(lib.dtf_conv_wgrad_all, _p(jt), _p(mt), len(wmap), cset, lds)
        if side and getattr(self, "_forked", False):
            self._add("endfork", None)
        self._wg_jobs = {k: v for k, v in self._wg_jobs.items() if only_c is not None and k[0] != only_c}

    def _maybe_overlap_wgrad(self, i):
        """After block i's backward: issue the queued deferred wgrad jobs of its width on the side stream when the
        next block to process has another width (stage boundary) or OVERLAP_CHUNK jobs are queued."""
        if not (self.overlap_wg and self._wg_jobs):
            return
        C = self.hs[i].shape[3]
        nxt = self.hs[i - 1].shape[3] if i > 0 else None
        queued = sum(len(v) for (c, _), v in self._wg_jobs.items() if c == C)
        if nxt != C or (OVERLAP_CHUNK and queued >= OVERLAP_CHUNK):
            self._emit_deferred_wgrad(only_c=C, side=True)

    def _fresh_like(self, t):
        u = torch.empty_like(t)
        self._keep(u)
        return u

    def _piggyback(self, pend):
        """Reduce the previous launch's C = 16 / 32 slabs inside the next backward launch when that adds few
        workgroups (the trailing workgroups carry the fused kernel's register budget: low occupancy).  C = 64 slabs
        are deferred to one launch after the backward (a looping piggyback reduction measured slower:
        profiles/r2_piggyback_c64_ab.log)."""
        _, red, rc, _ = pend
        return rc != 64 and (self._slab_elems(rc) // 32) * red.shape[0] <= PIGGYBACK_MAX_WG

    def _reduce_wgs(self, rc):
        """Reduce workgroups per member of a piggybacked slab reduction: one per 32 slab elements."""
        return self._slab_elems(rc) // 32

    def _flush_deferred(self):
        """Every deferred dW slab (conv slabs of each width, dense wgrad slabs) reduced by one launch
        (slab_reduce_all_kernel; one launch per width plus one for the dense slabs measured 10 us slower)."""
        if not (self._deferred or self._deferred_dense):
            return
        sj = (SlabJob * max(1, len(self._deferred)))()
        dj = (DenseJob * max(1, len(self._deferred_dense)))()
        nmax = bmax = 0
        for i, (buf, red, goff, C) in enumerate(self._deferred):
            sj[i] = SlabJob(buf, _p(red), goff, red.shape[0], C)
            nmax = max(nmax, red.shape[0])
            nb = self._slab_elems(C) // 256
            bmax = max(bmax, min(nb, SLAB_X_BLOCKS) if SLAB_X_BLOCKS > 0 else nb)
        for i, (buf, red, goff, kel) in enumerate(self._deferred_dense):
            dj[i] = DenseJob(buf, _p(red), goff, kel, red.shape[0])
            nmax = max(nmax, red.shape[0])
            bmax = max(bmax, min(-(-kel // 32), DENSE_REDUCE_BLOCKS))
        st = torch.frombuffer(bytearray(bytes(sj)), dtype=torch.uint8).to(self.be.dev)
        dt = torch.frombuffer(bytearray(bytes(dj)), dtype=torch.uint8).to(self.be.dev)
        self._keep(st)
        self._keep(dt)
        self._add(ops.lib().dtf_slab_reduce_all, _p(st), len(self._deferred), _p(dt), len(self._deferred_dense),
                  nmax, bmax, _p(self.e.grads), self.e.Pp)
        self._deferred, self._deferred_dense = [], []

    def _flush_slab(self):
        """Standalone reduction of a pending slab (no later fused launch can take it)."""
        pend = self._pending_slab
        if pend is None:
            return
        buf, red, rc, goff = pend
        self._add(ops.lib().dtf_dw_slab_reduce, buf, _p(red), red.shape[0], _p(self.e.grads), self.e.Pp, goff, rc)
        self._pending_slab = None

    @staticmethod
    def _slab_elems(C):
        return ((9 * C // 16 + 3) // 4) * (C // 16) * 4 * 256

    def _fused_nwg(self, C, bands, mode_dy=0):
        if self.be.det:
            return DET_WG_PER_MEMBER * len(self.slots)  # = the rows _work_iters gives every member
        # per-launch budget for the dW partials (bytes of slab stores, or of atomics without slabs): bounds the
        # workgroup count of the fused kernel
        wn = 9 * C * C
        n_wg = max(64, min(128 * len(self.slots), int(FUSED_SLAB_BYTES[C] / (4.0 * wn))))
        # floor of 256 workgroups: a single member would otherwise run the C = 16 / 32 layers on 128 of the 256
        # CUs (pop 1: 1.54 -> 1.50 ms/step; larger populations already exceed it)
        n_wg = max(n_wg, FUSED_MIN_WG)
        # per-member cap: fewer, fuller workgroups write fewer dW slab bytes.  C = 32 at 128 per member (2 bands
        # each): pop 1 1.52 -> 1.44-1.47 ms/step over two runs (profiles/r1_s7_variants.log); pop >= 2 unchanged
        if C in FUSED_MAX_WG:
            n_wg = min(n_wg, FUSED_MAX_WG[C] * len(self.slots))
        if C in FUSED_TOTAL_MAX and FUSED_TOTAL_MAX[C] > 0 and len(self.slots) >= FUSED_TOTAL_MIN_POP[C]:
            n_wg = min(n_wg, max(FUSED_TOTAL_MAX[C], FUSED_MIN_WG))
        n_wg = min(n_wg, self.N * bands)
        res = _n_cu() * _fused_wgs_per_cu(C, mode_dy)
        if FUSED_RESIDENT and n_wg > res:
            n_wg = n_wg // res * res
            if FUSED_ROUNDS > 0:
                n_wg = min(n_wg, FUSED_ROUNDS * res)
        return self._det_cap(n_wg)

    def _slab_floats(self):
        cfg = self.be.L.cfg
        need = 0
        for st in range(len(cfg.block_sizes)):
            C = cfg.num_filters * (2 ** st)
            H = cfg.image_size >> st
            if C in (16, 32, 64) and H == 512 // C:
                need = max(need, max(self._fused_nwg(C, H // 8, m) for m in (0, 3)) * self._slab_elems(C))
        return need

    def _head_slab(self, ha, hwork):
        """Dense-layer gradients of the head as per-workgroup slabs, reduced with the deferred wgrad slabs (instead
        of every head workgroup adding the same ncls x C addresses atomically)."""
        if not self.wslab:
            return
        nwg, ncls, C = hwork.shape[0], ha.ncls, ha.C
        sw = self._layer_slab(nwg * ncls * C)
        sb = self._layer_slab(nwg * ncls)
        ha.slab, ha.slab_b = _p(sw), _p(sb)
        red = self._slab_table(hwork)
        prog = self.be.L.prog
        self._deferred_dense.append((ha.slab, red, prog.dense_w_off, ncls * C))
        self._deferred_dense.append((ha.slab_b, red, prog.dense_b_off, ncls))

    def _layer_slab(self, n):
        t = torch.empty(max(n, 1), dtype=torch.float32, device=self.be.dev)
        self._keep(t)
        return t

    def _slab(self, n):
        """The plan's two ping-pong slab buffers (sized once for the largest fused layer)."""
        if getattr(self, "slab_buf", None) is None:
            self.slab_buf = [torch.empty(max(n, 1), dtype=torch.float32, device=self.be.dev) for _ in range(2)]
        assert self.slab_buf[0].numel() >= n, "slab must be sized once per plan"
        return self.slab_buf

    def _slab_table(self, work):
        """(first wg, n wgs, 0, slot) per member of a work-item array grouped by member.  An elastic work table's rows
        per member change with the batch sizes: its table is shared and rewritten on the device by work_gen."""
        red = self.__dict__.setdefault("_elastic_red", {})
        if work.data_ptr() in red:
            return red[work.data_ptr()]
        w = work.cpu().tolist()
        rows = []
        for i, it in enumerate(w):
            if rows and rows[-1][3] == it[3] and rows[-1][0] + rows[-1][1] == i:
                rows[-1][1] += 1
            else:
                rows.append([i, 1, 0, it[3]])
        t = torch.tensor(rows, dtype=torch.int32, device=self.be.dev)
        self._keep(t)
        if self.elastic and any(wg[0].data_ptr() == work.data_ptr() for wg in self._wgen):
            assert len(rows) == len(self.slots), "elastic slab table: one row per member"
            red[work.data_ptr()] = t
        return t

    def _stamp_row(self, kind, label=""):
        """Row of the DTF_STAMP diagnostic buffer for the next launch of ``kind`` (fwd: 0.., fused: 64..)."""
        if not hasattr(self, "_stamp_n"):
            self._stamp_n = {"fwd": 0, "fused": 0}
        row = self._stamp_n[kind] + (64 if kind == "fused" else 0)
        self._stamp_n[kind] += 1
        self.stamp_rows = getattr(self, "stamp_rows", []) + [(row, label)]
        return row

    def _keep(self, obj):
        if not hasattr(self, "_keepalive"):
            self._keepalive = []
        self._keepalive.append(obj)

    def _build(self):
        if self.v1:
            return self._build_v1()
        be, e, L = self.be, self.e, self.be.L
        prog, cfg = L.prog, L.cfg
        lib = ops.lib()
        N = self.N
        nslots = len(self.slots)
        # 0. weights for this step
        self._add(lib.dtf_weight_prep, _p(e.state), e.S, _p(be.conv_table_t), len(L.conv_table), _p(self.slots_t),
                  nslots, _p(be.wf), _p(be.wd), L.wtot, *self._zero_args())
        if self.src is not None:
            self._add("augment", None)  # gather + pad/crop/flip + standardize + bf16 pack (data.hip)
        else:
            self._add(lib.dtf_prep_input, _p(self.x_in), _p(self.xin16), N * cfg.image_size * cfg.image_size, 3)
        # ---------------- forward
        self._forward_v2()
        nblk = len(prog.blocks)
        # head (fwd + bwd of GAP/dense/CE + final-BN reductions)
        fb = prog.final_bn
        hw = L.final_hw
        hwork = self._head_work()
        ha = HeadArgs()
        ha.x, ha.labels, ha.work = _p(self.xs[-1]), _p(self.labels), _p(hwork)
        ha.params, ha.p_mstride = _p(e.state), e.S
        ha.gamma_off, ha.beta_off = self._bn(fb)
        ha.dw_off, ha.db_off = prog.dense_w_off, prog.dense_b_off
        ha.grads, ha.g_mstride = _p(e.grads), e.Pp
        ha.st_f, ha.st_b, ha.cnt = _p(be.st_f(fb)), _p(be.st_b(fb)), _p(self.cnt)
        ha.dfeat, ha.loss, ha.correct = _p(self.dfeat), _p(be.loss), _p(be.correct)
        ha.logits_out = None
        ha.hw, ha.C, ha.ncls, ha.train = hw, cfg.final_size, cfg.num_classes, 1
        ha.loss_scale = be.loss_scale
        self._head_slab(ha, hwork)
        self._keep(ha)
        self._add(lib.dtf_head, ctypes.byref(ha), hwork.shape[0])
        # (the moving-statistics update of the forward BNs runs at the end of the step, with the BN gradients)
        # ---------------- backward
        hwL = self.xs[-1].shape[1]
        g_cur = self.tmp[hwL]["g"][0]
        self._add(lib.dtf_head_bwd_apply, _p(self.xs[-1]), _p(self.dfeat), _p(g_cur), _p(self.img_slot), _p(e.state),
                  e.S, ha.gamma_off, ha.beta_off, _p(be.st_f(fb)), _p(be.st_b(fb)), _p(self.cnt), hw,
                  cfg.final_size, N)
        pend = None  # deferred BN1-backward of the block just processed: (dz1, x, add, out, bn1)
        for i in range(nblk - 1, -1, -1):
            blk = prog.blocks[i]
            bn1, bn2 = blk.bns
            x, h = self.xs[i], self.hs[i]
            Hi, Ho = x.shape[1], h.shape[1]
            T = self.tmp[Ho]
            if h.shape[3] in self.defer_cs:  # deferred wgrad: this block's dz2 is read again after the backward
                T = dict(T, dz2=self._fresh_like(T["dz2"]))
            ca, cb = blk.convs
            # conv_b: dgrad -> dz2 (mask by BN2(h), BN2 reductions); wgrad
            if pend is not None:
                # the previous block's g = BN1-backward(dz1, x) [+ g] is computed while staging conv_b's dY
                # and written out once (band interiors) for the projection / next BN-backward
                dz1p, xp, addp, outp, bn1p = pend
                self._conv_bwd_fused(cb, dz1p, T["dz2"], h, mode_dy=3 if addp is not None else 2, dy2=xp,
                                     dy3=addp, dy_out=outp, dy_bn=bn1p, x_bn=bn2)
                g_cur, pend = outp, None
            else:
                self._conv_bwd_fused(cb, g_cur, T["dz2"], h, mode_dy=0, x_bn=bn2)
            Tin = self.tmp[Hi] if Hi != Ho else T
            pd = None
            ca_spec = prog.convs[ca]
            if blk.proj is not None and self._trans_multi(ca_spec):
                # stage transition: conv_a wgrad + projection dgrad + projection wgrad in one launch
                pd = self.pd[id(blk)]
                self._grab = []
                self._conv_wgrad(ca, x, T["dz2"], mode_x=1, mode_dy=2, x_bn=bn1, dy_bn=bn2, dy2=h)
                self._conv_dgrad(blk.proj, g_cur, pd, Hi, mode=0, epi=0)
                self._conv_wgrad(blk.proj, x, g_cur, mode_x=1, mode_dy=0, x_bn=bn1)
                grabbed, self._grab = self._grab, None
                self._add_trans_multi(grabbed, ca_spec)
                self._conv_dgrad(ca, T["dz2"], Tin["dz1"], Hi, mode=2, epi=2 | 1, dy2=h, in_bn=bn2, res=pd, xm=x,
                                 ep_bn=bn1)
            elif blk.proj is not None:
                pd = self.pd[id(blk)]
                self._conv_dgrad(blk.proj, g_cur, pd, Hi, mode=0, epi=0)
                self._conv_wgrad(blk.proj, x, g_cur, mode_x=1, mode_dy=0, x_bn=bn1)
            # conv_a: dgrad of BN2-backward(dz2, h) [+ proj dgrad], mask by BN1(x), BN1 reductions
            if blk.proj is not None and self._trans_multi(ca_spec):
                pass  # conv_a done above
            elif ca_spec.stride == 1 and ca_spec.cin == ca_spec.cout:
                self._conv_bwd_fused(ca, T["dz2"], Tin["dz1"], x, mode_dy=2, dy2=h, dy_bn=bn2, x_bn=bn1, res=pd)
            else:
                self._conv_dgrad(ca, T["dz2"], Tin["dz1"], Hi, mode=2, epi=2 | (1 if pd is not None else 0), dy2=h,
                                 in_bn=bn2, res=pd, xm=x, ep_bn=bn1)
                self._conv_wgrad(ca, x, T["dz2"], mode_x=1, mode_dy=2, x_bn=bn1, dy_bn=bn2, dy2=h)
            # g_in = BN1-backward(dz1, x) [+ g_out if identity shortcut]
            g_next = Tin["g"][1] if g_cur is Tin["g"][0] else Tin["g"][0]
            if x.shape[3] in self.defer_cs:  # g (read by the previous block's deferred conv_b wgrad) stays alive
                g_next = self._fresh_like(Tin["g"][0])
            add = None if blk.proj is not None else g_cur
            if i > 0:
                pend = (Tin["dz1"], x, add, g_next, bn1)
            else:
                self._bn_bwd_apply(Tin["dz1"], x, add, g_next, bn1)
            g_cur = g_next
            self._maybe_overlap_wgrad(i)
        # stem wgrad (input = padded image, real channels 3)
        self._conv_wgrad(prog.stem, self.xin16, g_cur, mode_x=0, mode_dy=0, cin_real=cfg.in_channels)
        self._emit_deferred_wgrad()
        if getattr(self, "_forked", False):
            self._add("join", None)  # the side-stream wgrad branch ends before the slab reduction
        # BN parameter gradients from the backward reductions
        self._flush_slab()
        self._flush_deferred()
        self._add(lib.dtf_bn_step_end, _p(e.state), e.S, 3 * e.Pp, _p(be.bn_table_t), len(L.bn_table),
                  _p(be.stats[0]), _p(be.stats[1]), be.stats_bn_stride, _p(self.slots_t), nslots, _p(self.cnt),
                  _p(e.grads), e.Pp)
        # optimizer over every member row (+ zero grads), step counters
        self._add("optim", None)
        self._add("step", None)

    def _forward_v2(self):
        """Stem + every pre-activation block (BN+ReLU prologues, BN-statistic epilogues, residual adds)."""
        prog = self.be.L.prog
        first_bn = prog.blocks[0].bns[0]
        self._conv_fwd(prog.stem, self.xin16, self.xs[0], stats_bn=first_bn, in_bn=None)
        nblk = len(prog.blocks)
        for i, blk in enumerate(prog.blocks):
            bn1, bn2 = blk.bns
            nxt = prog.blocks[i + 1].bns[0] if i + 1 < nblk else prog.final_bn
            x, h, y = self.xs[i], self.hs[i], self.xs[i + 1]
            if blk.proj is not None:
                self._conv_fwd(blk.proj, x, self.scs[i], stats_bn=None, in_bn=bn1)
            self._conv_fwd(blk.convs[0], x, h, stats_bn=bn2, in_bn=bn1)
            res = self.scs[i] if blk.proj is not None else x
            self._conv_fwd(blk.convs[1], h, y, stats_bn=nxt, in_bn=bn2, res=res)

    def _forward_v1(self):
        """v1 stem (conv -> BN -> ReLU) + post-activation blocks (``_building_block_v1``)."""
        prog, cfg = self.be.L.prog, self.be.L.cfg
        lib = ops.lib()
        H = cfg.image_size
        self._conv_fwd(prog.stem, self.xin16, self.h0, stats_bn=prog.stem_bn, in_bn=None)
        self._bn_ew(lib.dtf_bn_add_relu, (H * H, cfg.num_filters), prog.stem_bn, self.h0, out=self.xs[0])
        for i, blk in enumerate(prog.blocks):
            bna, bnb = blk.bns
            x, ha, hb, y = self.xs[i], self.hs[i], self.hb[i], self.xs[i + 1]
            if blk.proj is not None:
                self._conv_fwd(blk.proj, x, self.scs[i], stats_bn=blk.proj_bn, in_bn=None)
            self._conv_fwd(blk.convs[0], x, ha, stats_bn=bna, in_bn=None)
            self._conv_fwd(blk.convs[1], ha, hb, stats_bn=bnb, in_bn=bna)
            hw_o = y.shape[1] * y.shape[2]
            if blk.proj is not None:
                self._bn_ew(lib.dtf_bn_add_relu, (hw_o, y.shape[3]), bnb, hb, bn2=blk.proj_bn, h2=self.scs[i], out=y)
            else:
                self._bn_ew(lib.dtf_bn_add_relu, (hw_o, y.shape[3]), bnb, hb, add=x, out=y)

    # ----- eval mode: BN with moving statistics (resnet_run_loop.py:463-466 ``classifier.evaluate``)
    def _st_r(self, bn):
        """Statistics a BN consumer normalises with: this step's batch statistics, or (eval) the moving ones."""
        return self.ev_stats[bn] if self.eval else self.be.st_f(bn)

    def _st_w(self, bn):
        """Where a conv epilogue adds the statistics of its output (eval: a sink nobody reads)."""
        return self.ev_sink if self.eval else self.be.st_f(bn)

    def _build_eval(self):
        """Forward-only launch list of an eval chunk: bf16 weights of the evaluated members, moving statistics in
        accumulator form, input packing, the training forward kernels reading those statistics, and the head
        in inference mode (per-member correct count; optional logits)."""
        be, e, L = self.be, self.e, self.be.L
        prog, cfg = L.prog, L.cfg
        lib = ops.lib()
        nslots = len(self.slots)
        self._add(lib.dtf_weight_prep, _p(e.state), e.S, _p(be.conv_table_t), len(L.conv_table), _p(self.slots_t),
                  nslots, _p(be.wf), _p(be.wd), L.wtot, None, 0)
        self._add(lib.dtf_bn_eval_stats, _p(e.state), e.S, 3 * e.Pp, _p(be.bn_table_t), len(L.bn_table),
                  _p(self.ev_stats), be.stats_bn_stride, _p(self.slots_t), nslots, _p(self.cnt))
        self._add(lib.dtf_prep_input, _p(self.x_in), _p(self.xin16), self.N * cfg.image_size * cfg.image_size, 3)
        if self.v1:
            self._forward_v1()
        else:
            self._forward_v2()
        hwork = self._work_member(target_items=HEAD_ITEMS)
        ha = HeadArgs()
        ha.x, ha.labels, ha.work = _p(self.xs[-1]), _p(self.labels), _p(hwork)
        ha.params, ha.p_mstride = _p(e.state), e.S
        if self.v1:
            ha.gamma_off, ha.beta_off = -1, -1
            ha.st_f = _p(self.ev_sink)
        else:
            ha.gamma_off, ha.beta_off = self._bn(prog.final_bn)
            ha.st_f = _p(self._st_r(prog.final_bn))
        ha.dw_off, ha.db_off = prog.dense_w_off, prog.dense_b_off
        ha.grads, ha.g_mstride = None, e.Pp
        ha.st_b, ha.cnt = _p(self.ev_sink), _p(self.cnt)
        ha.dfeat, ha.correct, ha.loss = None, _p(self.ev_acc[0]), _p(self.ev_acc[1])
        ha.logits_out = None
        ha.hw, ha.C, ha.ncls, ha.train = L.final_hw, cfg.final_size, cfg.num_classes, 0
        ha.loss_scale = 1.0
        self._keep(ha)
        self._head_args = ha
        self._add(lib.dtf_head, ctypes.byref(ha), hwork.shape[0])

    def want_logits(self):
        """Also write fp32 logits [N, ncls] of the next eval runs (numerics tests)."""
        if self.logits is None:
            self.logits = torch.zeros(self.N, self.be.L.cfg.num_classes, dtype=torch.float32, device=self.be.dev)
            self._head_args.logits_out = _p(self.logits)
        return self.logits

    def load_eval(self, x, y):
        """The same eval images for every member: [m, H, W, 3] fp32 -> this plan's [members * m] input."""
        m = x.shape[0]
        k = len(self.slots)
        assert all(n == m for n in self.sizes), "eval plans hold the same chunk for every member"
        self.x_in.view(k, m, *self.x_in.shape[1:]).copy_(x.reshape(1, m, *self.x_in.shape[1:]).expand(k, -1, -1, -1,
                                                                                                       -1))
        self.labels.view(k, m).copy_(y.reshape(1, m).expand(k, -1))

    def _zero_args(self):
        """(buffer, n) zeroed by weight_prep: the statistic accumulators, losses and correct counts."""
        be = self.be
        return _p(be.zbuf), be.zbuf.numel()

    def _bn_bwd_apply(self, dz, x, add, out, bn):
        """out = BN-backward(dz, x) [+ add] (bn_bwd_apply_kernel)."""
        be, e = self.be, self.e
        ba = BnBwdArgs()
        ba.dz, ba.x, ba.add, ba.out = _p(dz), _p(x), _p(add), _p(out)
        ba.img_slot, ba.params, ba.p_mstride = _p(self.img_slot), _p(e.state), e.S
        ba.gamma_off = self._bn(bn)[0]
        ba.st_f, ba.st_b, ba.cnt = _p(be.st_f(bn)), _p(be.st_b(bn)), _p(self.cnt)
        ba.hw, ba.C, ba.nimg = x.shape[1] * x.shape[2], x.shape[3], self.N
        self._keep(ba)
        self._add(ops.lib().dtf_bn_bwd_apply, ctypes.byref(ba))

    def _bn_ew(self, fn, n_hw_c, bn1, h1, bn2=None, h2=None, add=None, out=None, d=None):
        """bn_add_relu (forward, out=...) or bn_bwd_reduce (backward, d=...) of a v1 block / the v1 stem."""
        be, e = self.be, self.e
        hw, C = n_hw_c
        a = BnEwArgs()
        a.h1, a.h2, a.add, a.out, a.d = _p(h1), _p(h2), _p(add), _p(out), _p(d)
        a.img_slot, a.params, a.p_mstride = _p(self.img_slot), _p(e.state), e.S
        a.g1, a.b1 = self._bn(bn1)
        a.st1, a.sb1 = _p(self._st_r(bn1)), _p(be.st_b(bn1))
        if bn2 is not None:
            a.g2, a.b2 = self._bn(bn2)
            a.st2, a.sb2 = _p(self._st_r(bn2)), _p(be.st_b(bn2))
        a.cnt, a.hw, a.C, a.nimg = _p(self.cnt), hw, C, self.N
        a.cap = self.sizes[0] if self.elastic else 0  # elastic: skip each member's capacity padding
        det_reduce = self.be.det and d is not None
        if det_reduce:  # deterministic build: per-image partial rows, added per member in image order
            if getattr(self, "_det_rows", None) is None:
                self._det_rows = torch.zeros(self.N * 192, dtype=torch.float32, device=self.be.dev)
                self._first_t = torch.tensor([self.first[s] for s in self.slots], dtype=torch.int32,
                                             device=self.be.dev)
            a.slab = _p(self._det_rows)
        self._keep(a)
        self._add(fn, ctypes.byref(a))
        if det_reduce:
            self._add(ops.lib().dtf_bn_bwd_reduce_finish, ctypes.byref(a), _p(self._first_t), _p(self.slots_t),
                      len(self.slots))

    def _build_v1(self):
        """ResNet v1 (``_building_block_v1``, resnet_model.py:127-168): conv -> BN -> ReLU -> conv -> BN
        (+ shortcut [projection conv -> BN]) -> ReLU; stem conv -> BN -> ReLU; no final BN.

        Forward: convs read the post-ReLU block input directly (identity prologue) and reduce their own BN
        statistics; conv_b applies BN_a+ReLU on load; ``bn_add_relu`` materialises the block output.
        Backward: ``d`` = dL/d(pre-ReLU sum) arrives already masked (head / previous conv_a epilogue);
        ``bn_bwd_reduce`` takes BN_b's (and BN_p's) reductions; conv_b runs the fused dgrad+wgrad with the
        BN_b-backward transform on load and the BN_a mask + reductions in the epilogue; conv_a adds the shortcut
        gradient and masks by the block input (> 0), which yields the previous block's ``d``.
        """
        be, e, L = self.be, self.e, self.be.L
        prog, cfg = L.prog, L.cfg
        lib = ops.lib()
        N = self.N
        nslots = len(self.slots)
        H = cfg.image_size
        self._add(lib.dtf_weight_prep, _p(e.state), e.S, _p(be.conv_table_t), len(L.conv_table), _p(self.slots_t),
                  nslots, _p(be.wf), _p(be.wd), L.wtot, *self._zero_args())
        if self.src is not None:
            self._add("augment", None)
        else:
            self._add(lib.dtf_prep_input, _p(self.x_in), _p(self.xin16), N * H * H, 3)
        # ---------------- forward
        self._forward_v1()
        # head: GAP + dense + CE on the last block output (no final BN: gamma_off = -1)
        hw = L.final_hw
        hwork = self._head_work()
        ha_ = HeadArgs()
        ha_.x, ha_.labels, ha_.work = _p(self.xs[-1]), _p(self.labels), _p(hwork)
        ha_.params, ha_.p_mstride = _p(e.state), e.S
        ha_.gamma_off, ha_.beta_off = -1, -1
        ha_.dw_off, ha_.db_off = prog.dense_w_off, prog.dense_b_off
        ha_.grads, ha_.g_mstride = _p(e.grads), e.Pp
        ha_.st_f, ha_.st_b, ha_.cnt = _p(be.stats), _p(be.stats), _p(self.cnt)
        ha_.dfeat, ha_.loss, ha_.correct = _p(self.dfeat), _p(be.loss), _p(be.correct)
        ha_.logits_out = None
        ha_.hw, ha_.C, ha_.ncls, ha_.train = hw, cfg.final_size, cfg.num_classes, 1
        ha_.loss_scale = be.loss_scale
        self._head_slab(ha_, hwork)
        self._keep(ha_)
        self._add(lib.dtf_head, ctypes.byref(ha_), hwork.shape[0])
        # (the moving-statistics update of the forward BNs runs at the end of the step, with the BN gradients)
        # ---------------- backward
        hwL = self.xs[-1].shape[1]
        d = self.tmp[hwL]["g"][0]
        self._add(lib.dtf_head_bwd_apply, _p(self.xs[-1]), _p(self.dfeat), _p(d), _p(self.img_slot), _p(e.state),
                  e.S, -1, -1, _p(be.stats), _p(be.stats), _p(self.cnt), hw, cfg.final_size, N)
        chained = set()  # blocks whose BN_b backward sums the next block's conv_a epilogue already took
        for i in range(len(prog.blocks) - 1, -1, -1):
            blk = prog.blocks[i]
            bna, bnb = blk.bns
            ca, cb = blk.convs
            x, ha, hb = self.xs[i], self.hs[i], self.hb[i]
            Hi, Ho = x.shape[1], ha.shape[1]
            T, Tin = self.tmp[Ho], self.tmp[Hi]
            hp = self.scs[i]
            if i not in chained:
                self._bn_ew(lib.dtf_bn_bwd_reduce, (Ho * Ho, ha.shape[3]), bnb, hb,
                            bn2=blk.proj_bn if hp is not None else None, h2=hp, d=d)
            # conv_b: dy = BN_b-backward(d, hb); dz_a = dgrad masked by BN_a(ha) + BN_a reductions; dW_b
            self._conv_bwd_fused(cb, d, T["dz2"], ha, mode_dy=2, dy2=hb, dy_bn=bnb, x_bn=bna)
            res = d
            if hp is not None:
                res = self.pd[id(blk)]
                self._conv_dgrad(blk.proj, d, res, Hi, mode=2, epi=0, dy2=hp, in_bn=blk.proj_bn)
                self._conv_wgrad(blk.proj, x, d, mode_x=0, mode_dy=2, dy_bn=blk.proj_bn, dy2=hp)
            # conv_a: dy = BN_a-backward(dz_a, ha); + shortcut grad; mask by x > 0 -> previous block's d
            d_next = Tin["g"][1] if d is Tin["g"][0] else Tin["g"][0]
            ca_spec = prog.convs[ca]
            if ca_spec.stride == 1 and ca_spec.cin == ca_spec.cout:
                # d_next = dL/d(block i-1's pre-ReLU sum): block i-1's BN_b sums ride in this epilogue when that
                # block has no projection BN (which would need a second x-hat) and the build is not deterministic
                # (whose BN_b reduction is the per-image fixed-order pass)
                chain = (i > 0 and prog.blocks[i - 1].proj is None and not self.be.det and V1_CHAIN_BN)
                if chain:
                    chained.add(i - 1)
                self._conv_bwd_fused(ca, T["dz2"], d_next, x, mode_dy=2, dy2=ha, dy_bn=bna, res=res, ident_x=True,
                                     chain_bn=prog.blocks[i - 1].bns[1] if chain else None,
                                     chain_h=self.hb[i - 1] if chain else None)
            else:
                self._conv_dgrad(ca, T["dz2"], d_next, Hi, mode=2, epi=1 | 4, dy2=ha, in_bn=bna, res=res, xm=x)
                self._conv_wgrad(ca, x, T["dz2"], mode_x=0, mode_dy=2, dy_bn=bna, dy2=ha)
            d = d_next
        # stem: BN_stem reductions of d (= dL/d relu-input of the stem), then wgrad with BN_stem-backward on load
        self._bn_ew(lib.dtf_bn_bwd_reduce, (H * H, cfg.num_filters), prog.stem_bn, self.h0, d=d)
        self._conv_wgrad(prog.stem, self.xin16, d, mode_x=0, mode_dy=2, dy_bn=prog.stem_bn, dy2=self.h0,
                         cin_real=cfg.in_channels)
        self._flush_slab()
        self._flush_deferred()
        self._add(lib.dtf_bn_step_end, _p(e.state), e.S, 3 * e.Pp, _p(be.bn_table_t), len(L.bn_table),
                  _p(be.stats[0]), _p(be.stats[1]), be.stats_bn_stride, _p(self.slots_t), nslots, _p(self.cnt),
                  _p(e.grads), e.Pp)
        self._add("optim", None)
        self._add("step", None)

    # -------------------------------------------------------------------- execution
    def slot_index(self, slots):
        """Positions of ``slots`` in this plan's member list (device tensor, cached)."""
        key = tuple(slots)
        cache = self.__dict__.setdefault("_slot_index", {})
        if key not in cache:
            pos = {s: i for i, s in enumerate(self.slots)}
            cache[key] = torch.tensor([pos[s] for s in slots], dtype=torch.long, device=self.be.dev)
        return cache[key]

    def load_batch(self, batches, slots=None):
        """Stage the members' batches (``slots``: the members they belong to, default every plan member)."""
        slots = list(self.slots) if slots is None else [s for s in self.slots if s in set(slots)]
        # member regions start at self.first[slot] (packed for exact plans, capacity-strided for elastic ones)
        if self.src is None and same_batches(self, batches):
            return  # the staged copy is still current (same unmodified source storage)
        if self.src is not None:
            for s, b in zip(slots, batches):
                n, off = len(b), self.first[s]
                self.idx[off:off + n].copy_(b.idx, non_blocking=True)
            if getattr(self, "_rng_stage", None) is None:
                self._rng_stage = PinnedStager(2, torch.int32)
            self._rng_stage.upload(self.rng, self.src.next_rng())
            return
        for s, (x, y) in zip(slots, batches):
            n, off = x.shape[0], self.first[s]
            self.x_in[off:off + n].copy_(x.reshape(n, *self.x_in.shape[1:]), non_blocking=True)
            self.labels[off:off + n].copy_(y, non_blocking=True)

    def _run_eager(self):
        e = self.e
        main = torch.cuda.current_stream() if self.be.dev.type == "cuda" else None
        target = None  # None: the current stream; else the side stream of a fork
        for fn, args in self.launches:
            if fn == "fork":  # the side stream waits for everything issued so far on the main stream
                if getattr(self, "_side", None) is None:
                    self._side = torch.cuda.Stream(device=self.be.dev)
                self._side.wait_stream(main)
                target = self._side
            elif fn == "endfork":
                target = None
            elif fn == "join":
                main.wait_stream(self._side)
            elif target is not None:
                err = fn(*args, target.cuda_stream)
                if err != 0:
                    raise RuntimeError("kernel launch %s failed with %d" % (getattr(fn, "__name__", fn), err))
            elif fn == "augment":
                # crops keyed per member (its step counter + dataset row): placement-invariant (data.hip)
                ops.augment_cifar(self.src.train_x, self.src.train_y, self.idx, self.rng, True, out16=self.xin16,
                                  lab32=self.labels, member_keys=(self.img_slot, e.state, e.S, 3 * e.Pp + e.R))
            elif fn == "optim":
                e.dp_sync_grads(self.slots)  # data-parallel member groups only (no-op otherwise)
                ops.fused_optimizer(e.state, e.grads, e.hyper, e.Pp, e.P, e.n_reg, shadow=None, zero_grads=True,
                                    grad_scale=1.0 / self.be.loss_scale)
            elif fn == "step":
                # step counters + per-member losses gathered inside the step (graph) so a replay leaves one copy
                # for loss_view
                advance_steps(e, self.slots_long, self.slots_t, self.be.loss, self.loss_sel, ring=self.ring)
            else:
                err = fn(*args, ops.stream())
                if err != 0:
                    raise RuntimeError("kernel launch %s failed with %d" % (getattr(fn, "__name__", fn), err))

    def run_eval(self):
        assert self.eval
        self._run_eager()

    def run(self, train=True):
        run_captured(self)
        if self.ring is not None:
            self.ring.advance()

    def loss_view(self):
        # callers keep per-step losses across later replays (engine_model.loss_acc): a ring row (valid for
        # LossRing.ROWS steps), else a copy
        return self.ring.last() if self.ring is not None else self.loss_sel.clone()
