"""ResNet v1/v2 (building + bottleneck) as a declarative layer program.

Architecture parity with the reference's vendored TF "official" ResNet
(``resnet/resnet_model.py``):
  * BN momentum 0.997, eps 1e-5, gamma/beta trainable (``:34-52``);
  * stride-2 convs pad ``(k-1)//2`` at the front, rest at the back (``:55-92``),
    which equals symmetric padding for k in {1, 3, 7};
  * conv ``use_bias=False``, initializer / regularizer from the hparams
    (``:80-121``); regularizer applies to conv kernels only;
  * blocks ``_building_block_v1/v2`` and ``_bottleneck_block_v1/v2``
    (``:127-320``), first block of every stage has a projection shortcut
    (``:323-359``), v2 projections take the pre-activated input;
  * v1 stem has BN+ReLU, v2 has a final BN+ReLU, then spatial mean + dense
    (``:487-554``); CIFAR config from ``cifar10_main.py:146-185`` (6n+2 depth,
    16 filters, strides [1,2,2], no pooling); ImageNet-shape ResNet-50
    (SURVEY.md C12'): 7x7/2 stem with 64 filters, 3x3/2 SAME max-pool,
    [3,4,6,3] bottleneck stages, strides [1,2,2,2], final size 2048.

Memory layout is MI355X-first: activations NHWC, conv weights OHWI
(``[Cout][kh][kw][Cin]``, K-contiguous for the MFMA A-operand), all trainable
parameters of one member in one flat fp32 vector (conv kernels first so the
regularizer covers a prefix), BN running stats in a second flat vector.

``forward_reference`` is the plain-PyTorch numerics oracle used by the tests;
the production hot path for the CIFAR configs is ``engine/hip_resnet.py``.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

BN_MOMENTUM = 0.997
BN_EPS = 1e-5


@dataclass
class ResNetConfig:
    resnet_size: int
    bottleneck: bool
    num_classes: int
    num_filters: int
    kernel_size: int
    conv_stride: int
    first_pool_size: Optional[int]
    first_pool_stride: Optional[int]
    block_sizes: List[int]
    block_strides: List[int]
    final_size: int
    version: int = 2
    image_size: int = 32
    in_channels: int = 3

    @property
    def name(self) -> str:
        shape = "cifar" if self.image_size == 32 else "imagenet%d" % self.image_size
        return "resnet%d_v%d_%s" % (self.resnet_size, self.version, shape)


def cifar_config(resnet_size: int = 56, version: int = 2, num_classes: int = 10) -> ResNetConfig:
    if resnet_size % 6 != 2:
        raise ValueError("resnet_size must be 6n + 2: %d" % resnet_size)
    n = (resnet_size - 2) // 6
    return ResNetConfig(resnet_size, False, num_classes, 16, 3, 1, None, None, [n] * 3, [1, 2, 2], 64,
                        version=version, image_size=32, in_channels=3)


_IMAGENET_BLOCKS = {18: ([2, 2, 2, 2], False), 34: ([3, 4, 6, 3], False), 50: ([3, 4, 6, 3], True),
                    101: ([3, 4, 23, 3], True), 152: ([3, 8, 36, 3], True), 200: ([3, 24, 36, 3], True)}


def imagenet_config(resnet_size: int = 50, version: int = 2, num_classes: int = 1001,
                    image_size: int = 224) -> ResNetConfig:
    blocks, bottleneck = _IMAGENET_BLOCKS[resnet_size]
    return ResNetConfig(resnet_size, bottleneck, num_classes, 64, 7, 2, 3, 2, blocks, [1, 2, 2, 2],
                        2048 if bottleneck else 512, version=version, image_size=image_size, in_channels=3)


# --------------------------------------------------------------------------- program

@dataclass
class ConvSpec:
    idx: int
    cin: int
    cout: int
    k: int
    stride: int
    off: int = 0          # offset of the OHWI weight in the flat param vector

    @property
    def numel(self):
        return self.cout * self.k * self.k * self.cin


@dataclass
class BNSpec:
    idx: int
    c: int
    gamma_off: int = 0
    beta_off: int = 0
    run_off: int = 0      # running mean at run_off, running var at run_off + c


@dataclass
class BlockSpec:
    stride: int
    convs: List[int]              # main-path convs in order
    bns: List[int]                # v2: pre-activation BNs (len == len(convs)); v1: post-conv BNs
    proj: Optional[int] = None    # projection conv
    proj_bn: Optional[int] = None  # v1 only


@dataclass
class ResNetProgram:
    cfg: ResNetConfig
    convs: List[ConvSpec] = field(default_factory=list)
    bns: List[BNSpec] = field(default_factory=list)
    blocks: List[BlockSpec] = field(default_factory=list)
    stem: int = 0
    stem_bn: Optional[int] = None
    final_bn: Optional[int] = None
    dense_w_off: int = 0
    dense_b_off: int = 0
    n_params: int = 0
    n_reg: int = 0        # conv-kernel prefix covered by the regularizer
    n_running: int = 0

    def conv(self, i) -> ConvSpec:
        return self.convs[i]


def build_program(cfg: ResNetConfig) -> ResNetProgram:
    prog = ResNetProgram(cfg)

    def conv(cin, cout, k, s):
        prog.convs.append(ConvSpec(len(prog.convs), cin, cout, k, s))
        return len(prog.convs) - 1

    def bn(c):
        prog.bns.append(BNSpec(len(prog.bns), c))
        return len(prog.bns) - 1

    prog.stem = conv(cfg.in_channels, cfg.num_filters, cfg.kernel_size, cfg.conv_stride)
    if cfg.version == 1:
        prog.stem_bn = bn(cfg.num_filters)
    cin = cfg.num_filters
    for stage, (nblocks, stride) in enumerate(zip(cfg.block_sizes, cfg.block_strides)):
        f = cfg.num_filters * (2 ** stage)
        fout = 4 * f if cfg.bottleneck else f
        for b in range(nblocks):
            s = stride if b == 0 else 1
            blk = BlockSpec(stride=s, convs=[], bns=[])
            if b == 0:
                blk.proj = conv(cin, fout, 1, s)
                if cfg.version == 1:
                    blk.proj_bn = bn(fout)
            if cfg.bottleneck:
                shapes = [(cin, f, 1, 1), (f, f, 3, s), (f, fout, 1, 1)]
            else:
                shapes = [(cin, f, 3, s), (f, f, 3, 1)]
            for (ci, co, k, st) in shapes:
                # v2: BN precedes each conv (on its input); v1: BN follows each conv
                if cfg.version == 2:
                    blk.bns.append(bn(ci))
                blk.convs.append(conv(ci, co, k, st))
                if cfg.version == 1:
                    blk.bns.append(bn(co))
            prog.blocks.append(blk)
            cin = fout
    if cfg.version == 2:
        prog.final_bn = bn(cin)
    assert cin == cfg.final_size, (cin, cfg.final_size)

    # flat layout: conv kernels (regularized prefix), BN gamma/beta, dense
    off = 0
    for c in prog.convs:
        c.off = off
        off += c.numel
    prog.n_reg = off
    for b in prog.bns:
        b.gamma_off = off
        b.beta_off = off + b.c
        off += 2 * b.c
    prog.dense_w_off = off
    off += cfg.num_classes * cfg.final_size
    prog.dense_b_off = off
    off += cfg.num_classes
    prog.n_params = off
    roff = 0
    for b in prog.bns:
        b.run_off = roff
        roff += 2 * b.c
    prog.n_running = roff
    return prog


# ------------------------------------------------------------------------ initialisation

def _trunc_normal_(t: torch.Tensor, std: float, gen: torch.Generator):
    # TF truncated_normal: resample |x| > 2 std
    t.normal_(0.0, 1.0, generator=gen)
    for _ in range(8):
        bad = t.abs() > 2.0
        if not bool(bad.any()):
            break
        t[bad] = torch.empty(int(bad.sum()), dtype=t.dtype).normal_(0.0, 1.0, generator=gen)
    t.clamp_(-2.0, 2.0).mul_(std)
    return t


def init_kernel(shape_ohwi: Tuple[int, ...], initializer: Optional[str], gen: torch.Generator) -> torch.Tensor:
    """Initialise an OHWI conv kernel (or [out, in] dense kernel) like TF1.

    ``glorot_normal`` / ``he_init`` use variance scaling with a truncated normal
    (stddev corrected by 0.8796), ``orthogonal`` a QR-orthogonal matrix over
    (fan_in, out), ``None`` -> glorot uniform (tf.layers default).
    """
    out = shape_ohwi[0]
    fan_in = int(math.prod(shape_ohwi[1:]))
    rf = int(math.prod(shape_ohwi[1:-1])) if len(shape_ohwi) > 2 else 1
    fan_out = out * rf
    w = torch.empty(shape_ohwi, dtype=torch.float32)
    if initializer == "glorot_normal":
        _trunc_normal_(w, math.sqrt(2.0 / (fan_in + fan_out)) / 0.87962566103423978, gen)
    elif initializer == "he_init":
        _trunc_normal_(w, math.sqrt(2.0 / fan_in) / 0.87962566103423978, gen)
    elif initializer == "orthogonal":
        rows, cols = fan_in, out
        a = torch.empty(max(rows, cols), min(rows, cols)).normal_(0.0, 1.0, generator=gen)
        q, r = torch.linalg.qr(a)
        q = q * torch.sign(torch.diagonal(r)).unsqueeze(0)
        if rows < cols:
            q = q.t()
        w = q[:rows, :cols].t().contiguous().reshape(shape_ohwi)
    else:
        lim = math.sqrt(6.0 / (fan_in + fan_out))
        w.uniform_(-lim, lim, generator=gen)
    return w


def init_params(prog: ResNetProgram, initializer: Optional[str], seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (flat params fp32 [P], flat running stats fp32 [R]) on CPU."""
    gen = torch.Generator().manual_seed(int(seed))
    p = torch.zeros(prog.n_params, dtype=torch.float32)
    for c in prog.convs:
        p[c.off:c.off + c.numel] = init_kernel((c.cout, c.k, c.k, c.cin), initializer, gen).flatten()
    for b in prog.bns:
        p[b.gamma_off:b.gamma_off + b.c] = 1.0
    cfg = prog.cfg
    dw = init_kernel((cfg.num_classes, cfg.final_size), None, gen)  # dense: glorot uniform
    p[prog.dense_w_off:prog.dense_w_off + dw.numel()] = dw.flatten()
    r = torch.zeros(prog.n_running, dtype=torch.float32)
    for b in prog.bns:
        r[b.run_off + b.c:b.run_off + 2 * b.c] = 1.0
    return p, r


# ---------------------------------------------------------------- reference forward

def conv_weight_oihw(prog: ResNetProgram, params: torch.Tensor, i: int) -> torch.Tensor:
    c = prog.convs[i]
    return params[c.off:c.off + c.numel].view(c.cout, c.k, c.k, c.cin).permute(0, 3, 1, 2)


def _conv(prog, params, x, i, dtype):
    c = prog.convs[i]
    w = conv_weight_oihw(prog, params, i).to(dtype)
    return F.conv2d(x, w, stride=c.stride, padding=(c.k - 1) // 2)


def _acc(t):
    """Accumulation precision of the oracle: fp32, or fp64 for a float64 run (the fp32 HIP step's tests compare
    against an fp64 evaluation of the same step)."""
    return t if t.dtype == torch.float64 else t.float()


def _bn(prog, params, running, x, i, training, update_running=True):
    b = prog.bns[i]
    g = params[b.gamma_off:b.gamma_off + b.c]
    be = params[b.beta_off:b.beta_off + b.c]
    rm = running[b.run_off:b.run_off + b.c]
    rv = running[b.run_off + b.c:b.run_off + 2 * b.c]
    if training:
        xf = _acc(x)
        mean = xf.mean(dim=(0, 2, 3))
        var = xf.var(dim=(0, 2, 3), unbiased=False)
        if update_running:
            n = xf.numel() // b.c
            with torch.no_grad():
                rm.mul_(BN_MOMENTUM).add_((1 - BN_MOMENTUM) * mean.detach())
                rv.mul_(BN_MOMENTUM).add_((1 - BN_MOMENTUM) * var.detach() * n / max(n - 1, 1))
    else:
        mean, var = rm, rv
    inv = torch.rsqrt(var + BN_EPS)
    y = (_acc(x) - mean[None, :, None, None]) * (inv * g)[None, :, None, None] + be[None, :, None, None]
    return y.to(x.dtype)


def block_forward(prog: ResNetProgram, params: torch.Tensor, running: torch.Tensor, x: torch.Tensor,
                  blk: BlockSpec, training: bool = True, dtype=torch.float32, update_running: bool = True):
    """One residual block on NCHW ``x`` (reference resnet_model.py:127-320).

    v2 (pre-activation, ``_building_block_v2`` / ``_bottleneck_block_v2``): BN+ReLU
    before every conv; the projection shortcut reads the pre-activated input.
    v1 (``_building_block_v1`` / ``_bottleneck_block_v1``): conv -> BN (-> ReLU),
    projection conv -> BN, ReLU after the residual add.
    """
    bn = lambda t, i: _bn(prog, params, running, t, i, training, update_running)  # noqa: E731
    if prog.cfg.version == 2:
        shortcut = x
        pre = F.relu(bn(x, blk.bns[0]))
        if blk.proj is not None:
            shortcut = _conv(prog, params, pre, blk.proj, dtype)
        h = _conv(prog, params, pre, blk.convs[0], dtype)
        for j in range(1, len(blk.convs)):
            h = F.relu(bn(h, blk.bns[j]))
            h = _conv(prog, params, h, blk.convs[j], dtype)
        return h + shortcut
    shortcut = x
    if blk.proj is not None:
        shortcut = bn(_conv(prog, params, x, blk.proj, dtype), blk.proj_bn)
    h = x
    n = len(blk.convs)
    for j in range(n):
        h = bn(_conv(prog, params, h, blk.convs[j], dtype), blk.bns[j])
        if j < n - 1:
            h = F.relu(h)
    return F.relu(h + shortcut)


def single_block_program(cin: int, filters: int, stride: int, projection: bool, version: int,
                         bottleneck: bool) -> Tuple[ResNetProgram, BlockSpec]:
    """A one-block program (flat parameter layout of build_program) for block-level tests."""
    cfg = ResNetConfig(resnet_size=0, version=version, bottleneck=bottleneck, num_classes=1, num_filters=filters,
                       kernel_size=3, conv_stride=1, first_pool_size=0, first_pool_stride=0, block_sizes=[1],
                       block_strides=[stride], final_size=(4 * filters if bottleneck else filters), image_size=0,
                       in_channels=cin)
    prog = ResNetProgram(cfg)
    fout = cfg.final_size
    blk = BlockSpec(stride=stride, convs=[], bns=[])

    def conv(ci, co, k, s):
        prog.convs.append(ConvSpec(len(prog.convs), ci, co, k, s))
        return len(prog.convs) - 1

    def bn(c):
        prog.bns.append(BNSpec(len(prog.bns), c))
        return len(prog.bns) - 1

    if projection:
        blk.proj = conv(cin, fout, 1, stride)
        if version == 1:
            blk.proj_bn = bn(fout)
    shapes = ([(cin, filters, 1, 1), (filters, filters, 3, stride), (filters, fout, 1, 1)] if bottleneck
              else [(cin, filters, 3, stride), (filters, filters, 3, 1)])
    for (ci, co, k, st) in shapes:
        if version == 2:
            blk.bns.append(bn(ci))
        blk.convs.append(conv(ci, co, k, st))
        if version == 1:
            blk.bns.append(bn(co))
    prog.blocks.append(blk)
    off = 0
    for c in prog.convs:
        c.off = off
        off += c.numel
    prog.n_reg = off
    for b in prog.bns:
        b.gamma_off, b.beta_off = off, off + b.c
        off += 2 * b.c
    prog.dense_w_off = prog.dense_b_off = off
    prog.n_params = off
    roff = 0
    for b in prog.bns:
        b.run_off = roff
        roff += 2 * b.c
    prog.n_running = roff
    return prog, blk


def forward_reference(prog: ResNetProgram, params: torch.Tensor, running: torch.Tensor, x_nhwc: torch.Tensor,
                      training: bool = True, dtype=torch.float32, update_running: bool = True) -> torch.Tensor:
    """Plain-PyTorch forward. ``x_nhwc`` [B, H, W, C]; returns fp32 logits [B, classes]."""
    cfg = prog.cfg
    x = x_nhwc.permute(0, 3, 1, 2).to(dtype)
    bn = lambda t, i: _bn(prog, params, running, t, i, training, update_running)  # noqa: E731
    x = _conv(prog, params, x, prog.stem, dtype)
    if cfg.version == 1:
        x = F.relu(bn(x, prog.stem_bn))
    if cfg.first_pool_size:
        # TF 'SAME' max-pool pads at the end only
        k, s = cfg.first_pool_size, cfg.first_pool_stride
        h = x.shape[-1]
        out = (h + s - 1) // s
        pad = max((out - 1) * s + k - h, 0)
        x = F.pad(x, (pad // 2, pad - pad // 2, pad // 2, pad - pad // 2), value=float("-inf"))
        x = F.max_pool2d(x, k, s)
    for blk in prog.blocks:
        x = block_forward(prog, params, running, x, blk, training, dtype, update_running)
    if cfg.version == 2:
        x = F.relu(bn(x, prog.final_bn))
    feat = _acc(x).mean(dim=(2, 3))
    w = params[prog.dense_w_off:prog.dense_w_off + cfg.num_classes * cfg.final_size].view(cfg.num_classes, cfg.final_size)
    b = params[prog.dense_b_off:prog.dense_b_off + cfg.num_classes]
    return feat @ w.t() + b


def regularization_loss(prog_n_reg: int, params: torch.Tensor, regularizer: Optional[str], weight_decay: float):
    """TF1 contrib regularizers over the conv-kernel prefix (tf.nn.l2_loss = sum/2)."""
    w = params[:prog_n_reg]
    if regularizer == "l2_regularizer":
        return weight_decay * 0.5 * (w * w).sum()
    if regularizer == "l1_regularizer":
        return weight_decay * w.abs().sum()
    if regularizer == "l1_l2_regularizer":
        return weight_decay * w.abs().sum() + weight_decay * 0.5 * (w * w).sum()
    return params.new_zeros(())


def tf_variables(prog: ResNetProgram, params, slot1, slot2, running, optimizer: str, step: int,
                 scope: str = "resnet_model", dtype="float32"):
    """The member's training state under the reference's TF variable names and layouts
    (``resnet_model.py``: ``tf.layers.conv2d`` kernels HWIO named conv2d, conv2d_1, .. in creation order;
    ``batch_normalization[_N]/{gamma,beta,moving_mean,moving_variance}``; ``dense/{kernel [C, classes], bias}``;
    optimizer slots; ``global_step``).  Inputs are 1-D numpy views of one state row."""
    from ..engine.optim import tf_optimizer_tensors
    cfg = prog.cfg
    out, trainable = {}, []

    def var(name, sl, reshape, layout):
        t = [layout(a[sl].reshape(reshape)).astype(dtype) for a in (params, slot1, slot2)]
        out[name] = t[0]
        trainable.append((name, t[0], t[1], t[2]))

    pre = scope + "/" if scope else ""
    for c in prog.convs:
        name = "%sconv2d%s/kernel" % (pre, "_%d" % c.idx if c.idx else "")
        var(name, slice(c.off, c.off + c.numel), (c.cout, c.k, c.k, c.cin), lambda w: w.transpose(1, 2, 3, 0))
    for b in prog.bns:
        base = "%sbatch_normalization%s" % (pre, "_%d" % b.idx if b.idx else "")
        var(base + "/gamma", slice(b.gamma_off, b.gamma_off + b.c), (b.c,), lambda v: v)
        var(base + "/beta", slice(b.beta_off, b.beta_off + b.c), (b.c,), lambda v: v)
        out[base + "/moving_mean"] = running[b.run_off:b.run_off + b.c].astype(dtype)
        out[base + "/moving_variance"] = running[b.run_off + b.c:b.run_off + 2 * b.c].astype(dtype)
    ncls, C = cfg.num_classes, cfg.final_size
    var(pre + "dense/kernel", slice(prog.dense_w_off, prog.dense_w_off + ncls * C), (ncls, C), lambda w: w.T)
    var(pre + "dense/bias", slice(prog.dense_b_off, prog.dense_b_off + ncls), (ncls,), lambda v: v)
    out.update(tf_optimizer_tensors(optimizer, trainable, step))
    return out


class ResNetArch:
    """Architecture handle consumed by ``engine.PopulationEngine``."""

    def __init__(self, cfg: ResNetConfig):
        self.cfg = cfg
        self.prog = build_program(cfg)
        self.n_params = self.prog.n_params
        self.n_running = self.prog.n_running
        self.n_reg = self.prog.n_reg
        self.num_classes = cfg.num_classes
        self.input_shape = (cfg.image_size, cfg.image_size, cfg.in_channels)
        # population-batched HIP kernels: CIFAR-shape building-block nets (v1 and v2, engine/hip_resnet.py) and
        # the ImageNet-shape v1 / v2 bottleneck nets (engine/hip_imagenet.py)
        self.hip_supported = ((cfg.image_size == 32 and not cfg.bottleneck and cfg.version in (1, 2))
                              or (cfg.bottleneck and cfg.version in (1, 2) and cfg.first_pool_size == 3
                                  and cfg.image_size % 32 == 0))

    @property
    def name(self):
        return self.cfg.name

    def init_params(self, initializer, seed):
        return init_params(self.prog, initializer, seed)

    def tf_variables(self, params, slot1, slot2, running, optimizer, step, dtype="float32"):
        return tf_variables(self.prog, params, slot1, slot2, running, optimizer, step, dtype=dtype)

    def forward(self, params, running, x_nhwc, training=True, dtype=torch.float32):
        return forward_reference(self.prog, params, running, x_nhwc, training=training, dtype=dtype)

    def flops_per_image(self) -> float:
        """Forward multiply-adds x2 of convs + dense (for MFU reporting)."""
        cfg, h = self.cfg, self.cfg.image_size
        total = 0.0
        hw = h // cfg.conv_stride
        total += 2.0 * hw * hw * self.prog.convs[self.prog.stem].numel
        if cfg.first_pool_size:
            hw = (hw + cfg.first_pool_stride - 1) // cfg.first_pool_stride
        for blk in self.prog.blocks:
            if blk.proj is not None:
                c = self.prog.convs[blk.proj]
                total += 2.0 * (hw // c.stride) ** 2 * c.numel
            cur = hw
            for ci in blk.convs:
                c = self.prog.convs[ci]
                cur = cur // c.stride
                total += 2.0 * cur * cur * c.numel
            hw = hw // blk.stride
        total += 2.0 * cfg.final_size * cfg.num_classes
        return total
