"""One residual block, training-mode forward, on the large-channel HIP kernels (ops/csrc/convg.hip, convg_aux.hip).

The population engines run whole networks as captured launch lists; this runs a SINGLE block of any of the four
reference variants (``resnet_model.py:127-320``: v1 / v2 x building / bottleneck, with or without the projection
shortcut) through the same kernels the ImageNet step uses -- implicit-GEMM convolutions with BN-statistic
epilogues (convg_fwd), channel statistics of a tensor no conv produced (cg_chan_stats), BN finalize
(cg_bn_final), BN + ReLU apply (cg_bn_relu_apply) and the v1 BN + shortcut + ReLU (cg_bn_add_relu) -- so a block can
be checked against the reference's own block fixtures (``resnet/official/utils/testing/reference_data/resnet``,
tests/test_gpu_golden_hip.py) at their shape (batch 32, 8 x 8, 4 channels).

Channel padding: the kernels need power-of-two channel counts >= 8.  Every tensor is carried with its channels
zero-padded to ``_cpad(c)``; the padded input channels meet zero weights and the padded output channels get zero
weights, so their conv outputs are exactly 0.  Their BatchNorm has mean 0, variance 0 and beta 0 -> output
0 * gamma * rsqrt(eps) + 0 = 0, and ReLU(0) = 0: a padded channel never contributes to a real one, which the caller
can verify by reading the returned padded tensor (``forward(..., keep_padding=True)``).
"""

from __future__ import annotations

import ctypes
from typing import Dict

import torch

from .. import ops
from . import hip_imagenet as hi

c_int = ctypes.c_int


def _cpad(c: int) -> int:
    p = 8
    while p < c:
        p *= 2
    return p


class HipBlockForward:
    """``HipBlockForward(prog, blk, device)(params, x)`` -> the block output (NHWC fp32), training-mode BN.

    ``prog`` / ``blk``: a ResNetProgram and its BlockSpec (``models.resnet.single_block_program``); ``params``: the
    program's flat fp32 parameter row (conv kernels OHWI at ``conv.off``, BN gamma / beta); ``x``: NHWC fp32."""

    def __init__(self, prog, blk, device):
        hi._register()
        self.prog, self.blk, self.dev = prog, blk, torch.device(device)
        self.v1 = prog.cfg.version == 1
        cs = [prog.convs[i] for i in ([blk.proj] if blk.proj is not None else []) + list(blk.convs)]
        self.cmax = max(_cpad(max(c.cin, c.cout)) for c in cs)
        self.acc_dtype = torch.int64 if ops.lib().dtf_fixed_acc() else torch.float32

    # ---------------------------------------------------------------------------------------------- helpers
    def _bn_state(self, params):
        """One state row: per BN padded gamma (pad 1) / beta (pad 0) + a scratch for the running statistics."""
        off, lay = 0, {}
        for b in self.prog.bns:
            cp = _cpad(b.c)
            lay[b.idx] = (off, off + cp, off + 2 * cp, cp)
            off += 4 * cp
        st = torch.zeros(1, max(off, 1), dtype=torch.float32)
        for b in self.prog.bns:
            g, be, _, cp = lay[b.idx]
            st[0, g:g + cp] = 1.0
            st[0, g:g + b.c] = params[b.gamma_off:b.gamma_off + b.c].float().cpu()
            st[0, be:be + b.c] = params[b.beta_off:b.beta_off + b.c].float().cpu()
        return st.to(self.dev), lay

    def _weights(self, params, ci):
        """Conv ``ci``: padded OHWI bf16 rows [cout_p][k][k][cin_p]."""
        c = self.prog.convs[ci]
        w = params[c.off:c.off + c.numel].float().cpu().view(c.cout, c.k, c.k, c.cin)
        wp = torch.zeros(_cpad(c.cout), c.k, c.k, _cpad(c.cin))
        wp[:c.cout, :, :, :c.cin] = w
        return wp.to(ops.act_dtype()).to(self.dev).contiguous()

    def _conv(self, ci, w, src, out, epi=0, res=None, st=None):
        c = self.prog.convs[ci]
        N, Hi, _, Cip = src.shape
        Ho = (Hi + c.stride - 1) // c.stride
        Cop = _cpad(c.cout)
        assert out.shape == (N, Ho, Ho, Cop) and Cip == _cpad(c.cin)
        a = hi.CgArgs()
        a.x, a.y, a.res = src.data_ptr(), out.data_ptr(), None if res is None else res.data_ptr()
        a.w, a.w_mstride, a.w_off = w.data_ptr(), w.numel(), 0
        a.st_out = None if st is None else st.data_ptr()
        a.Hi = a.Wi = Hi
        a.Ho = a.Wo = Ho
        a.Ci, a.Co = Cip, Cop
        a.kh = a.kw = c.k
        a.stride, a.pad = c.stride, (c.k - 1) // 2  # 'SAME' (stride 1) / fixed_padding + 'VALID' (resnet_model.py:55-92)
        a.cmax = self.cmax
        a.log2ci = hi._log2(Cip)
        a.cin_real = 0
        tc = 128 if Cop >= 128 else 64
        items = [[0, p0, min(p0 + 128, N * Ho * Ho), o0] for p0 in range(0, N * Ho * Ho, 128)
                 for o0 in range(0, Cop, tc)]
        work = torch.tensor(items, dtype=torch.int32, device=self.dev)
        a.work = work.data_ptr()
        self._keep += [a, work]
        ops.check(ops.lib().dtf_convg_fwd(ctypes.byref(a), tc, 0, epi, 0, work.shape[0], ops.stream()),
                  "convg_fwd (block conv %d)" % ci)

    def _final(self, bn, sums, coef, hw):
        g, be, run, cp = self.lay[bn]
        a = hi.BnFinArgs()
        a.state, a.s_mstride = self.state.data_ptr(), self.state.shape[1]
        a.sums, a.coef, a.fcoef = sums.data_ptr(), coef.data_ptr(), None
        a.grads, a.g_mstride = None, 0
        a.slots, a.cnt = self.slots.data_ptr(), self.cnt.data_ptr()
        a.gamma_off, a.beta_off, a.run_off = g, be, run
        a.C, a.hw, a.cmax = cp, hw, self.cmax
        self._keep.append(a)
        ops.check(ops.lib().dtf_cg_bn_final(ctypes.byref(a), 0, 1, ops.stream()), "cg_bn_final")

    def _relu_apply(self, h, coef, out):
        a = hi.EwArgs()
        a.dz, a.h, a.add, a.out, a.coef = None, h.data_ptr(), None, out.data_ptr(), coef.data_ptr()
        a.img_slot, a.hw, a.C, a.cmax, a.nimg = self.img_slot.data_ptr(), h.shape[1] * h.shape[2], h.shape[3], \
            self.cmax, h.shape[0]
        self._keep.append(a)
        ops.check(ops.lib().dtf_cg_bn_relu_apply(ctypes.byref(a), ops.stream()), "cg_bn_relu_apply")

    def _sums(self):
        return torch.zeros(1, 2, self.cmax, dtype=self.acc_dtype, device=self.dev)

    def _coef(self):
        return torch.zeros(1, 4, self.cmax, dtype=torch.float32, device=self.dev)

    def _act(self, n, hw, c):
        return torch.zeros(n, hw, hw, _cpad(c), dtype=ops.act_dtype(), device=self.dev)

    # ---------------------------------------------------------------------------------------------- forward
    @torch.no_grad()
    def forward(self, params: torch.Tensor, x: torch.Tensor, keep_padding: bool = False) -> torch.Tensor:
        prog, blk = self.prog, self.blk
        N, H, _, C = x.shape
        self._keep = []
        self.state, self.lay = self._bn_state(params)
        self.slots = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.cnt = torch.full((1,), float(N), dtype=torch.float32, device=self.dev)
        self.img_slot = torch.zeros(N, dtype=torch.int32, device=self.dev)
        xb = self._act(N, H, C)
        xb[..., :C] = x.to(self.dev).to(xb.dtype)
        W: Dict[int, torch.Tensor] = {ci: self._weights(params, ci) for ci in
                                      ([blk.proj] if blk.proj is not None else []) + list(blk.convs)}
        convs = [prog.convs[i] for i in blk.convs]
        hws = [H]
        for c in convs:
            hws.append((hws[-1] + c.stride - 1) // c.stride)
        Ho = hws[-1]
        fout = convs[-1].cout
        L = ops.lib()
        if not self.v1:
            # pre-activation: BN1 statistics of the block input, relu(BN1(x)) feeds the projection and conv 1
            s0, k0 = self._sums(), self._coef()
            ops.check(L.dtf_cg_chan_stats(xb.data_ptr(), self.img_slot.data_ptr(), s0.data_ptr(), N, H * H,
                                          xb.shape[3], self.cmax, ops.stream()), "cg_chan_stats")
            self._final(blk.bns[0], s0, k0, H * H)
            pre = torch.empty_like(xb)
            self._relu_apply(xb, k0, pre)
            short = xb
            if blk.proj is not None:
                short = self._act(N, Ho, fout)
                self._conv(blk.proj, W[blk.proj], pre, short, epi=0)
            h = pre
            for j, ci in enumerate(blk.convs):
                last = j + 1 == len(blk.convs)
                out = self._act(N, hws[j + 1], prog.convs[ci].cout)
                s, k = self._sums(), self._coef()
                # every conv's epilogue reduces its output's statistics (the next BN's; the block output's are the
                # next block's BN1 -- drained into a scratch here) and the last adds the shortcut
                self._conv(ci, W[ci], h, out, epi=5 if last else 4, res=short if last else None, st=s)
                if last:
                    h = out
                    break
                self._final(blk.bns[j + 1], s, k, hws[j + 1] ** 2)
                h = torch.empty_like(out)
                self._relu_apply(out, k, h)
        else:
            short, ks = xb, None
            if blk.proj is not None:
                short = self._act(N, Ho, fout)
                sp, ks = self._sums(), self._coef()
                self._conv(blk.proj, W[blk.proj], xb, short, epi=4, st=sp)
                self._final(blk.proj_bn, sp, ks, Ho * Ho)
            h = xb
            for j, ci in enumerate(blk.convs):
                out = self._act(N, hws[j + 1], prog.convs[ci].cout)
                s, k = self._sums(), self._coef()
                self._conv(ci, W[ci], h, out, epi=4, st=s)
                self._final(blk.bns[j], s, k, hws[j + 1] ** 2)
                if j + 1 < len(blk.convs):
                    h = torch.empty_like(out)
                    self._relu_apply(out, k, h)
                    continue
                # relu(BN_last(h) + shortcut), the shortcut through its projection BN when there is one
                y = torch.empty_like(out)
                a = hi.BnAddArgs()
                a.h, a.s, a.out = out.data_ptr(), short.data_ptr(), y.data_ptr()
                a.coef_h, a.coef_s = k.data_ptr(), None if ks is None else ks.data_ptr()
                a.img_slot, a.hw, a.C, a.cmax, a.nimg = self.img_slot.data_ptr(), Ho * Ho, y.shape[3], self.cmax, N
                self._keep.append(a)
                ops.check(L.dtf_cg_bn_add_relu(ctypes.byref(a), ops.stream()), "cg_bn_add_relu")
                h = y
        torch.cuda.synchronize(self.dev)
        self._keep = []
        return h.float() if keep_padding else h[..., :fout].float()

    __call__ = forward
