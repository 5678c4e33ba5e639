"""Stride-1 3x3 conv kernel with LDS-resident input rows (ops/csrc/convg.hip convg_t3_kernel) vs fp32 PyTorch.

Forward (statistics epilogue) and data gradient (A operand from the forward weight layout, ReLU mask by BN(xm),
BN-backward statistics) at every instantiated geometry: 56 x 56 x 64 (8-row tiles of 448 pixels), 28 x 28 x 128
(8-row tiles) and 14 x 14 x 256 (whole images in 224-pixel tiles); two members with their own weight rows.
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CMAX = 512


def _relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("hw,c", [(56, 64), (28, 128), (14, 256)])
@pytest.mark.parametrize("dgrad", [False, True])
@pytest.mark.parametrize("flags", [1, 0])  # 1: staged A (product default, hip_imagenet.T3_FLAGS); 0: direct A
def test_convg_t3_matches_torch(hw, c, dgrad, flags):
    from distributedtf_amd import ops
    from distributedtf_amd.engine import hip_imagenet as hi
    hi._register()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(hw + int(dgrad))
    slots = [0, 0, 1]  # image -> member
    n = len(slots)
    x = torch.randn(n, hw, hw, c, generator=g).bfloat16()
    w = (torch.randn(2, c, 3, 3, c, generator=g) / (3 * c ** 0.5)).bfloat16()  # [member][o][ky][kx][i]
    xm = torch.randn(n, hw, hw, c, generator=g).bfloat16()
    ep = torch.zeros(2, 4, CMAX)
    ep[:, 0, :c] = 1.0 + 0.1 * torch.randn(2, c, generator=g)
    ep[:, 1, :c] = 0.1 * torch.randn(2, c, generator=g)
    ep[:, 2, :c] = 0.1 * torch.randn(2, c, generator=g)
    ep[:, 3, :c] = 1.0 + 0.1 * torch.rand(2, c, generator=g)
    xd, wd, xmd, epd = x.to(dev), w.to(dev), xm.to(dev), ep.to(dev)
    y = torch.zeros(n, hw, hw, c, dtype=torch.bfloat16, device=dev)
    st = torch.zeros(2, 2, CMAX, device=dev)
    rows = hi._CG_T3[hw]
    tc = 64 if hw == 56 else 128
    items = []
    for img, s in enumerate(slots):
        for y0 in range(0, hw, rows):
            p0 = (img * hw + y0) * hw
            for o0 in range(0, c, tc):
                items.append([s, p0, p0 + rows * hw, o0])
    work = torch.tensor(items, dtype=torch.int32, device=dev)
    a = hi.CgArgs()
    a.x, a.y, a.w, a.work, a.st_out = xd.data_ptr(), y.data_ptr(), wd.data_ptr(), work.data_ptr(), st.data_ptr()
    a.w_mstride, a.w_off = c * 9 * c, 0
    a.Hi = a.Wi = a.Ho = a.Wo = hw
    a.Ci = a.Co = c
    a.kh = a.kw = 3
    a.stride, a.pad = 1, 1
    a.cmax = CMAX
    a.log2ci = c.bit_length() - 1
    a.flags = flags
    if dgrad:
        a.xm, a.c_ep = xmd.data_ptr(), epd.data_ptr()
    rc = ops.lib().dtf_convg_t3(ctypes.byref(a), tc, 6 if dgrad else 4, int(dgrad), hw, work.shape[0], 0,
                                ops.stream())  # mode 0: plain operand (no folded BN)
    assert rc == 0, rc
    torch.cuda.synchronize()
    yh, sth = y.float().cpu(), st.cpu()
    xf = x.float().permute(0, 3, 1, 2)
    for s in (0, 1):
        sel = [i for i, t in enumerate(slots) if t == s]
        wo = w[s].float().permute(0, 3, 1, 2)  # [o][i][ky][kx]
        if dgrad:
            ref = F.conv_transpose2d(xf[sel], wo, padding=1).permute(0, 2, 3, 1)
            xms = xm[sel].float()
            keep = xms * ep[s, 0, :c] + ep[s, 1, :c] > 0
            ref = torch.where(keep, ref, torch.zeros_like(ref))
            xhat = (xms - ep[s, 2, :c]) * ep[s, 3, :c]
            out = yh[sel]
            s0, s1 = out.sum((0, 1, 2)), (out * xhat).sum((0, 1, 2))
        else:
            ref = F.conv2d(xf[sel], wo, padding=1).permute(0, 2, 3, 1)
            out = yh[sel]
            s0, s1 = out.sum((0, 1, 2)), (out * out).sum((0, 1, 2))
        assert _relerr(out, ref) < 1e-2, (s, _relerr(out, ref))
        assert _relerr(sth[s, 0, :c], s0) < 1e-3 and _relerr(sth[s, 1, :c], s1) < 1e-3
