"""The reference's block goldens through the HIP kernels.

tests/test_golden_fixtures.py checks ``resnet/official/utils/testing/reference_data/resnet/*`` (TF tensor-bundle
checkpoints + results.json: [input shape, first, last, sum, output shape, first, last, sum]) against the PyTorch
block.  Here the same eight block fixtures -- v1 / v2 x building / bottleneck x with / without projection, batch 32,
8 x 8, 4 channels -- run through the large-channel HIP kernels the ImageNet step uses (engine/hip_block.py:
convg implicit-GEMM convs with BN-statistic epilogues, cg_chan_stats, cg_bn_final, cg_bn_relu_apply,
cg_bn_add_relu), channels zero-padded to the kernels' 8-wide minimum.  Checked:

  * the fixture's output shape and first / last / sum within bf16 tolerance (the kernels store bf16
    activations; the fixture is fp32 TF);
  * the whole output against the fp32 PyTorch block on the same weights (rel. L2 <= 2 %);
  * the padding contributes nothing: every padded output channel is exactly 0.
"""
import json
import os

import numpy as np
import pytest
import torch

from distributedtf_amd.models import resnet
from distributedtf_amd.utils.tf_bundle import load_bundle

# data-only copies of the reference fixtures (tests/fixtures/reference_resnet/README.md): the GPU box has no
# /root/reference
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "reference_resnet")
pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.isdir(ROOT), reason="fixtures not present")]

BLOCKS = [(b, p, v) for b in (False, True) for p in (False, True) for v in (1, 2)]


def _load(bottleneck, projection, version):
    name = "batch-size-32_%s%s_version-%d_width-8_channels-4" % (
        "bottleneck" if bottleneck else "building", "_projection" if projection else "", version)
    d = os.path.join(ROOT, name)
    t = load_bundle(os.path.join(d, "model.ckpt"))
    res = json.load(open(os.path.join(d, "results.json")))
    channels = 4
    stride, cout = (2, 2 * channels) if projection else (1, channels)
    filters = cout // 4 if bottleneck else cout
    prog, blk = resnet.single_block_program(channels, filters, stride, projection, version, bottleneck)
    params = torch.zeros(prog.n_params)
    for i, c in enumerate(prog.convs):  # TF creation order = single_block_program order (test_golden_fixtures.py)
        k = t["conv2d%s/kernel" % ("_%d" % i if i else "")]  # HWIO -> OHWI
        params[c.off:c.off + c.numel] = torch.from_numpy(np.ascontiguousarray(k.transpose(3, 0, 1, 2))).flatten()
    for i, b in enumerate(prog.bns):
        pre = "batch_normalization%s/" % ("_%d" % i if i else "")
        params[b.gamma_off:b.gamma_off + b.c] = torch.from_numpy(t[pre + "gamma"])
        params[b.beta_off:b.beta_off + b.c] = torch.from_numpy(t[pre + "beta"])
    return name, prog, blk, params, torch.from_numpy(t["input_tensor"]), res


@pytest.mark.parametrize("bottleneck,projection,version", BLOCKS)
def test_hip_block_matches_reference_golden(bottleneck, projection, version):
    from distributedtf_amd.engine.hip_block import HipBlockForward
    name, prog, blk, params, x, res = _load(bottleneck, projection, version)
    dev = torch.device("cuda")
    run = HipBlockForward(prog, blk, dev)
    yp = run(params, x, keep_padding=True).cpu()
    cout = prog.convs[blk.convs[-1]].cout
    y = yp[..., :cout]
    assert torch.count_nonzero(yp[..., cout:]) == 0, "padded channels must stay exactly zero"
    # fixture summary: [input shape (4), first, last, sum, output shape (4), first, last, sum]
    out = res[7:]
    assert list(y.shape) == out[:4], (name, y.shape, out[:4])
    flat = y.double().reshape(-1)
    first, last, total = out[4:7]
    tol = lambda v: 3e-2 * abs(v) + 3e-2  # noqa: E731  bf16 activations (8 mantissa bits) through 2-3 convs
    assert abs(float(flat[0]) - first) <= tol(first), (name, "first", float(flat[0]), first)
    assert abs(float(flat[-1]) - last) <= tol(last), (name, "last", float(flat[-1]), last)
    assert abs(float(flat.sum()) - total) <= 1e-2 * float(flat.abs().sum()) + 0.5, (name, "sum", float(flat.sum()),
                                                                                   total)
    # the whole tensor against the fp32 PyTorch block (itself pinned to the fixture by test_golden_fixtures.py)
    ref = resnet.block_forward(prog, params, torch.zeros(prog.n_running), x.permute(0, 3, 1, 2), blk, training=True,
                               update_running=False).permute(0, 2, 3, 1)
    rel = float((y.double() - ref.double()).norm() / ref.double().norm())
    print("%s: first %.5f/%.5f last %.5f/%.5f sum %.3f/%.3f rel %.2e" % (name, float(flat[0]), first, float(flat[-1]),
                                                                       last, float(flat.sum()), total, rel))
    assert rel < 2e-2, (name, rel)
