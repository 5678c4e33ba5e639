"""Golden-value regression against the reference's own numerics fixtures.

The reference ships TF 1.8 tensor-bundle checkpoints + ``results.json`` for a BN
layer and every ResNet block variant (v1/v2 x building/bottleneck x projection,
batch 32, width 8, 4 channels) under
``resnet/official/utils/testing/reference_data`` (produced by the
upstream block test, which the reference tree does not contain).  Each
checkpoint holds the block's weights AND its input tensor; ``results.json`` is
``[input shape..., first, last, sum, output shape..., first, last, sum]`` of the
NHWC tensors.  The files are read with the pure-Python bundle parser
(``utils/tf_bundle.py``: no code from the files runs) and our block
implementation (``models/resnet.block_forward``, training-mode BN) must
reproduce the outputs.
"""
import json
import os

import numpy as np
import pytest
import torch

from distributedtf_amd.models import resnet
from distributedtf_amd.utils.tf_bundle import load_bundle

ROOT = "/root/reference/resnet/official/utils/testing/reference_data"
pytestmark = pytest.mark.skipif(not os.path.isdir(ROOT), reason="reference fixtures not present")

BLOCKS = [(b, p, v) for b in (False, True) for p in (False, True) for v in (1, 2)]


def _fixture(name):
    d = os.path.join(ROOT, name)
    return load_bundle(os.path.join(d, "model.ckpt")), json.load(open(os.path.join(d, "results.json")))


def _check_summary(arr, expect, what):
    a = np.asarray(arr, dtype=np.float64)
    nd = a.ndim
    assert list(a.shape) == expect[:nd], (what, a.shape, expect[:nd])
    first, last, total = expect[nd:nd + 3]
    flat = a.reshape(-1)
    np.testing.assert_allclose(flat[0], first, rtol=1e-4, atol=1e-5, err_msg=what + " first")
    np.testing.assert_allclose(flat[-1], last, rtol=1e-4, atol=1e-5, err_msg=what + " last")
    # the fixture sums were accumulated in fp32 by TF: for a near-zero-mean tensor (BN output) the rounding of
    # the accumulation dominates, so the absolute slack scales with sum(|x|)
    np.testing.assert_allclose(flat.sum(), total, rtol=2e-5, atol=max(5e-3, 5e-6 * np.abs(flat).sum()),
                               err_msg=what + " sum")
    return expect[nd + 3:]


def test_bundle_parser_uniform_random():
    t, res = _fixture("reference_data_test/uniform_random")
    assert t["input_tensor"].shape == (1, 1)
    np.testing.assert_allclose(t["input_tensor"].reshape(-1)[0], res[0], rtol=1e-7)


def test_dense_stack():
    t, res = _fixture("reference_data_test/dense")
    x = t["input_tensor"]
    h = x @ t["dense/kernel"] + t["dense/bias"]
    y = h @ t["dense_1/kernel"] + t["dense_1/bias"]
    _check_summary(y, res, "dense")


def test_batch_norm_training():
    t, res = _fixture("resnet/batch_norm")
    x = torch.from_numpy(t["input_tensor"])  # NHWC
    rest = _check_summary(x, res, "input")
    prog, _ = resnet.single_block_program(3, 3, 1, False, 2, False)
    params = torch.zeros(prog.n_params)
    running = torch.zeros(prog.n_running)
    b = prog.bns[0]
    params[b.gamma_off:b.gamma_off + 3] = torch.from_numpy(t["batch_normalization/gamma"])
    params[b.beta_off:b.beta_off + 3] = torch.from_numpy(t["batch_normalization/beta"])
    y = resnet._bn(prog, params, running, x.permute(0, 3, 1, 2), 0, True, False)
    _check_summary(y.permute(0, 2, 3, 1).numpy(), rest, "bn output")


@pytest.mark.parametrize("bottleneck,projection,version", BLOCKS)
def test_resnet_block(bottleneck, projection, version):
    name = "resnet/batch-size-32_%s%s_version-%d_width-8_channels-4" % (
        "bottleneck" if bottleneck else "building", "_projection" if projection else "", version)
    t, res = _fixture(name)
    channels = 4
    stride, cout = (2, 2 * channels) if projection else (1, channels)
    filters = cout // 4 if bottleneck else cout
    prog, blk = resnet.single_block_program(channels, filters, stride, projection, version, bottleneck)
    params = torch.zeros(prog.n_params)
    running = torch.zeros(prog.n_running)
    # TF names layers in creation order, which single_block_program mirrors: conv2d_<i> <-> convs[i],
    # batch_normalization_<i> <-> bns[i]
    for i, c in enumerate(prog.convs):
        k = t["conv2d%s/kernel" % ("_%d" % i if i else "")]  # HWIO
        assert k.shape == (c.k, c.k, c.cin, c.cout), (name, i, k.shape)
        params[c.off:c.off + c.numel] = torch.from_numpy(np.ascontiguousarray(k.transpose(3, 0, 1, 2))).flatten()
    for i, b in enumerate(prog.bns):
        pre = "batch_normalization%s/" % ("_%d" % i if i else "")
        params[b.gamma_off:b.gamma_off + b.c] = torch.from_numpy(t[pre + "gamma"])
        params[b.beta_off:b.beta_off + b.c] = torch.from_numpy(t[pre + "beta"])
    assert len([k for k in t if k.endswith("/kernel")]) == len(prog.convs)
    assert len([k for k in t if k.endswith("/gamma")]) == len(prog.bns)
    x = torch.from_numpy(t["input_tensor"])
    rest = _check_summary(x, res, name + " input")
    y = resnet.block_forward(prog, params, running, x.permute(0, 3, 1, 2), blk, training=True, update_running=False)
    _check_summary(y.permute(0, 2, 3, 1).detach().numpy(), rest, name + " output")

