"""fp16 HIP step (--dtype fp16): the half build of the bf16 kernels (ops/csrc/common.h DTF_HALF -- fp16 activation /
weight-shadow storage, v_mfma_f32_16x16x32_f16) with the reference's static loss scaling
(resnet/official/utils/flags/_performance.py:30-33,105-108: fp16 -> loss_scale 128; resnet_run_loop.py:284-294:
gradients of loss_scale * loss, divided by loss_scale before the update).

Like tests/test_gpu_resnet_step.py: one gradient-descent step (lr = 1) of a ragged two-member population turns the
parameter delta into the gradient, compared PER LAYER with the fp32 PyTorch oracle within 2.5x what a bf16 PyTorch
run of the same step deviates (floor 6 %), plus the loss.  Runs in a child process: the fp16 library is chosen at
load time (DTF_HALF=1, ops.lib()), one per process.  Covers the CIFAR ResNet v2 step and the ImageNet-shape
bottleneck v2 step (64 x 64 input), and that the unscale matches the scale: loss scales 128 and 2^15 give the
same update up to fp16 rounding."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, torch
from distributedtf_amd import ops
from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.resnet import ResNetArch, cifar_config, imagenet_config
assert ops.half_mode() and ops.build_half(), "child must load the fp16 build"
dev = torch.device("cuda")

def hp(bs):
    return {"opt_case": {"optimizer": "gd", "lr": 1.0}, "batch_size": bs, "regularizer": "None",
            "weight_decay": 0.0, "initializer": "he_init", "decay_steps": 0, "decay_rate": 1.0}

def relerr(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))

def run(arch, sizes, image, ncls, scales=(128.0,)):
    torch.manual_seed(0)
    n = len(sizes)
    ref = PopulationEngine(arch, n, dev, backend="torch", compute_dtype=torch.float32, optimizer_impl="hip")
    r16 = PopulationEngine(arch, n, dev, backend="torch", compute_dtype=torch.bfloat16, optimizer_impl="hip")
    hips = [PopulationEngine(arch, n, dev, backend="hip", compute_dtype=torch.float16, loss_scale=s) for s in scales]
    for h in hips:
        assert h.backend.name == "hip" and h.backend.half and h.backend.loss_scale == h.loss_scale
    slots = []
    for i, bs in enumerate(sizes):
        s = ref.add_member(None, hp(bs), seed=10 + i)
        r16.add_member(None, hp(bs), seed=10 + i)
        for h in hips:
            assert h.add_member(None, hp(bs), seed=10 + i) == s
        slots.append(s)
    g = torch.Generator().manual_seed(1)
    for b in arch.prog.bns:
        ng, nb = 1.0 + 0.2 * torch.randn(n, b.c, generator=g), 0.1 * torch.randn(n, b.c, generator=g)
        for e in [ref, r16] + hips:
            e.state[:n, b.gamma_off:b.gamma_off + b.c] = ng.to(dev)
            e.state[:n, b.beta_off:b.beta_off + b.c] = nb.to(dev)
    batches = [(torch.randn(bs, image, image, 3, generator=g).to(dev), torch.randint(0, ncls, (bs,), generator=g).to(dev))
               for bs in sizes]
    hps = [hp(bs) for bs in sizes]
    for e in [ref, r16] + hips:
        e.train_step(slots, batches, hps, [0.0] * n)  # eager warm-up + graph capture
    before = ref.params.clone()
    l_ref = ref.train_step(slots, batches, hps, [1.0] * n)
    r16.train_step(slots, batches, hps, [1.0] * n)
    l_h = [h.train_step(slots, batches, hps, [1.0] * n) for h in hips]
    torch.cuda.synchronize()
    g_ref, g_16 = before - ref.params, before - r16.params
    segs = [("conv%d" % c.idx, c.off, c.off + c.numel) for c in arch.prog.convs]
    for bn in arch.prog.bns:
        segs += [("bn%d.gamma" % bn.idx, bn.gamma_off, bn.gamma_off + bn.c), ("bn%d.beta" % bn.idx, bn.beta_off, bn.beta_off + bn.c)]
    segs.append(("dense", arch.prog.dense_w_off, arch.prog.dense_b_off + arch.cfg.num_classes))
    worst = []
    for h, l in zip(hips, l_h):
        lrel = float(((l.float() - l_ref.float()).abs() / l_ref.float().abs()).max())
        assert lrel < 3e-2, ("loss", h.loss_scale, l.tolist(), l_ref.tolist())
        g_h = before - h.params
        assert torch.isfinite(g_h).all(), "non-finite fp16 update"
        bad, mx = [], 0.0
        for s in slots:
            for name, lo, hi in segs:
                r = relerr(g_h[s, lo:hi], g_ref[s, lo:hi])
                tol = max(2.5 * relerr(g_16[s, lo:hi], g_ref[s, lo:hi]), 0.06)
                mx = max(mx, r / tol)
                if r > tol:
                    bad.append("%s member %d rel %.4f tol %.4f" % (name, s, r, tol))
        assert not bad, (h.loss_scale, bad[:20])
        worst.append(round(mx, 3))
        print("ARCH %s loss_scale %g: loss rel %.2e, worst layer err / tol %.3f" % (arch.name, h.loss_scale, lrel, mx))
    if len(hips) > 1:  # the unscale matches the scale: two loss scales give the same update up to fp16 rounding
        # (measured 0.06 between 128 and 2^15 over the whole row; a missing / doubled unscale gives >= 1)
        d = relerr(before - hips[1].params, before - hips[0].params)
        print("update rel diff between loss scales:", d)
        assert d < 0.15, d
    return worst

run(ResNetArch(cifar_config(20, 2)), [12, 20], 32, 10, scales=(128.0, 32768.0))
run(ResNetArch(imagenet_config(50, 2, num_classes=1001, image_size=64)), [4, 6], 64, 1001)
print("FP16_OK")
"""


def test_fp16_hip_step_matches_fp32_oracle():
    env = dict(os.environ, DTF_HALF="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.pop("DTF_DETERMINISTIC", None)
    r = subprocess.run([sys.executable, "-u", "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=280)
    out = r.stdout + r.stderr
    print(out[-4000:])
    assert r.returncode == 0 and "FP16_OK" in r.stdout, out[-4000:]


def test_fp16_deterministic_build_replays_bitwise():
    """--dtype fp16 --deterministic: the deterministic half build (libdtf_kernels_f16_det.so: DTF_HALF with the
    deterministic build's fixed-order / fixed-point reductions) replays the fp16 ResNet v2 steps bitwise --
    CIFAR at pop 1 / 2 / 4 and the ImageNet-shape bottleneck net (tools/det_check.py, fp16 branch)."""
    env = dict(os.environ, DTF_HALF="1", DTF_DETERMINISTIC="1",
               PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "det_check.py")], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=280)
    out = r.stdout + r.stderr
    print(out[-4000:])
    assert r.returncode == 0 and "DET_OK" in r.stdout, out[-4000:]
    assert "library: " in out and "libdtf_kernels_f16_det.so" in out, out[-2000:]
