"""fp32 HIP ImageNet-shape ResNet-50 step (engine/hip_imagenet_f32.py: f32conv.hip MFMA convs, f32net.hip pool /
GAP / softmax) vs the PyTorch fp32 oracle.

The bf16 test (test_gpu_imagenet_step.py) bounds the HIP step by the bf16 rounding band; this one is fp32 against
fp32: one gradient-descent step (lr = 2^20 after an lr = 0 warm-up, so the parameter delta is the gradient to fp32
rounding) of two members with ragged batches at 64 x 64 (stem 32 -> pool 16 -> stages 16/8/4/2), v1 and v2, graph
and eager.  Every conv / BN / dense gradient tensor is compared with an fp64 evaluation of the same step
(models/resnet.forward_reference in float64, as tests/test_gpu_f32.py): within relative L2 1e-3, or 3x how far the
PyTorch fp32 oracle lands from it, or 3x the fp64 gradient's own movement under 1e-5 input noise; the loss within
1e-4 of the fp32 oracle, the running statistics within 1e-4.
"""
import pytest
import torch

from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.resnet import ResNetArch, imagenet_config

pytestmark = pytest.mark.gpu


def _hp(bs):
    return {"opt_case": {"optimizer": "gd", "lr": 1.0}, "batch_size": bs, "regularizer": "None",
            "weight_decay": 0.0, "initializer": "he_init"}


def _relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("version,graph", [(2, "1"), (2, "0"), (1, "1")])
def test_hip_imagenet_f32_step_matches_fp32_oracle(monkeypatch, version, graph):
    monkeypatch.setenv("DTF_HIP_GRAPH", graph)
    torch.manual_seed(0)
    image = 64
    arch = ResNetArch(imagenet_config(50, version, num_classes=1001, image_size=image))
    dev = torch.device("cuda")
    sizes = [4, 6]
    ref = PopulationEngine(arch, 2, dev, backend="torch", compute_dtype=torch.float32, optimizer_impl="hip")
    hip = PopulationEngine(arch, 2, dev, backend="hip", compute_dtype=torch.float32)
    assert hip.backend.__class__.__name__ == "HipImageNetF32Backend"
    slots = []
    for i, bs in enumerate(sizes):
        s1 = ref.add_member(None, _hp(bs), seed=3 + i)
        assert hip.add_member(None, _hp(bs), seed=3 + i) == s1
        slots.append(s1)
    g = torch.Generator().manual_seed(1)
    for b in arch.prog.bns:
        ng = 1.0 + 0.2 * torch.randn(2, b.c, generator=g)
        nb = 0.1 * torch.randn(2, b.c, generator=g)
        for st in (ref.state, hip.state):
            st[:, b.gamma_off:b.gamma_off + b.c] = ng.to(dev)
            st[:, b.beta_off:b.beta_off + b.c] = nb.to(dev)
    batches = [(torch.randn(bs, image, image, 3, generator=g).to(dev),
                torch.randint(0, 1001, (bs,), generator=g).to(dev)) for bs in sizes]
    hps = [_hp(bs) for bs in sizes]
    for e in (ref, hip):
        e.train_step(slots, batches, hps, [0.0, 0.0])
    torch.cuda.synchronize()
    before = hip.params.clone()
    assert torch.equal(before, ref.params)
    plan = next(iter(hip.backend._plans.values()))
    assert (plan.graph is not None) == (graph == "1")
    # lr = 2^20: (before - after) / lr recovers the gradient to fp32 rounding (lr = 1 leaves ulp(w) / |g| ~ 1e-2)
    LR = float(2 ** 20)
    l_ref = ref.train_step(slots, batches, hps, [LR, LR])
    l_hip = hip.train_step(slots, batches, hps, [LR, LR])
    torch.cuda.synchronize()
    print("loss hip %s ref %s" % (l_hip.tolist(), l_ref.tolist()))
    torch.testing.assert_close(l_hip.float(), l_ref.float(), rtol=1e-4, atol=1e-4)
    g_ref, g_hip = (before - ref.params) / LR, (before - hip.params) / LR
    from distributedtf_amd.models.resnet import forward_reference
    run0 = hip.running.clone()

    def grad64(rel_noise=0.0, seed=0):
        out = torch.zeros_like(before, dtype=torch.float64)
        gn = torch.Generator(device=dev).manual_seed(seed)
        for i, s in enumerate(slots):
            p = before[s].double().clone().requires_grad_(True)
            x, y = batches[i]
            x = x.double() * (1.0 + rel_noise * torch.randn(x.shape, generator=gn, device=dev, dtype=torch.float64))
            logits = forward_reference(arch.prog, p, run0[s].double().clone(), x, training=True,
                                       dtype=torch.float64, update_running=False)
            out[s], = torch.autograd.grad(torch.nn.functional.cross_entropy(logits, y.long()), p)
        return out

    # the fp64 gradient, and how far it moves under fp32-sized (1e-5) input perturbations: no fp32 implementation
    # can be closer than that (ReLU masks of pre-activations within rounding distance of zero flip)
    g64 = grad64()
    g_pert = [grad64(1e-5, seed) for seed in (1, 2)]
    prog = arch.prog
    segs = [("conv%d" % c.idx, c.off, c.off + c.numel) for c in prog.convs]
    for bn in prog.bns:
        segs += [("bn%d.gamma" % bn.idx, bn.gamma_off, bn.gamma_off + bn.c),
                 ("bn%d.beta" % bn.idx, bn.beta_off, bn.beta_off + bn.c)]
    segs.append(("dense", prog.dense_w_off, prog.dense_b_off + arch.cfg.num_classes))
    bad, worst, worst_ref, worst_sens = [], 0.0, 0.0, 0.0
    for s in slots:
        for name, lo, hi in segs:
            err = _relerr(g_hip[s, lo:hi], g64[s, lo:hi])
            err32 = _relerr(g_ref[s, lo:hi], g64[s, lo:hi])
            sens = max(_relerr(gp[s, lo:hi], g64[s, lo:hi]) for gp in g_pert)
            worst, worst_ref, worst_sens = max(worst, err), max(worst_ref, err32), max(worst_sens, sens)
            if err > max(1e-3, 3.0 * err32, 3.0 * sens):
                bad.append("%s member %d rel %.2e (torch fp32 %.2e, fp64 sensitivity %.2e)" % (name, s, err, err32,
                                                                                                  sens))
    print("worst per-tensor relative error vs fp64: HIP fp32 %.2e, torch fp32 %.2e; fp64 sensitivity %.2e"
          % (worst, worst_ref, worst_sens))
    assert not bad, "\n".join(bad)
    torch.testing.assert_close(hip.running, ref.running, rtol=1e-4, atol=1e-5)


def test_hip_imagenet_f32_eval_matches_oracle():
    arch = ResNetArch(imagenet_config(50, 2, num_classes=1001, image_size=64))
    dev = torch.device("cuda")
    hip = PopulationEngine(arch, 2, dev, backend="hip", compute_dtype=torch.float32)
    for i in range(2):
        hip.add_member(None, _hp(4), seed=i)
    g = torch.Generator().manual_seed(2)
    for b in arch.prog.bns:  # moving statistics away from (0, 1): mean 0.1 N(0, 1), variance 1 + 0.2 |N(0, 1)|
        hip.running[:, b.run_off:b.run_off + b.c] = (0.1 * torch.randn(2, b.c, generator=g)).to(dev)
        hip.running[:, b.run_off + b.c:b.run_off + 2 * b.c] = (1.0 + 0.2 * torch.randn(2, b.c, generator=g).abs()).to(dev)
    x = torch.randn(6, 64, 64, 3, generator=g).to(dev)
    y = torch.randint(0, 1001, (6,), generator=g).to(dev)
    for s in (0, 1):
        lg = hip.backend.infer(s, x)
        ref = arch.forward(hip.params[s], hip.running[s], x, training=False, dtype=torch.float32)
        assert _relerr(lg, ref) < 1e-3, _relerr(lg, ref)
    acc = hip.backend.evaluate_population([0, 1], x, y, chunk=4)
    for s in (0, 1):
        ref = arch.forward(hip.params[s], hip.running[s], x, training=False, dtype=torch.float32).argmax(1)
        assert abs(acc[s] - float((ref == y).float().mean())) < 1e-6
