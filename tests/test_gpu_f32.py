"""fp32 HIP step (engine/hip_f32.py, ops/csrc/f32conv.hip) vs the plain-PyTorch fp32 oracle: ``--dtype fp32``, the
reference's default dtype (resnet/official/utils/flags/_performance.py:30-33).

One gradient-descent step (lr = 2^20, after an lr = 0 warm-up that captures the graph) turns the parameter delta into
the gradient, compared PER LAYER against an fp64 evaluation of the same step (models/resnet.forward_reference in
float64): the HIP step must be within relative L2 1e-3 of it, or within 3x of how far the PyTorch fp32 oracle itself lands
from it, or within 3x of how far fp64 moves under a 1e-5 relative input perturbation, the size of the fp32 forward's own
accumulated deviation (pre-activations within rounding distance of zero flip their ReLU masks: on CPU, ResNet-14 at
batch 32 moves 2.8e-3 under a 1e-7 perturbation, so no fp32 implementation can be closer than that), plus the loss and the BN moving statistics vs the fp32 oracle.  Ragged
batch sizes, v2 and v1, graph and eager.
"""
import pytest
import torch

from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.resnet import ResNetArch, cifar_config

pytestmark = pytest.mark.gpu


def _hp(bs, opt="gd", lr=1.0):
    return {"opt_case": {"optimizer": opt, "lr": lr, "momentum": 0.9}, "batch_size": bs, "regularizer": "None",
            "weight_decay": 0.0, "initializer": "he_init", "decay_steps": 0, "decay_rate": 1.0}


def _relerr(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


@pytest.mark.parametrize("size,version,sizes,graph", [(14, 2, [8, 12, 6], "1"), (14, 1, [8, 12, 6], "1"),
                                                      (20, 2, [16, 9], "0"), (8, 1, [16], "0"),
                                                      (56, 2, [32, 32], "1")])
def test_f32_step_matches_fp32_oracle(size, version, sizes, graph, monkeypatch):
    monkeypatch.setenv("DTF_HIP_GRAPH", graph)
    torch.manual_seed(0)
    arch = ResNetArch(cifar_config(size, version=version))
    dev = torch.device("cuda")
    n = len(sizes)
    ref = PopulationEngine(arch, n, dev, backend="torch", compute_dtype=torch.float32, optimizer_impl="hip")
    hip = PopulationEngine(arch, n, dev, backend="hip", compute_dtype=torch.float32)
    assert hip.backend.__class__.__name__ == "HipResNetF32Backend"
    slots = []
    for i, bs in enumerate(sizes):
        s = ref.add_member(None, _hp(bs), seed=10 + i)
        assert hip.add_member(None, _hp(bs), seed=10 + i) == s
        slots.append(s)
    g = torch.Generator().manual_seed(1)
    for b in arch.prog.bns:  # BN gammas / betas away from identity
        ng = 1.0 + 0.2 * torch.randn(n, b.c, generator=g)
        nb = 0.1 * torch.randn(n, b.c, generator=g)
        for e in (ref, hip):
            e.state[:n, b.gamma_off:b.gamma_off + b.c] = ng.to(dev)
            e.state[:n, b.beta_off:b.beta_off + b.c] = nb.to(dev)
    batches = [(torch.randn(bs, 32, 32, 3, generator=g).to(dev), torch.randint(0, 10, (bs,), generator=g).to(dev))
               for bs in sizes]
    hps = [_hp(bs) for bs in sizes]
    for e in (ref, hip):
        e.train_step(slots, batches, hps, [0.0] * n)
    before = hip.params.clone()
    assert torch.equal(before, ref.params)
    # lr = 2^20: the update lr * g dominates the parameter, so (before - after) / lr recovers g to fp32 rounding
    # (with lr = 1 the subtraction's rounding, ulp(w) / |g|, swamps small fp32 gradients)
    LR = float(2 ** 20)
    l_ref = ref.train_step(slots, batches, hps, [LR] * n)
    l_hip = hip.train_step(slots, batches, hps, [LR] * n)
    torch.cuda.synchronize()
    plan = next(iter(hip.backend._plans.values()))
    assert (plan.graph is not None) == (graph == "1")
    torch.testing.assert_close(l_hip, l_ref, rtol=1e-4, atol=1e-4)
    g_ref, g_hip = (before - ref.params) / LR, (before - hip.params) / LR
    # fp64 gradient of the same step (same parameters, same batches, training-mode BN)
    from distributedtf_amd.models.resnet import forward_reference
    run0 = hip.running.clone()  # unused by the gradient (training BN uses batch statistics)

    def grad64(rel_noise=0.0, seed=0):
        out = torch.zeros_like(before, dtype=torch.float64)
        gn = torch.Generator(device=dev).manual_seed(seed)
        for i, s in enumerate(slots):
            p = before[s].double().clone().requires_grad_(True)
            x, y = batches[i]
            x = x.double() * (1.0 + rel_noise * torch.randn(x.shape, generator=gn, device=dev, dtype=torch.float64))
            logits = forward_reference(arch.prog, p, run0[s].double().clone(), x, training=True,
                                       dtype=torch.float64, update_running=False)
            loss = torch.nn.functional.cross_entropy(logits, y.long())
            out[s], = torch.autograd.grad(loss, p)
        return out

    g64 = grad64()
    # sensitivity of the exact gradient to fp32-sized perturbations: ReLU masks of pre-activations within rounding
    # distance of zero flip, so ANY fp32 implementation lands about this far from the fp64 gradient.  1e-5 relative
    # input noise: the fp32 forward's own deviation from fp64 grows to ~8e-6 relative at the last of ResNet-56's 27
    # blocks (tools/f32_diag.py, profiles/r4_f32_forward_deviation.txt)
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
    assert not bad, "\n".join(bad)
    print("worst per-layer relative error vs fp64: HIP fp32 %.2e, torch fp32 %.2e; fp64 sensitivity to 1e-5 input "
          "noise %.2e" % (worst, worst_ref, worst_sens))
    torch.testing.assert_close(hip.running, ref.running, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(hip.step_col(), ref.step_col())


def test_f32_trains_and_evaluates():
    """Momentum / Adam members learn a fixed batch over replayed fp32 steps; eval (moving statistics) runs the same
    forward kernels and agrees with the torch eval forward on the same rows."""
    arch = ResNetArch(cifar_config(20))
    dev = torch.device("cuda")
    hip = PopulationEngine(arch, 2, dev, backend="hip", compute_dtype=torch.float32)
    ref = PopulationEngine(arch, 2, dev, backend="torch", compute_dtype=torch.float32)
    hps = [_hp(32, "Momentum", 0.05), _hp(32, "Adam", 1e-3)]
    for i, hp in enumerate(hps):
        hip.add_member(None, hp, seed=i)
        ref.add_member(None, hp, seed=i)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(32, 32, 32, 3, generator=g).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    L = [hip.train_step([0, 1], [(x, y)] * 2, hps, [0.05, 1e-3]).cpu() for _ in range(15)]
    L = torch.stack(L)
    assert torch.isfinite(L).all() and (L[-1] < L[0]).all(), L
    ref.state.copy_(hip.state)
    ex = torch.randn(64, 32, 32, 3, generator=g).to(dev)
    ey = torch.randint(0, 10, (64,), generator=g).to(dev)
    a_hip = hip.evaluate_population([0, 1], ex, ey)
    a_ref = ref.evaluate_population([0, 1], ex, ey)
    for s in (0, 1):
        assert abs(a_hip[s] - a_ref[s]) <= 1.0 / 64 + 1e-9, (a_hip, a_ref)
    logits = hip.backend.infer(0, ex)
    with torch.no_grad():
        want = arch.forward(ref.params[0], ref.running[0].clone(), ex, training=False)
    torch.testing.assert_close(logits, want, rtol=1e-3, atol=1e-3)
