"""HIP ImageNet-shape ResNet-50 v2 step (ops/csrc/convg.hip, convg_aux.hip, gemm.hip) vs the fp32 oracle.

Small 64x64 input (stem 32 -> pool 16 -> stages 16/8/4/2) keeps the oracle cheap while exercising every
kernel variant: 7x7/2 stem on channel-padded input, 3x3/2 'SAME' max-pool, bottleneck convs with BN+ReLU
prologues / BN-stat epilogues, stride-2 transposed-gather data gradients, split-K weight gradients, GAP +
1001-class dense (padded GEMM) + softmax CE.  One gradient-descent step (lr = 1) turns the parameter delta
into the gradient, compared per tensor; members use ragged batch sizes.
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


@pytest.mark.parametrize("image,sizes,graph,version", [(64, (4, 6), "1", 2), (64, (4, 6), "0", 2),
                                                       (224, (16, 16), "1", 2), (64, (4, 6), "1", 1),
                                                       (64, (4, 6), "0", 1), (224, (16, 16), "1", 1)])
def test_hip_imagenet_step_matches_reference(monkeypatch, image, sizes, graph, version):
    """Step 1 (lr 0) is the eager warm-up that captures the graph; step 2 (lr 1) is the first graph REPLAY (graph
    "1") or a second eager run ("0") -- its parameter delta is compared.  224 x 224 at 2 x 16 runs the benchmark's
    tile / split-K choices.  Version 1: the post-activation bottleneck (reference resnet_model.py:215-264; stem
    BN+ReLU, projection BN on the shortcut, ReLU after the residual add, no final BN)."""
    monkeypatch.setenv("DTF_HIP_GRAPH", graph)
    torch.manual_seed(0)
    arch = ResNetArch(imagenet_config(50, version, num_classes=1001, image_size=image))
    dev = torch.device("cuda")
    sizes = list(sizes)
    ref = PopulationEngine(arch, 2, dev, backend="torch", compute_dtype=torch.float32, optimizer_impl="hip")
    r16 = PopulationEngine(arch, 2, dev, backend="torch", compute_dtype=torch.bfloat16, optimizer_impl="hip")
    hip = PopulationEngine(arch, 2, dev, backend="hip")
    assert hip.backend.__class__.__name__ == "HipImageNetBackend"
    slots = []
    for i, bs in enumerate(sizes):
        s1 = ref.add_member(None, _hp(bs), seed=3 + i)
        r16.add_member(None, _hp(bs), seed=3 + i)
        assert hip.add_member(None, _hp(bs), seed=3 + i) == s1
        slots.append(s1)
    g = torch.Generator().manual_seed(1)
    for b in arch.prog.bns:
        ng = 1.0 + 0.2 * torch.randn(2, b.c, generator=g)
        nb = 0.1 * torch.randn(2, b.c, generator=g)
        for st in (ref.state, hip.state, r16.state):
            st[:, b.gamma_off:b.gamma_off + b.c] = ng.to(dev)
            st[:, b.beta_off:b.beta_off + b.c] = nb.to(dev)
    batches = [(torch.randn(bs, image, image, 3, generator=g).to(dev),
                torch.randint(0, 1001, (bs,), generator=g).to(dev)) for bs in sizes]
    before = hip.params.clone()
    hps = [_hp(bs) for bs in sizes]
    for e in (ref, r16, hip):
        e.train_step(slots, batches, hps, [0.0, 0.0])
    torch.cuda.synchronize()
    assert torch.equal(hip.params, before)
    plan = next(iter(hip.backend._plans.values()))
    assert (plan.graph is not None) == (graph == "1")
    l_ref = ref.train_step(slots, batches, hps, [1.0, 1.0])
    l16 = r16.train_step(slots, batches, hps, [1.0, 1.0])
    l_hip = hip.train_step(slots, batches, hps, [1.0, 1.0])
    torch.cuda.synchronize()
    # loss tolerance: 3% (v1 at 64 x 64: 5%), or 2.5x how far a bf16 PyTorch forward of the same net lands from fp32.
    # The random-init loss of this net is chaotic in the bf16 rounding: the features after 16 blocks differ from
    # fp32 by ~50% (v1) / ~30% (v2) relative L2 for the HIP path and for torch bf16 alike, so the two land on
    # different sides of the fp32 loss by a few % (v1: HIP -2.2 / +2.9 %, torch bf16 +1.4 / -0.5 % on the same
    # members), while every HIP block adds LESS error than the torch bf16 block does from the same input
    # (tools/imagenet_v1_diag.py, profiles/r5_imagenet_v1_diag.txt; test_hip_imagenet_block_local_error below pins
    # that per block); at 224 x 224 the loss agrees to 0.3%
    floor = 5e-2 if (version == 1 and image == 64) else 3e-2
    rt = max(floor, 2.5 * float(((l16.float() - l_ref.float()).abs() / l_ref.float().abs()).max()))
    print("loss rel: hip %s, torch bf16 %s" % (((l_hip.float() - l_ref.float()) / l_ref.float()).tolist(),
                                               ((l16.float() - l_ref.float()) / l_ref.float()).tolist()))
    torch.testing.assert_close(l_hip.float(), l_ref.float(), rtol=rt, atol=3e-2)
    g_ref, g_hip, g16 = before - ref.params, before - hip.params, before - r16.params
    prog = arch.prog
    segs = [("conv%d" % c.idx, c.off, c.off + c.numel) for c in prog.convs]
    for bn in prog.bns:
        segs += [("bn%d.gamma" % bn.idx, bn.gamma_off, bn.gamma_off + bn.c),
                 ("bn%d.beta" % bn.idx, bn.beta_off, bn.beta_off + bn.c)]
    segs.append(("dense", prog.dense_w_off, prog.dense_b_off + arch.cfg.num_classes))
    bad = []
    for s in slots:
        for name, lo, hi in segs:
            a, b, c16 = g_hip[s, lo:hi], g_ref[s, lo:hi], g16[s, lo:hi]
            tol = max(2.5 * _relerr(c16, b), 0.06)
            err = _relerr(a, b)
            if err > tol:
                bad.append("%s member %d rel %.4f tol %.4f" % (name, s, err, tol))
    assert not bad, "\n".join(bad)
    # (atol 5e-3: a near-zero running mean moved 3.3e-3 by bf16 rounding in one of 106k elements)
    torch.testing.assert_close(hip.running, ref.running, rtol=3e-2, atol=5e-3)


@pytest.mark.parametrize("knobs", [{"CG_GFOLD_MAXF": 128}, {"CG_FOLD3_MAXC": 2048}, {"CG_FOLD": True},
                                   {"CG_FOLD1": False, "CG_COMPACT_PD": False}])
def test_hip_imagenet_step_plan_variants(monkeypatch, knobs):
    """The off-by-default plan switches of engine/hip_imagenet.py against the same fp32 oracle: the block-input
    gradient applied inside conv3's data gradient (convg MODE 3 + xout, with and without the residual operand),
    the BN3 fold into conv3, the full BN fold, and the plain path without the read-once BN1 fold and the compact
    projection gradient.  (Module constants are read when a plan is built, so patching them selects the path.)"""
    from distributedtf_amd.engine import hip_imagenet
    for k, v in knobs.items():
        monkeypatch.setattr(hip_imagenet, k, v)
    test_hip_imagenet_step_matches_reference(monkeypatch, 64, (4, 6), "1", 2)


@pytest.mark.parametrize("version", [1, 2])
def test_hip_imagenet_block_local_error(version):
    """The loss bound above has to absorb the chaotic growth of bf16 rounding through 16 blocks; this pins the
    HIP forward per block instead: each block's output (plan.xs after an lr = 0 step) against the fp32 PyTorch block
    applied to the HIP block's OWN input must be within 1.25x the error of the bf16 PyTorch block on the same input
    (measured 0.95-0.97x for every block of v1 and v2: profiles/r5_imagenet_v1_diag.txt), the stem + max-pool
    within 1.25x of torch bf16 from the image, and the loss within 1e-3 of the fp32 head on the HIP features."""
    import torch.nn.functional as F
    from distributedtf_amd.models import resnet as R
    torch.manual_seed(0)
    image, sizes = 64, [4, 6]
    arch = ResNetArch(imagenet_config(50, version, num_classes=1001, image_size=image))
    prog, cfg = arch.prog, arch.cfg
    dev = torch.device("cuda")
    hip = PopulationEngine(arch, 2, dev, backend="hip")
    slots = [hip.add_member(None, _hp(bs), seed=3 + i) for i, bs in enumerate(sizes)]
    g = torch.Generator().manual_seed(1)
    for b in prog.bns:
        hip.state[:, b.gamma_off:b.gamma_off + b.c] = (1.0 + 0.2 * torch.randn(2, b.c, generator=g)).to(dev)
        hip.state[:, b.beta_off:b.beta_off + b.c] = (0.1 * torch.randn(2, b.c, generator=g)).to(dev)
    batches = [(torch.randn(bs, image, image, 3, generator=g).to(dev),
                torch.randint(0, 1001, (bs,), generator=g).to(dev)) for bs in sizes]
    run0 = hip.running.clone()
    loss = hip.train_step(slots, batches, [_hp(bs) for bs in sizes], [0.0, 0.0])
    torch.cuda.synchronize()
    plan = next(iter(hip.backend._plans.values()))
    xs = [t.float() for t in plan.xs]
    bad, off = [], 0
    for i, s in enumerate(slots):
        n, p, run = sizes[i], hip.params[s].float(), run0[s].float().clone()
        x_in, y = batches[i]
        part = lambda t: t[off:off + n].permute(0, 3, 1, 2)  # noqa: E731

        def stem(dtype):
            x = R._conv(prog, p, x_in.permute(0, 3, 1, 2).to(dtype), prog.stem, dtype)
            if version == 1:
                x = F.relu(R._bn(prog, p, run, x, prog.stem_bn, True, False))
            return F.max_pool2d(F.pad(x, (0, 1, 0, 1), value=float("-inf")), 3, 2)  # TF 'SAME' at even sizes

        s32, s16 = stem(torch.float32), stem(torch.bfloat16)
        e_hip, e16 = _relerr(part(xs[0]), s32), _relerr(s16, s32)
        if e_hip > 1.25 * e16 + 1e-4:
            bad.append("stem member %d: %.3e vs torch bf16 %.3e" % (s, e_hip, e16))
        for bi, blk in enumerate(prog.blocks):
            hin = part(xs[bi])
            l32 = R.block_forward(prog, p, run, hin, blk, True, torch.float32, False)
            l16 = R.block_forward(prog, p, run, hin.bfloat16(), blk, True, torch.bfloat16, False)
            e_hip, e16 = _relerr(part(xs[bi + 1]), l32), _relerr(l16, l32)
            if e_hip > 1.25 * e16 + 1e-4:
                bad.append("block %d member %d: %.3e vs torch bf16 %.3e" % (bi, s, e_hip, e16))
        feat = part(xs[-1])
        if version == 2:
            feat = F.relu(R._bn(prog, p, run, feat, prog.final_bn, True, False))
        w = p[prog.dense_w_off:prog.dense_w_off + cfg.num_classes * cfg.final_size].view(cfg.num_classes, cfg.final_size)
        b = p[prog.dense_b_off:prog.dense_b_off + cfg.num_classes]
        lh = float(F.cross_entropy(feat.mean(dim=(2, 3)) @ w.t() + b, y.long()))
        assert abs(float(loss[i]) - lh) <= 1e-3 * abs(lh), (float(loss[i]), lh)
        off += n
    assert not bad, "\n".join(bad)
