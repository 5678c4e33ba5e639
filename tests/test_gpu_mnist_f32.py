"""fp32 HIP MNIST step (engine/hip_mnist_f32.py: f32conv.hip MFMA convs + mnist.hip pool / head) vs the fp32 oracle.

One population step with gradient descent (lr = 1) of two members with ragged batch sizes: ``params_before -
params_after`` is the gradient, compared PER TENSOR against torch autograd of ``MnistArch.forward`` in fp32 fed the
head kernel's dropout mask (``dropout_keep_mask``) -- within 1e-3 relative L2 (fp32 numerics,
not the bf16 tolerance).  Also: eval logits vs the oracle, a few steps of learning, and the deterministic build's
bitwise replay (when libdtf_kernels_det.so is loaded, tools/det_check.py runs the full-run version).
"""
import pytest
import torch

from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.mnist import MnistArch

pytestmark = pytest.mark.gpu


def _relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _hp(bs):
    return {"opt_case": {"optimizer": "gd", "lr": 1.0}, "batch_size": bs, "initializer": "he_init"}


def _engine(n):
    eng = PopulationEngine(MnistArch(), n, torch.device("cuda"), backend="hip", compute_dtype=torch.float32)
    assert eng.backend.__class__.__name__ == "HipMnistF32Backend"
    return eng


@pytest.mark.parametrize("graph", ["1", "0"])
def test_hip_mnist_f32_step_matches_fp32_oracle(graph, monkeypatch):
    monkeypatch.setenv("DTF_HIP_GRAPH", graph)
    from distributedtf_amd.engine.hip_mnist import dropout_keep_mask
    arch = MnistArch()
    dev = torch.device("cuda")
    sizes = [24, 40]
    hip = _engine(2)
    slots = [hip.add_member(None, _hp(bs), seed=7 + i) for i, bs in enumerate(sizes)]
    g = torch.Generator().manual_seed(3)
    for name in ("conv1_b", "conv2_b", "dense1_b", "dense2_b"):  # non-zero biases: every bias path exercised
        off, shp = arch.offsets[name]
        hip.state[:, off:off + shp[0]] = (0.05 * torch.randn(2, shp[0], generator=g)).to(dev)
    batches = [((torch.rand(bs, 28, 28, 1, generator=g) * 255.0).to(dev),
                torch.randint(0, 10, (bs,), generator=g).to(dev)) for bs in sizes]
    before = hip.params.clone()
    hip.train_step(slots, batches, [_hp(bs) for bs in sizes], [0.0, 0.0])  # warm-up (+ graph capture)
    torch.cuda.synchronize()
    assert torch.equal(hip.params, before)
    plan = next(iter(hip.backend._plans.values()))
    assert (plan.graph is not None) == (graph == "1")
    losses = hip.train_step(slots, batches, [_hp(bs) for bs in sizes], [1.0, 1.0])
    torch.cuda.synchronize()
    seed, ctr = hip.backend.last_rng
    mask = torch.from_numpy(dropout_keep_mask(seed, ctr, sum(sizes), arch.dropout))
    g_hip = before - hip.params
    first = 0
    for s, (x, y) in zip(slots, batches):
        n = x.shape[0]
        p = before[s].detach().clone().requires_grad_(True)
        logits = arch.forward(p, None, x, training=True, dtype=torch.float32, dropout_mask=mask[first:first + n])
        loss = torch.nn.functional.cross_entropy(logits, y)
        gref, = torch.autograd.grad(loss, p)
        assert abs(float(losses[slots.index(s)]) - float(loss)) < 1e-3 * max(1.0, abs(float(loss)))
        for name, (off, shp) in arch.offsets.items():
            numel = 1
            for d in shp:
                numel *= d
            err = _relerr(g_hip[s, off:off + numel], gref[off:off + numel])
            print("member %d %s rel err %.2e" % (s, name, err))
            assert err < 1e-3, "%s member %d rel err %.2e" % (name, s, err)
        first += n


def test_hip_mnist_f32_infer_and_eval():
    arch = MnistArch()
    eng = _engine(2)
    for i in range(2):
        eng.add_member(None, _hp(16), seed=i)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(50, 28, 28, 1, generator=g) * 255.0).cuda()
    y = torch.randint(0, 10, (50,), generator=g).cuda()
    for s in (0, 1):
        lg = eng.backend.infer(s, x)
        ref = arch.forward(eng.params[s], None, x, training=False, dtype=torch.float32)
        assert _relerr(lg, ref) < 1e-4, _relerr(lg, ref)
    acc = eng.backend.evaluate_population([0, 1], x, y, chunk=20)
    for s in (0, 1):
        ref = arch.forward(eng.params[s], None, x, training=False, dtype=torch.float32).argmax(1)
        assert abs(acc[s] - float((ref == y).float().mean())) < 1e-6


def test_hip_mnist_f32_learns():
    eng = _engine(3)
    opts = [("Momentum", 0.01), ("Adam", 1e-4), ("gd", 1e-3)]
    hps = []
    for i, (o, lr) in enumerate(opts):
        hp = {"opt_case": {"optimizer": o, "lr": lr, "momentum": 0.9}, "batch_size": 32, "initializer": "he_init"}
        eng.add_member(None, hp, seed=i)
        hps.append(hp)
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(32, 28, 28, 1, generator=g) * 255.0).cuda()
    y = torch.randint(0, 10, (32,), generator=g).cuda()
    L = torch.stack([eng.train_step([0, 1, 2], [(x, y)] * 3, hps, [h["opt_case"]["lr"] for h in hps]).cpu()
                     for _ in range(15)])
    assert torch.isfinite(L).all()
    assert (L[-3:].mean(0) < L[:3].mean(0)).all(), L
