"""HIP MNIST step (ops/csrc/mnist.hip + gemm.hip) vs the plain-PyTorch fp32 oracle.

* grouped bf16 GEMM: every operand layout / output mode vs fp32 torch matmul of the same bf16 inputs;
* one population step with gradient descent (lr = 1): ``params_before - params_after`` is the gradient,
  compared PER TENSOR against torch autograd of ``MnistArch.forward`` fed the same dropout mask (the
  head kernel's counter hash, replicated on the host by ``dropout_keep_mask``).  Members use different
  batch sizes (ragged population packing).
"""
import pytest
import torch

from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.mnist import MnistArch

pytestmark = pytest.mark.gpu


def _relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("a_km,b_km,out", [(0, 0, 0), (0, 1, 1), (1, 1, 2), (1, 0, 0), (0, 0, 2)])
def test_grouped_gemm_modes(a_km, b_km, out):
    from distributedtf_amd.engine import hip_mnist as hm
    hm._register()
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    # two groups with ragged M (and K for K-major A)
    # (M, N, K): K % 32 wherever an operand is [rows][K]; M / N % 8 where K-major
    if a_km and b_km:
        probs = [(128, 192, 72), (64, 136, 40)]   # ragged K (wgrad: K = member batch)
    elif a_km:
        probs = [(128, 192, 96), (64, 136, 64)]
    else:
        probs = [(72, 192, 96), (136, 128, 64)]   # ragged M (fwd / dgrad: M = member batch)
    A_parts, B_parts, refs = [], [], []
    lda = max(p[2] for p in probs) if not a_km else max(p[0] for p in probs)
    ldb = max(p[2] for p in probs) if not b_km else max(p[1] for p in probs)
    lda, ldb = (lda + 7) // 8 * 8, (ldb + 7) // 8 * 8
    ldc = max(p[1] for p in probs)
    a_rows = sum(p[2] if a_km else p[0] for p in probs)
    b_rows = sum(p[2] if b_km else p[1] for p in probs)
    A = torch.zeros(a_rows, lda, dtype=torch.bfloat16)
    B = torch.zeros(b_rows, ldb, dtype=torch.bfloat16)
    c_rows = sum(p[0] for p in probs)
    C0 = torch.randn(c_rows, ldc, generator=g) if out == 2 else torch.zeros(c_rows, ldc)
    problems = []
    ao = bo = co = 0
    for (M, N, K) in probs:
        a = torch.randn(M, K, generator=g).bfloat16()
        b = torch.randn(K, N, generator=g).bfloat16()
        if a_km:
            A[ao // lda:ao // lda + K, :M] = a.t()
        else:
            A[ao // lda:ao // lda + M, :K] = a
        if b_km:
            B[bo // ldb:bo // ldb + K, :N] = b
        else:
            B[bo // ldb:bo // ldb + N, :K] = b.t()
        refs.append((co, M, N, a.float() @ b.float()))
        problems.append((ao, bo, co * ldc, M, N, K))
        ao += (K if a_km else M) * lda
        bo += (K if b_km else N) * ldb
        co += M
    Ad, Bd = A.to(dev), B.to(dev)
    Cd = C0.to(dev) if out != 1 else torch.zeros(c_rows, ldc, dtype=torch.bfloat16, device=dev)
    gg = hm.GroupedGemm(Ad, Bd, Cd, lda, ldb, ldc, problems, bool(a_km), bool(b_km), out, dev)
    from distributedtf_amd import ops
    gg.launch(ops.stream())
    torch.cuda.synchronize()
    C = Cd.float().cpu()
    for (r0, M, N, ref) in refs:
        exp = ref + (C0[r0:r0 + M, :N] if out == 2 else 0)
        tol = 2e-2 if out == 1 else 1e-3
        assert _relerr(C[r0:r0 + M, :N], exp) < tol


def _hp(bs):
    return {"opt_case": {"optimizer": "gd", "lr": 1.0}, "batch_size": bs, "initializer": "he_init"}


@pytest.mark.parametrize("graph", ["1", "0"])
def test_hip_mnist_step_matches_reference(graph, monkeypatch):
    monkeypatch.setenv("DTF_HIP_GRAPH", graph)
    from distributedtf_amd.engine.hip_mnist import dropout_keep_mask
    torch.manual_seed(0)
    arch = MnistArch()
    dev = torch.device("cuda")
    sizes = [24, 40]
    hip = PopulationEngine(arch, 2, dev, backend="hip")
    assert hip.backend.__class__.__name__ == "HipMnistBackend"
    slots = [hip.add_member(None, _hp(bs), seed=7 + i) for i, bs in enumerate(sizes)]
    g = torch.Generator().manual_seed(3)
    # non-zero biases so every bias path is exercised
    for name in ("conv1_b", "conv2_b", "dense1_b", "dense2_b"):
        off, shp = arch.offsets[name]
        hip.state[:, off:off + shp[0]] = (0.05 * torch.randn(2, shp[0], generator=g)).to(dev)
    hip.backend.on_params_changed(slots)
    batches = [((torch.rand(bs, 28, 28, 1, generator=g) * 255.0).to(dev), torch.randint(0, 10, (bs,), generator=g).to(dev))
               for bs in sizes]
    before = hip.params.clone()
    # step 1 (lr 0): the eager warm-up that also captures the step graph; step 2 (lr 1): with DTF_HIP_GRAPH=1 the
    # first graph REPLAY (device-side step advance, hyper table, dropout counter), else a second eager run
    hip.train_step(slots, batches, [_hp(bs) for bs in sizes], [0.0, 0.0])
    torch.cuda.synchronize()
    assert torch.equal(hip.params, before)
    plan = next(iter(hip.backend._plans.values()))
    assert (plan.graph is not None) == (graph == "1")
    losses = hip.train_step(slots, batches, [_hp(bs) for bs in sizes], [1.0, 1.0])
    torch.cuda.synchronize()
    seed, ctr = hip.backend.last_rng
    mask = torch.from_numpy(dropout_keep_mask(seed, ctr, sum(sizes), arch.dropout))
    assert 0.55 < mask.float().mean().item() < 0.65
    g_hip = before - hip.params
    first = 0
    for s, (x, y) in zip(slots, batches):
        n = x.shape[0]
        p = before[s].detach().clone().requires_grad_(True)
        logits = arch.forward(p, None, x, training=True, dtype=torch.float32, dropout_mask=mask[first:first + n])
        loss = torch.nn.functional.cross_entropy(logits, y)
        gref, = torch.autograd.grad(loss, p)
        # the same step through PyTorch in bf16: its distance from the fp32 oracle is the scale of the bf16 rounding
        # (max-pool argmax / ReLU decisions flipped by bf16 activations reroute whole gradient entries)
        p16 = before[s].detach().clone().requires_grad_(True)
        logits16 = arch.forward(p16, None, x, training=True, dtype=torch.bfloat16, dropout_mask=mask[first:first + n])
        g16, = torch.autograd.grad(torch.nn.functional.cross_entropy(logits16.float(), y), p16)
        loss = float(loss.detach())
        assert abs(float(losses[slots.index(s)]) - loss) < 3e-2 * max(1.0, abs(loss))
        for name, (off, shp) in arch.offsets.items():
            numel = 1
            for d in shp:
                numel *= d
            a, b = g_hip[s, off:off + numel], gref[off:off + numel]
            err = _relerr(a, b)
            tol = max(0.05, 2.5 * _relerr(g16[off:off + numel], b))  # as the ResNet / ImageNet tests
            assert err < tol, "%s member %d rel err %.4f (tol %.4f)" % (name, s, err, tol)
        first += n


def test_hip_mnist_repeat_learns():
    arch = MnistArch()
    dev = torch.device("cuda")
    eng = PopulationEngine(arch, 3, dev, backend="hip")
    opts = [("Momentum", 0.01), ("Adam", 1e-4), ("gd", 1e-3)]
    hps = []
    for i, (o, lr) in enumerate(opts):
        hp = {"opt_case": {"optimizer": o, "lr": lr, "momentum": 0.9}, "batch_size": 32, "initializer": "he_init"}
        eng.add_member(None, hp, seed=i)
        hps.append(hp)
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(32, 28, 28, 1, generator=g) * 255.0).to(dev)
    y = torch.randint(0, 10, (32,), generator=g).to(dev)
    L = []
    for _ in range(15):
        L.append(eng.train_step([0, 1, 2], [(x, y)] * 3, hps, [h["opt_case"]["lr"] for h in hps]).cpu())
    L = torch.stack(L)
    assert torch.isfinite(L).all()
    assert (L[-3:].mean(0) < L[:3].mean(0)).all(), L


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_mnist_train_probabilities(dtype):
    """The "probabilities" hook's source (reference mnist_model.py:149-151): with keep_probs set before the first
    step, the HIP training plan also writes the head's logits, and train_probabilities returns each member's softmax
    of its last batch -- rows sum to 1 and their argmax agrees with the head kernel's own correct count."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    sizes = [40, 72]
    e = PopulationEngine(MnistArch(), len(sizes), dev, backend="hip", compute_dtype=dtype)
    e.backend.keep_probs = True
    hps = []
    for i, bs in enumerate(sizes):
        hp = {"opt_case": {"optimizer": "Adam", "lr": 1e-3}, "batch_size": bs, "initializer": "he_init"}
        e.add_member(None, hp, seed=5 + i)
        hps.append(hp)
    g = torch.Generator().manual_seed(1)
    batches = [((torch.rand(bs, 28, 28, 1, generator=g) * 255).to(dev), torch.randint(0, 10, (bs,), generator=g).to(dev))
               for bs in sizes]
    for _ in range(2):
        e.train_step([0, 1], batches, hps, [1e-3, 1e-3])
    torch.cuda.synchronize()
    probs = e.backend.train_probabilities([0, 1])
    corr = e.backend.train_correct([0, 1]).cpu().tolist()
    for s, (p, (x, y)) in enumerate(zip(probs, batches)):
        assert p is not None and tuple(p.shape) == (sizes[s], 10)
        assert torch.isfinite(p).all()
        torch.testing.assert_close(p.sum(dim=1), torch.ones(sizes[s], device=dev), atol=1e-5, rtol=0)
        hits = int((p.argmax(dim=1) == y).sum())
        assert hits == int(round(corr[s])), (s, hits, corr[s])
