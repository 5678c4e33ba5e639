"""Diagnostic: two members with identical state rows, hparams and batch must get (near-)identical gradients.
One GD step (lr = 1): params delta = gradient; per-layer relative differences twin vs twin and vs a solo run."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.resnet import ResNetArch, cifar_config


def grads(size, slots, bs, cap=4, seed_batch=0):
    arch = ResNetArch(cifar_config(size))
    dev = torch.device("cuda")
    e = PopulationEngine(arch, cap, dev, backend="hip")
    hp = {"opt_case": {"optimizer": "gd", "lr": 1.0}, "batch_size": bs, "regularizer": "None",
          "weight_decay": 0.0, "initializer": "he_init", "decay_steps": 0, "decay_rate": 1.0}
    for i in range(cap):
        e.add_member(None, dict(hp), seed=5)
    e.state[:] = e.state[0:1].clone()
    g = torch.Generator().manual_seed(seed_batch)
    x = torch.randn(bs, 32, 32, 3, generator=g).to(dev)
    y = torch.randint(0, 10, (bs,), generator=g).to(dev)
    e.train_step(slots, [(x, y)] * len(slots), [hp] * len(slots), [0.0] * len(slots))  # warm-up / capture
    before = e.params.clone()
    e.train_step(slots, [(x, y)] * len(slots), [hp] * len(slots), [1.0] * len(slots))
    torch.cuda.synchronize()
    return arch, (before - e.params).double()


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


def report(tag, size, slots, bs):
    arch, d = grads(size, slots, bs)
    _, solo = grads(size, [0], bs)
    a, b = d[slots[0]], d[slots[1]]
    rows = []
    for c in arch.prog.convs:
        s = slice(c.off, c.off + c.numel)
        rows.append((rel(a[s], b[s]), rel(a[s], solo[0][s]), c.idx))
    for bn in arch.prog.bns:
        s = slice(bn.gamma_off, bn.gamma_off + bn.c)
        rows.append((rel(a[s], b[s]), rel(a[s], solo[0][s]), 1000 + bn.idx))
    rows.sort(reverse=True)
    print("%s size %d slots %s bs %d: worst twin diffs %s" % (tag, size, slots, bs,
          " ".join("[%d t%.1e s%.1e]" % (i, t, s_) for t, s_, i in rows[:6])), flush=True)


tag = os.environ.get("TAG", "")
for args in [(20, [0, 1], 16), (20, [0, 1], 128), (56, [0, 1], 128)]:
    report(tag, *args)
