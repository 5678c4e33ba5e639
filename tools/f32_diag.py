"""Diagnostic: per-block forward deviation of the fp32 HIP step (engine/hip_f32.py) from an fp64 forward.

    python tools/f32_diag.py [resnet_size] [batch]

Runs one lr = 0 step of a 2-member HIP fp32 engine, then replays the v2 forward in fp64 block by block on the same
parameters and batches and prints, per block, the relative L2 deviation of the HIP block output (plan.xs[i + 1]) and
of the BN batch statistics (mean / inv std the HIP bn_final derived) from fp64.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.nn.functional as F
    from distributedtf_amd.engine.population import PopulationEngine
    from distributedtf_amd.models.resnet import ResNetArch, cifar_config, _conv
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 56
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    dev = torch.device("cuda")
    arch = ResNetArch(cifar_config(size, version=2))
    prog = arch.prog
    hip = PopulationEngine(arch, 2, dev, backend="hip", compute_dtype=torch.float32)
    hp = {"opt_case": {"optimizer": "gd", "lr": 0.0}, "batch_size": bs, "regularizer": "None", "weight_decay": 0.0,
          "initializer": "he_init", "decay_steps": 0, "decay_rate": 1.0}
    for i in range(2):
        hip.add_member(None, hp, seed=10 + i)
    g = torch.Generator().manual_seed(1)
    for b in prog.bns:
        hip.state[:2, b.gamma_off:b.gamma_off + b.c] = (1.0 + 0.2 * torch.randn(2, b.c, generator=g)).to(dev)
        hip.state[:2, b.beta_off:b.beta_off + b.c] = (0.1 * torch.randn(2, b.c, generator=g)).to(dev)
    batches = [(torch.randn(bs, 32, 32, 3, generator=g).to(dev), torch.randint(0, 10, (bs,), generator=g).to(dev))
               for _ in range(2)]
    hip.train_step([0, 1], batches, [hp, hp], [0.0, 0.0])
    torch.cuda.synchronize()
    plan = next(iter(hip.backend._plans.values()))
    be = hip.backend
    for s in range(2):
        p = hip.params[s].double()
        x = batches[s][0].permute(0, 3, 1, 2).double()
        x = _conv(prog, p, x, prog.stem, torch.float64)
        rows = []
        for i, blk in enumerate(prog.blocks):
            b1 = blk.bns[0]
            mean = x.mean(dim=(0, 2, 3))
            var = x.var(dim=(0, 2, 3), unbiased=False)
            co = be.coef[0, b1, s].double()
            c = prog.bns[b1].c
            dm = float((co[2, :c] - mean).norm() / (mean.norm() + 1e-30))
            dinv = float((co[3, :c] - torch.rsqrt(var + 1e-5)).norm() / torch.rsqrt(var + 1e-5).norm())
            bnp = prog.bns[b1]
            gm, bt = p[bnp.gamma_off:bnp.gamma_off + c], p[bnp.beta_off:bnp.beta_off + c]
            pre = F.relu((x - mean[None, :, None, None]) * (torch.rsqrt(var + 1e-5) * gm)[None, :, None, None]
                         + bt[None, :, None, None])
            sc = x if blk.proj is None else _conv(prog, p, pre, blk.proj, torch.float64)
            h = _conv(prog, p, pre, blk.convs[0], torch.float64)
            b2 = blk.bns[1]
            m2, v2 = h.mean(dim=(0, 2, 3)), h.var(dim=(0, 2, 3), unbiased=False)
            bn2 = prog.bns[b2]
            h = F.relu((h - m2[None, :, None, None]) * (torch.rsqrt(v2 + 1e-5) * p[bn2.gamma_off:bn2.gamma_off + bn2.c])
                       [None, :, None, None] + p[bn2.beta_off:bn2.beta_off + bn2.c][None, :, None, None])
            x = _conv(prog, p, h, blk.convs[1], torch.float64) + sc
            got = plan.xs[i + 1][plan.first[s]:plan.first[s] + bs].permute(0, 3, 1, 2).double()
            rel = float((got - x).norm() / x.norm())
            near0 = float(((pre > 0) != (pre > 0)).float().mean())
            rows.append("block %2d: out rel %.2e | BN1 mean rel %.2e inv rel %.2e | |mean|/std %.2f" % (
                i, rel, dm, dinv, float((mean.abs() / var.sqrt()).max())))
        print("member %d" % s)
        print("\n".join(rows))


if __name__ == "__main__":
    main()
