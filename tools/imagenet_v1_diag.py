"""Where does the bf16 HIP ImageNet forward drift from fp32?  Per-stage diagnosis of the loss deviation that
tests/test_gpu_imagenet_step.py bounds (v1 at 64 x 64: HIP 2-4 % vs torch bf16 <= 2 %).

    python tools/imagenet_v1_diag.py [--version 1] [--image 64]        (GPU)

Same setup as the test (two members, ragged batches 4 / 6, randomised BN gammas / betas).  After one lr = 0 step the
HIP plan's block outputs (plan.xs) are compared per member with
  local : the fp32 PyTorch block (models/resnet.block_forward) applied to the HIP block's own input -- the error
          this block adds;
  chain : the fp32 PyTorch forward from the image -- the accumulated error;
and the same two numbers for a bf16 PyTorch forward (the yardstick: what bf16 storage alone costs).  Last rows: the
loss of the fp32 head (GAP + dense + softmax CE) on the HIP features against the HIP loss, and the chained losses.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--version", type=int, default=1)
    ap.add_argument("--image", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    import torch
    import torch.nn.functional as F
    from distributedtf_amd.engine.population import PopulationEngine
    from distributedtf_amd.models import resnet as R
    from distributedtf_amd.models.resnet import ResNetArch, imagenet_config

    torch.manual_seed(args.seed)
    dev = torch.device("cuda")
    image = args.image
    arch = ResNetArch(imagenet_config(50, args.version, num_classes=1001, image_size=image))
    prog, cfg = arch.prog, arch.cfg
    hip = PopulationEngine(arch, 2, dev, backend="hip", compute_dtype=torch.bfloat16)
    sizes = [4, 6]
    hp = lambda bs: {"opt_case": {"optimizer": "gd", "lr": 1.0}, "batch_size": bs, "regularizer": "None",  # noqa
                     "weight_decay": 0.0, "initializer": "he_init"}
    slots = [hip.add_member(None, hp(bs), seed=3 + i) for i, bs in enumerate(sizes)]
    g = torch.Generator().manual_seed(1)
    for b in prog.bns:
        ng = 1.0 + 0.2 * torch.randn(2, b.c, generator=g)
        nb = 0.1 * torch.randn(2, b.c, generator=g)
        hip.state[:, b.gamma_off:b.gamma_off + b.c] = ng.to(dev)
        hip.state[:, b.beta_off:b.beta_off + b.c] = nb.to(dev)
    batches = [(torch.randn(bs, image, image, 3, generator=g).to(dev),
                torch.randint(0, 1001, (bs,), generator=g).to(dev)) for bs in sizes]
    run0 = hip.running.clone()
    loss_hip = hip.train_step(slots, batches, [hp(bs) for bs in sizes], [0.0, 0.0])
    torch.cuda.synchronize()
    plan = next(iter(hip.backend._plans.values()))
    xs = [t.float() for t in plan.xs]  # NHWC, members' images packed in slot order
    print("v%d %dx%d, HIP loss %s" % (args.version, image, image, [round(float(v), 5) for v in loss_hip]))
    print("%-10s %5s | %-9s %-9s | %-9s %-9s" % ("stage", "mbr", "HIP loc", "bf16 loc", "HIP chain", "bf16 chain"))
    off = 0
    for i, s in enumerate(slots):
        n = sizes[i]
        p = hip.params[s].float()
        run = run0[s].float().clone()
        x_in, y = batches[i]
        nchw = lambda t: t[off:off + n].permute(0, 3, 1, 2)  # noqa: E731

        def stem(x, dtype):
            x = x.permute(0, 3, 1, 2).to(dtype)
            x = R._conv(prog, p, x, prog.stem, dtype)
            if cfg.version == 1:
                x = F.relu(R._bn(prog, p, run, x, prog.stem_bn, True, False))
            k, st = cfg.first_pool_size, cfg.first_pool_stride
            h = x.shape[-1]
            pad = max(((h + st - 1) // st - 1) * st + k - h, 0)
            x = F.pad(x, (pad // 2, pad - pad // 2, pad // 2, pad - pad // 2), value=float("-inf"))
            return F.max_pool2d(x, k, st)

        c32 = stem(x_in, torch.float32)
        c16 = stem(x_in, torch.bfloat16)
        h0 = nchw(xs[0])
        print("%-10s %5d | %-9s %-9s | %9.2e %9.2e" % ("stem+pool", s, "", "", rel(h0, c32), rel(c16, c32)))
        for bi, blk in enumerate(prog.blocks):
            hin = nchw(xs[bi])
            hout = nchw(xs[bi + 1])
            l32 = R.block_forward(prog, p, run, hin, blk, True, torch.float32, False)
            l16 = R.block_forward(prog, p, run, hin.bfloat16(), blk, True, torch.bfloat16, False)
            c32 = R.block_forward(prog, p, run, c32, blk, True, torch.float32, False)
            c16 = R.block_forward(prog, p, run, c16, blk, True, torch.bfloat16, False)
            print("%-10s %5d | %9.2e %9.2e | %9.2e %9.2e" % ("block %d" % bi, s, rel(hout, l32), rel(l16, l32),
                                                             rel(hout, c32), rel(c16, c32)))

        def head(x):
            if cfg.version == 2:
                x = F.relu(R._bn(prog, p, run, x, prog.final_bn, True, False))
            feat = x.float().mean(dim=(2, 3))
            w = p[prog.dense_w_off:prog.dense_w_off + cfg.num_classes * cfg.final_size].view(cfg.num_classes,
                                                                                               cfg.final_size)
            b = p[prog.dense_b_off:prog.dense_b_off + cfg.num_classes]
            return F.cross_entropy(feat @ w.t() + b, y.long())

        lh = float(head(nchw(xs[-1])))
        l32, l16 = float(head(c32)), float(head(c16))
        print("loss mbr %d: HIP %.5f | fp32 head on HIP features %.5f | fp32 chain %.5f | bf16 chain %.5f  "
              "(HIP %+.2f %%, bf16 torch %+.2f %%)" % (s, float(loss_hip[i]), lh, l32, l16,
                                                       100 * (float(loss_hip[i]) - l32) / l32, 100 * (l16 - l32) / l32))
        off += n


if __name__ == "__main__":
    main()
