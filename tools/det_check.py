"""Deterministic HIP build check (run with DTF_DETERMINISTIC=1): two identically initialised engines train the same
steps on the same batches (graph replay, ragged populations) and must hold bitwise-identical state rows -- the
CIFAR ResNet v2, ResNet v1, ImageNet ResNet-50 v2 / v1 (fixed-point accumulation), MNIST and the fp32 CIFAR
ResNet v2 / v1 (fixed-point accumulation) families.  With DTF_HALF=1 as well: the deterministic half build
(libdtf_kernels_f16_det.so) on the fp16 ResNet v2 families (CIFAR, ImageNet shape; static loss scale 128).  Prints
DET_OK."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedtf_amd import ops  # noqa: E402
from distributedtf_amd.engine.population import PopulationEngine  # noqa: E402
from distributedtf_amd.models.resnet import ResNetArch, cifar_config, imagenet_config  # noqa: E402

assert ops.deterministic_mode(), "run with DTF_DETERMINISTIC=1"
_L = ops.lib()
print("library: %s" % getattr(getattr(_L, "_lib", _L), "_name", _L), flush=True)


def run(size, sizes, steps, opt="Momentum", version=2, image=32, dtype=torch.bfloat16, loss_scale=1.0):
    if image == 32:
        arch = ResNetArch(cifar_config(size, version=version))
    else:
        arch = ResNetArch(imagenet_config(size, version, num_classes=1001, image_size=image))
    dev = torch.device("cuda")
    out = []
    for rep in range(2):
        e = PopulationEngine(arch, len(sizes), dev, backend="hip", compute_dtype=dtype, loss_scale=loss_scale)
        hps = []
        for i, bs in enumerate(sizes):
            hp = {"opt_case": {"optimizer": opt, "lr": 0.05, "momentum": 0.9}, "batch_size": bs,
                  "regularizer": "l2_regularizer", "weight_decay": 1e-4, "initializer": "he_init"}
            e.add_member(None, hp, seed=7 + i)
            hps.append(hp)
        g = torch.Generator().manual_seed(3)
        ncls = arch.cfg.num_classes
        batches = [(torch.randn(bs, image, image, 3, generator=g).to(dev),
                    torch.randint(0, ncls, (bs,), generator=g).to(dev)) for bs in sizes]
        slots = list(range(len(sizes)))
        for _ in range(steps):
            losses = e.train_step(slots, batches, hps, [0.05] * len(sizes))
        torch.cuda.synchronize()
        out.append((e.state.clone(), losses.cpu()))
    st, ls = torch.equal(out[0][0], out[1][0]), torch.equal(out[0][1], out[1][1])
    same = st and ls
    print("image %d v%d size %d %s sizes %s steps %d: bitwise identical %s (state %s, losses %s), losses %s"
          % (image, version, size, str(dtype).split(".")[-1], sizes, steps, same, st, ls, out[0][1].tolist()),
          flush=True)
    return same


def run_mnist(sizes, steps, dtype=torch.bfloat16):
    """The MNIST HIP step (deterministic work splits: one accumulation workgroup per member, hip_mnist.py; fp32:
    hip_mnist_f32.py, int64 fixed-point gradient accumulation)."""
    from distributedtf_amd.models.mnist import MnistArch
    arch = MnistArch()
    dev = torch.device("cuda")
    out = []
    for rep in range(2):
        e = PopulationEngine(arch, len(sizes), dev, backend="hip", compute_dtype=dtype)
        hps = []
        for i, bs in enumerate(sizes):
            hp = {"opt_case": {"optimizer": "Adam", "lr": 1e-3}, "batch_size": bs, "initializer": "he_init"}
            e.add_member(None, hp, seed=7 + i)
            hps.append(hp)
        g = torch.Generator().manual_seed(3)
        batches = [((torch.rand(bs, 28, 28, 1, generator=g) * 255).to(dev),
                    torch.randint(0, 10, (bs,), generator=g).to(dev)) for bs in sizes]
        slots = list(range(len(sizes)))
        for _ in range(steps):
            losses = e.train_step(slots, batches, hps, [1e-3] * len(sizes))
        torch.cuda.synchronize()
        out.append((e.state.clone(), losses.cpu()))
    same = torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    print("mnist %s sizes %s steps %d: bitwise identical %s, losses %s" % (str(dtype).split(".")[-1], sizes, steps,
                                                                          same, out[0][1].tolist()),
          flush=True)
    return same


if ops.half_mode():
    h = dict(dtype=torch.float16, loss_scale=128.0)
    ok = all([run(20, [16, 24], 4, **h), run(56, [128], 3, **h), run(56, [128] * 4, 2, **h),
              run(50, [4, 6], 3, image=64, **h)])
    print("DET_OK" if ok else "DET_FAIL")
    sys.exit(0 if ok else 1)
ok = all([run(20, [16, 24], 4), run(56, [128], 3), run(56, [128] * 4, 2), run(20, [16, 24], 4, version=1),
          run(56, [128] * 2, 2, version=1), run_mnist([40, 72], 4),
          run(50, [4, 6], 3, image=64), run(50, [8, 8], 2, version=1, image=64),
          # the fp32 CIFAR step (f32conv.hip: int64 fixed-point accumulation in this build)
          run(20, [16, 24], 4, dtype=torch.float32), run(20, [16, 24], 3, version=1, dtype=torch.float32),
          run_mnist([40, 72], 4, dtype=torch.float32),
          # the fp32 ImageNet step (hip_imagenet_f32.py, f32conv.hip + f32net.hip)
          run(50, [4, 6], 2, image=64, dtype=torch.float32), run(50, [4, 4], 2, version=1, image=64, dtype=torch.float32)])
print("DET_OK" if ok else "DET_FAIL")
sys.exit(0 if ok else 1)
