"""Datasets: CIFAR-10 binary records, MNIST IDX, synthetic device batches, augmentation.

* CIFAR-10 (reference ``cifar10_main.py:34-135``): 3073-byte records (label +
  CHW uint8), ``data_batch_{1..5}.bin`` / ``test_batch.bin``; training
  preprocessing = pad to 40x40, random 32x32 crop, random horizontal flip, then
  ``per_image_standardization`` (mean / max(std, 1/sqrt(N))) for every image.
  The whole dataset is kept on the GPU as uint8 NHWC and batches are gathered
  and augmented on-device (no CPU input pipeline).
* MNIST (``mnist_model.py:131-138``): gz IDX files; pixels NOT normalised
  (0..255 floats, Appendix A5) unless ``normalize=True``.
* Synthetic (``model_helpers.py:59-86`` / ``resnet_run_loop.py:108-129``): the
  reference feeds constant zeros; here a fixed device-resident batch of
  standard-normal images and uniform labels (zeros would let DVFS inflate
  throughput numbers, and labels 0 make the loss trivial).
"""

from __future__ import annotations

import gzip
import os
from typing import Optional, Tuple

import numpy as np
import torch

CIFAR_TRAIN_FILES = ["data_batch_%d.bin" % i for i in range(1, 6)]
CIFAR_TEST_FILES = ["test_batch.bin"]
CIFAR_NUM_TRAIN, CIFAR_NUM_TEST = 50000, 10000
MNIST_NUM_TRAIN, MNIST_NUM_TEST = 60000, 10000


def _cifar_dir(data_dir: str) -> Optional[str]:
    for d in (os.path.join(data_dir, "cifar-10-batches-bin"), data_dir):
        if os.path.isfile(os.path.join(d, CIFAR_TEST_FILES[0])):
            return d
    return None


def cifar10_available(data_dir: Optional[str]) -> bool:
    return bool(data_dir) and _cifar_dir(data_dir) is not None


def load_cifar10(data_dir: str) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Returns uint8 NHWC images and int64 labels: (train_x, train_y, test_x, test_y)."""
    d = _cifar_dir(data_dir)
    if d is None:
        raise FileNotFoundError("CIFAR-10 binaries not found under %s" % data_dir)

    def read(files):
        raw = np.concatenate([np.fromfile(os.path.join(d, f), dtype=np.uint8) for f in files])
        rec = raw.reshape(-1, 3073)
        y = rec[:, 0].astype(np.int64)
        x = rec[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy()
        return x, y

    trx, tr_y = read(CIFAR_TRAIN_FILES)
    tex, te_y = read(CIFAR_TEST_FILES)
    return trx, tr_y, tex, te_y


def per_image_standardization(x: torch.Tensor) -> torch.Tensor:
    """tf.image.per_image_standardization over [B, H, W, C] float."""
    n = x[0].numel()
    flat = x.reshape(x.shape[0], -1)
    mean = flat.mean(dim=1, keepdim=True)
    std = flat.std(dim=1, unbiased=False, keepdim=True)
    adj = torch.clamp(std, min=1.0 / float(np.sqrt(n)))
    return ((flat - mean) / adj).reshape(x.shape)


def _mix32(h):
    h = h.astype(np.uint32)
    h ^= h >> np.uint32(16)
    h = (h * np.uint32(0x7FEB352D)).astype(np.uint32)
    h ^= h >> np.uint32(15)
    h = (h * np.uint32(0x846CA68B)).astype(np.uint32)
    h ^= h >> np.uint32(16)
    return h


def augment_params(seed: int, counter: int, n: int):
    """Crop offsets / flip bits drawn by the HIP augmentation kernel (data.hip) for batch positions 0..n-1."""
    with np.errstate(over="ignore"):
        pos = np.arange(n, dtype=np.uint32)
        inner = _mix32((np.uint32(counter & 0xFFFFFFFF) * np.uint32(0x9E3779B9)).astype(np.uint32) + pos)
        h = _mix32(np.uint32(seed & 0xFFFFFFFF) ^ inner)
    return (h % 9).astype(np.int64), ((h >> 8) % 9).astype(np.int64), ((h >> 16) & 1).astype(bool)


def augment_cifar_with(x_u8: torch.Tensor, oy, ox, flip) -> torch.Tensor:
    """pad 4 -> crop at (oy, ox) -> optional horizontal flip -> standardize (cifar10_main.py:98-108)."""
    b = x_u8.shape[0]
    dev = x_u8.device
    oy, ox, flip = (torch.as_tensor(t, device=dev) for t in (oy, ox, flip))
    x = x_u8.float()
    xp = torch.nn.functional.pad(x.permute(0, 3, 1, 2), (4, 4, 4, 4)).permute(0, 2, 3, 1)
    ar = torch.arange(32, device=dev)
    rows = (oy[:, None] + ar[None, :])  # [B, 32]
    cols = (ox[:, None] + ar[None, :])
    cols = torch.where(flip[:, None], cols.flip(1), cols)
    bi = torch.arange(b, device=dev)[:, None, None]
    out = xp[bi, rows[:, :, None], cols[:, None, :]]
    return per_image_standardization(out)


def augment_cifar(x_u8: torch.Tensor, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    """pad 4 -> random crop 32 -> random flip -> standardize. [B,32,32,3] uint8 -> float32 (torch ops)."""
    b = x_u8.shape[0]
    dev = x_u8.device
    oy = torch.randint(0, 9, (b,), device=dev, generator=gen)
    ox = torch.randint(0, 9, (b,), device=dev, generator=gen)
    flip = torch.rand(b, device=dev, generator=gen) < 0.5
    return augment_cifar_with(x_u8, oy, ox, flip)


def eval_cifar(x_u8: torch.Tensor) -> torch.Tensor:
    return per_image_standardization(x_u8.float())


def synthetic_images(n: int, shape, num_classes: int, seed: int, device, dtype=torch.float32):
    g = torch.Generator().manual_seed(int(seed))
    x = torch.randn((n,) + tuple(shape), generator=g).to(dtype)
    y = torch.randint(0, num_classes, (n,), generator=g)
    return x.to(device), y.to(device)


def learnable_cifar(n_train: int = 10000, n_test: int = 2000, seed: int = 7, noise: float = 2.5,
                    num_classes: int = 10):
    """A learnable CIFAR-shaped dataset that needs no download (the real CIFAR-10 is not on these machines):
    uint8 NHWC 32x32x3 images with labels, so it runs through the real input path (on-device gather, pad-4 random
    crop, flip, per-image standardisation: data.hip / cifar10_main.py:98-108).

    Each class has a fixed smooth random template (an 8x8x3 Gaussian field upsampled bilinearly to 32x32, so a
    random crop and a flip keep most of it) and every image is ``template[label] * contrast + noise`` with a
    per-image random contrast in [0.6, 1.4], brightness shift and i.i.d. pixel noise of ``noise`` template
    standard deviations.  Chance accuracy is 1/num_classes; a ResNet-20 reaches well above it within a few hundred
    steps (ResNet-8 fp32 on CPU at noise 2.5: training loss 2.1 -> 0.05 in 500 steps of batch 64; eval accuracy with the
    reference's 0.997-momentum moving BN statistics 0.58 / 0.77 after 600 steps, still rising), so loss / accuracy
    trajectories of two implementations can be compared (tests/test_gpu_trajectory.py).
    Returns (train_x, train_y, test_x, test_y) as numpy arrays."""
    g = torch.Generator().manual_seed(int(seed))
    base = torch.randn(num_classes, 3, 8, 8, generator=g)
    tmpl = torch.nn.functional.interpolate(base, size=(32, 32), mode="bilinear", align_corners=False)
    tmpl = tmpl / tmpl.flatten(1).std(dim=1).view(-1, 1, 1, 1)

    def make(n):
        y = torch.randint(0, num_classes, (n,), generator=g)
        contrast = 0.6 + 0.8 * torch.rand(n, 1, 1, 1, generator=g)
        shift = 0.3 * torch.randn(n, 1, 1, 1, generator=g)
        x = tmpl[y] * contrast + shift + noise * torch.randn(n, 3, 32, 32, generator=g)
        x = (x * 40.0 + 128.0).round().clamp(0, 255).to(torch.uint8)
        return x.permute(0, 2, 3, 1).contiguous().numpy(), y.numpy().astype(np.int64)

    trx, tr_y = make(n_train)
    tex, te_y = make(n_test)
    return trx, tr_y, tex, te_y


def _idx(path, offset, dtype=np.uint8):
    with gzip.open(path, "rb") as f:
        return np.frombuffer(f.read(), dtype, offset=offset)


def mnist_available(data_dir: Optional[str]) -> bool:
    return bool(data_dir) and os.path.isfile(os.path.join(data_dir, "t10k-images-idx3-ubyte.gz"))


def load_mnist(data_dir: str, normalize: bool = False):
    trx = _idx(os.path.join(data_dir, "train-images-idx3-ubyte.gz"), 16).astype(np.float32).reshape(-1, 28, 28, 1)
    tr_y = _idx(os.path.join(data_dir, "train-labels-idx1-ubyte.gz"), 8).astype(np.int64)
    tex = _idx(os.path.join(data_dir, "t10k-images-idx3-ubyte.gz"), 16).astype(np.float32).reshape(-1, 28, 28, 1)
    te_y = _idx(os.path.join(data_dir, "t10k-labels-idx1-ubyte.gz"), 8).astype(np.int64)
    if normalize:
        trx /= 255.0
        tex /= 255.0
    return trx, tr_y, tex, te_y


class IndexBatch:
    """A training batch named by dataset rows, materialised lazily.

    Engines with an on-device input path (the HIP ResNet step) consume the
    indices directly -- gather, augmentation and the bf16 stem packing run in
    one kernel inside the captured step graph; every other engine calls
    :meth:`materialize`.
    """

    def __init__(self, ds: "DeviceDataset", idx: torch.Tensor):
        self.ds, self.idx = ds, idx

    def __len__(self):
        return int(self.idx.numel())

    def materialize(self, gen=None):
        return self.ds.batch(self.idx, gen)


def batch_len(b) -> int:
    return len(b) if isinstance(b, IndexBatch) else int(b[1].shape[0])


class DeviceDataset:
    """Train/eval arrays resident on the device with per-member epoch shuffling.

    CIFAR-style uint8 32x32x3 data with ``augment=augment_cifar`` on a GPU uses
    the fused HIP kernel (data.hip) for gather + pad/crop/flip + standardize.
    """

    def __init__(self, train_x, train_y, test_x, test_y, device, augment=None, eval_transform=None, seed=0):
        self.train_x = torch.as_tensor(train_x).to(device).contiguous()
        self.train_y = torch.as_tensor(train_y).to(device).long().contiguous()
        self.test_x = torch.as_tensor(test_x).to(device).contiguous()
        self.test_y = torch.as_tensor(test_y).to(device).long().contiguous()
        self.augment = augment
        self.eval_transform = eval_transform
        self._eval_cache = None
        self.device = torch.device(device)
        self.hip_augment = (self.device.type == "cuda" and augment is augment_cifar
                            and self.train_x.dtype == torch.uint8 and tuple(self.train_x.shape[1:]) == (32, 32, 3))
        self.rng_seed = int(seed) & 0x7FFFFFFF
        self.rng_counter = 0

    @property
    def num_train(self):
        return int(self.train_x.shape[0])

    def next_rng(self):
        """(seed, counter) for one augmentation launch; the counter advances per launch."""
        self.rng_counter = (self.rng_counter + 1) & 0x7FFFFFFF
        return self.rng_seed, self.rng_counter

    def batch(self, idx: torch.Tensor, gen=None):
        if self.hip_augment:
            from .. import ops
            n = int(idx.numel())
            x = torch.empty(n, 32, 32, 3, dtype=torch.float32, device=self.device)
            y = torch.empty(n, dtype=torch.int64, device=self.device)
            rng = torch.tensor(self.next_rng(), dtype=torch.int32).to(self.device)
            ops.augment_cifar(self.train_x, self.train_y, idx.long().contiguous(), rng, True, out32=x, lab64=y)
            return x, y
        x = self.train_x[idx]
        x = self.augment(x, gen) if self.augment is not None else x.float()
        return x, self.train_y[idx]

    def eval_set(self):
        if self._eval_cache is None:
            x = self.test_x
            x = self.eval_transform(x) if self.eval_transform is not None else x.float()
            self._eval_cache = (x, self.test_y)
        return self._eval_cache


class SyntheticDataset:
    """Fixed device-resident batch reused every step (reference synthetic mode)."""

    def __init__(self, shape, num_classes, device, max_batch=256, n_eval=1000, seed=1234, dtype=torch.float32):
        self.x, self.y = synthetic_images(max_batch, shape, num_classes, seed, device, dtype)
        self.ex, self.ey = synthetic_images(n_eval, shape, num_classes, seed + 1, device, dtype)
        self.num_train = CIFAR_NUM_TRAIN if tuple(shape)[0] == 32 else 50000
        self.device = device

    def batch_slice(self, b: int):
        return self.x[:b], self.y[:b]

    def eval_set(self):
        return self.ex, self.ey
