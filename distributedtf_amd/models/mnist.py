"""MNIST 2-conv CNN (reference ``mnist_model.py:62-126``) as a flat-parameter arch.

conv5x5x32 SAME + bias + ReLU -> maxpool 2/2 -> conv5x5x64 SAME + bias + ReLU ->
maxpool 2/2 -> dense 3136->1024 + ReLU -> dropout 0.4 (train only) -> dense 10.
The initializer hparam applies to conv1, conv2 and dense1 (``:74,86,92``);
dense2 keeps the tf.layers default (glorot uniform); biases start at zero.
No regularizer (``n_reg = 0``).  Layout: NHWC activations, OHWI kernels,
dense kernels ``[out, in]`` with ``in`` in (H, W, C) order like TF's flatten.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .resnet import init_kernel

_SHAPES = [
    ("conv1_w", (32, 5, 5, 1)), ("conv1_b", (32,)),
    ("conv2_w", (64, 5, 5, 32)), ("conv2_b", (64,)),
    ("dense1_w", (1024, 7 * 7 * 64)), ("dense1_b", (1024,)),
    ("dense2_w", (10, 1024)), ("dense2_b", (10,)),
]


class MnistArch:
    name = "mnist_cnn"
    hip_supported = True  # engine/hip_mnist.py (ops/csrc/mnist.hip + gemm.hip)
    num_classes = 10
    input_shape = (28, 28, 1)

    def __init__(self, dropout: float = 0.4):
        self.dropout = dropout
        self.offsets = {}
        off = 0
        for n, shp in _SHAPES:
            numel = 1
            for d in shp:
                numel *= d
            self.offsets[n] = (off, shp)
            off += numel
        self.n_params = off
        self.n_running = 0
        self.n_reg = 0

    def tf_variables(self, params, slot1, slot2, running, optimizer, step, dtype="float32"):
        """Reference ``cnn_model_fn`` names/layouts: conv2d, conv2d_1 (HWIO kernels + bias), dense (3136 x 1024),
        dense_1 (1024 x 10), optimizer slots, global_step (``mnist_model.py:62-126``)."""
        from ..engine.optim import tf_optimizer_tensors
        out, trainable = {}, []
        names = {"conv1": "conv2d", "conv2": "conv2d_1", "dense1": "dense", "dense2": "dense_1"}
        for n, (off, shp) in self.offsets.items():
            layer, kind = n.split("_")
            numel = 1
            for d in shp:
                numel *= d
            if kind == "w":
                layout = (lambda a: a.transpose(1, 2, 3, 0)) if len(shp) == 4 else (lambda a: a.T)
                tf_name = names[layer] + "/kernel"
            else:
                layout, tf_name = (lambda a: a), names[layer] + "/bias"
            t = [layout(a[off:off + numel].reshape(shp)).astype(dtype) for a in (params, slot1, slot2)]
            out[tf_name] = t[0]
            trainable.append((tf_name, t[0], t[1], t[2]))
        out.update(tf_optimizer_tensors(optimizer, trainable, step))
        return out

    def view(self, params, name):
        off, shp = self.offsets[name]
        numel = 1
        for d in shp:
            numel *= d
        return params[off:off + numel].view(shp)

    def init_params(self, initializer, seed):
        gen = torch.Generator().manual_seed(int(seed))
        p = torch.zeros(self.n_params)
        for n, shp in _SHAPES:
            if n.endswith("_w"):
                init = None if n == "dense2_w" else initializer
                off, _ = self.offsets[n]
                w = init_kernel(shp, init, gen)
                p[off:off + w.numel()] = w.flatten()
        return p, torch.zeros(0)

    def forward(self, params, running, x_nhwc, training=True, dtype=torch.float32, dropout_mask=None):
        """``dropout_mask`` (bool [B, 1024], True = kept) replaces the random draw, e.g. with the HIP head
        kernel's counter-hash mask (``engine.hip_mnist.dropout_keep_mask``) for numerics tests."""
        x = x_nhwc.reshape(-1, 28, 28, 1).permute(0, 3, 1, 2).to(dtype)
        w1 = self.view(params, "conv1_w").permute(0, 3, 1, 2).to(dtype)
        w2 = self.view(params, "conv2_w").permute(0, 3, 1, 2).to(dtype)
        x = F.relu(F.conv2d(x, w1, self.view(params, "conv1_b").to(dtype), padding=2))
        x = F.max_pool2d(x, 2, 2)
        x = F.relu(F.conv2d(x, w2, self.view(params, "conv2_b").to(dtype), padding=2))
        x = F.max_pool2d(x, 2, 2)
        x = x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)  # TF flatten order (H, W, C)
        x = F.relu(F.linear(x, self.view(params, "dense1_w").to(dtype), self.view(params, "dense1_b").to(dtype)))
        if training and self.dropout > 0:
            if dropout_mask is not None:
                x = x * dropout_mask.to(x.device, x.dtype) / (1.0 - self.dropout)
            else:
                x = F.dropout(x, self.dropout, training=True)
        return F.linear(x.float(), self.view(params, "dense2_w"), self.view(params, "dense2_b"))

    def flops_per_image(self):
        return 2.0 * (28 * 28 * 32 * 25 + 14 * 14 * 64 * 800 + 3136 * 1024 + 1024 * 10)
