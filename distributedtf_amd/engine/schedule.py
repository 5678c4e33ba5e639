"""Per-member learning-rate schedules (host side, evaluated per step).

CIFAR-10 ResNet (reference ``cifar10_main.py:188-208`` +
``resnet_run_loop.py:135-173``):
  * ``lr0 = lr * batch_size / 128``;
  * decay is OFF unless ``decay_steps not in {0, 100}``; then there are
    ``ceil(100/decay_steps) - 1`` boundaries at multiples of
    ``250 * decay_steps / 100`` epochs with values ``lr0 * decay_rate^i``;
  * boundaries are converted to steps with ``int(50000/batch * epochs)`` and
    evaluated with TF ``piecewise_constant`` semantics (``step <= b0`` -> v0).

MNIST uses the optimizer's constant learning rate (``mnist_model.py:27-60``).
"""

from __future__ import annotations

import bisect
import math
from typing import Dict, List, Tuple


def cifar_boundaries(hparams: Dict, num_images: int = 50000, batch_denom: int = 128,
                     total_epochs: float = 250.0) -> Tuple[List[int], List[float]]:
    ds = int(hparams.get("decay_steps", 0))
    rate = float(hparams.get("decay_rate", 1.0))
    batch = int(hparams["batch_size"])
    lr0 = float(hparams["opt_case"]["lr"]) * batch / batch_denom
    if ds != 0 and ds != 100:
        n = int(math.ceil(100.0 / ds)) - 1
        decay_epochs = total_epochs * ds / 100.0
        rates = [1.0]
        epochs = []
        for i in range(n):
            rates.append(rate * rates[i])
            epochs.append(decay_epochs * (i + 1))
    else:
        epochs, rates = [total_epochs], [1.0, 1.0]
    per_epoch = num_images / float(batch)
    bounds = [int(per_epoch * e) for e in epochs]
    return bounds, [lr0 * r for r in rates]


def piecewise_constant(step: int, bounds: List[int], values: List[float]) -> float:
    if not bounds:
        return values[0] if values else 0.01
    return values[bisect.bisect_left(bounds, step)]


def cifar_lr(hparams: Dict, step: int, num_images: int = 50000) -> float:
    b, v = cifar_boundaries(hparams, num_images)
    return piecewise_constant(step, b, v)


def constant_lr(hparams: Dict, step: int) -> float:
    return float(hparams["opt_case"]["lr"])
