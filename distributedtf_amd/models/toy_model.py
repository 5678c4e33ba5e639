"""Toy quadratic from Jaderberg et al. 2017 (PBT paper), CPU plumbing model.

Reference ``toy_model.py:7-89``:
  * ``theta = (0.9, 0.9)``; objective ``Q = 1.2 - (t0^2 + t1^2)``;
  * surrogate ``1.2 - (h0*t0^2 + h1*t1^2)``, loss ``(Q - surrogate)^2``;
  * fixed gradient descent, lr 0.02 (optimizer hparams are ignored, Appendix A6);
  * member 0 gets ``h = (0, 1)``, every other member ``h = (1, 0)``;
  * logs ``theta.csv`` and ``learning_curve.csv`` (``global_step, accuracy,
    optimizer, lr``) BEFORE each step, checkpoint restored if the dir exists.

The gradient is closed-form (d/dt_i of ``((1-h_i) t_i^2 + ...)^2``) so a step is a
handful of scalar flops; no framework graph is built per call.
"""

from __future__ import annotations

import csv
import os
from typing import List

import torch

from .model_base import ModelBase

_LR = 0.02


def _objective(theta: torch.Tensor) -> float:
    return float(1.2 - (theta[0] ** 2 + theta[1] ** 2))


def _step(theta: torch.Tensor, h0: float, h1: float) -> torch.Tensor:
    # loss = (Q - S)^2 = (-(1-h0) t0^2 - (1-h1) t1^2)^2 ; r = (1-h0) t0^2 + (1-h1) t1^2
    r = (1.0 - h0) * theta[0] ** 2 + (1.0 - h1) * theta[1] ** 2
    grad = torch.stack([4.0 * r * (1.0 - h0) * theta[0], 4.0 * r * (1.0 - h1) * theta[1]])
    return theta - _LR * grad


def _append_csv(path: str, fields: List[str], rows: List[dict]):
    exists = os.path.isfile(path)
    with open(path, "a", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        if not exists:
            w.writeheader()
        for r in rows:
            w.writerow(r)


def run_training(hp, theta: torch.Tensor, global_step: int, save_dir: str, train_epochs: int):
    """Advance ``train_epochs`` GD steps, append CSV logs; returns (theta, step, obj)."""
    log = []
    h0, h1 = float(hp["h_0"]), float(hp["h_1"])
    opt = hp.get("opt_case", {})
    for _ in range(train_epochs):
        log.append((float(theta[0]), float(theta[1]), global_step, _objective(theta),
                    opt.get("optimizer"), opt.get("lr")))
        theta = _step(theta, h0, h1)
        global_step += 1
    os.makedirs(save_dir, exist_ok=True)
    _append_csv(os.path.join(save_dir, "theta.csv"), ["theta_0", "theta_1"],
                [{"theta_0": r[0], "theta_1": r[1]} for r in log])
    _append_csv(os.path.join(save_dir, "learning_curve.csv"), ["global_step", "accuracy", "optimizer", "lr"],
                [{"global_step": r[2], "accuracy": r[3], "optimizer": r[4], "lr": r[5]} for r in log])
    return theta, global_step, _objective(theta)


def main(hp, model_id, save_base_dir, data_dir, train_epochs):
    """Disk-resumable entry (reference ``toy_model.main``): returns ``[global_step, obj]``."""
    save_dir = save_base_dir + str(model_id)
    ckpt = os.path.join(save_dir, "model.ckpt")
    theta = torch.tensor([0.9, 0.9], dtype=torch.float64)
    step = 0
    if os.path.isfile(ckpt):
        blob = torch.load(ckpt, map_location="cpu", weights_only=True)
        theta = blob["state"][:2].clone()
        step = int(blob["state"][2])
    theta, step, obj = run_training(hp, theta, step, save_dir, train_epochs)
    torch.save({"state": torch.cat([theta, torch.tensor([float(step)], dtype=torch.float64)])}, ckpt)
    with open(os.path.join(save_dir, "checkpoint"), "w") as f:
        f.write('model_checkpoint_path: "model.ckpt"\n')
    return [step, obj]


class ToyModel(ModelBase):
    def __init__(self, cluster_id, hparams, save_base_dir, seed=None):
        super().__init__(cluster_id, hparams, save_base_dir, seed=seed)
        self._pin_h()
        self._state = torch.tensor([0.9, 0.9, 0.0], dtype=torch.float64)

    def _pin_h(self):
        if self.cluster_id == 0:
            self.hparams["h_0"], self.hparams["h_1"] = 0.0, 1.0
        else:
            self.hparams["h_0"], self.hparams["h_1"] = 1.0, 0.0

    def train(self, epoches_to_train, total_epochs):
        theta, step = self._state[:2].clone(), int(self._state[2])
        theta, step, obj = run_training(self.hparams, theta, step, self.save_dir, epoches_to_train)
        self._state = torch.cat([theta, torch.tensor([float(step)], dtype=torch.float64)])
        self.accuracy = obj
        self.epoches_trained += epoches_to_train
        self.save_checkpoint()

    def set_values(self, values):
        # hparams are NOT inherited for the toy problem (reference toy_model.py:83-89)
        self._pin_h()

    def export_state(self):
        return self._state

    def import_state(self, flat):
        self._state = flat.detach().to(torch.float64).clone()
