"""``ModelBase``: the population-member API.

Compatible with reference ``model_base.py:11-113``:
``ModelBase(cluster_id, hparams, save_base_dir)`` with ``train(num_epoch,
total_epochs)``, ``perturb_hparams()``, ``get_accuracy()``, ``get_values()`` ->
``[id, acc, hparams]`` and ``set_values(values)`` (hyper-parameters only).

Additions for the MI355X engine:
  * ``export_state()`` / ``import_state(t)`` -- the member's whole training state
    (weights, BN running stats, optimizer slots, step counter) as ONE flat
    tensor, so an exploit is a single RCCL send/recv (or a D2D copy);
  * ``save_checkpoint()`` / ``load_checkpoint()`` -- ``savedata/model_<id>/``;
  * ``train_population(members, ...)`` -- classmethod hook that lets a model
    family train all members resident on one GPU together (population-batched
    kernels) instead of the reference's serial loop (``training_worker.py:64``);
  * ``rng`` -- a per-member ``random.Random`` for reproducible explore steps.
"""

from __future__ import annotations

import os
import random
from typing import Any, Dict, List, Optional

import numpy as np

from ..pbt.hparams import perturb_hparams as _perturb


class ModelBase(object):
    # column-order contract of learning_curve.csv: 0=x, 1=accuracy, 3=lr
    CSV_X_COL, CSV_ACC_COL, CSV_LR_COL = 0, 1, 3

    def __init__(self, cluster_id: int, hparams: Dict[str, Any], save_base_dir: str,
                 seed: Optional[int] = None):
        self.cluster_id = int(cluster_id)
        self.hparams = hparams
        self.save_base_dir = save_base_dir
        self.epoches_trained = 0
        self.need_explore = False
        self._perturb_factors = [0.8, 1.2]
        if isinstance(self.hparams.get("batch_size"), np.ndarray):
            self.hparams["batch_size"] = self.hparams["batch_size"].item()
        self.accuracy = 0.0
        self.rng = random.Random(None if seed is None else seed * 7919 + self.cluster_id)

    # ------------------------------------------------------------------ paths
    @property
    def save_dir(self) -> str:
        return self.save_base_dir + str(self.cluster_id)

    def ensure_save_dir(self) -> str:
        os.makedirs(self.save_dir, exist_ok=True)
        return self.save_dir

    # ------------------------------------------------------------- training API
    def train(self, num_epoch: int, total_epochs: int):
        raise NotImplementedError

    @classmethod
    def train_population(cls, members: List["ModelBase"], num_epoch: int, total_epochs: int):
        """Train several resident members. Default: serial, like the reference.

        Returns ``{cluster_id: exception}`` for members that raised.
        """
        failed = {}
        for m in members:
            try:
                m.train(num_epoch, total_epochs)
            except Exception as e:  # member-level culling (training_worker.py:75-80)
                failed[m.cluster_id] = e
        return failed

    def perturb_hparams(self):
        _perturb(self.hparams, self.rng, tuple(self._perturb_factors))

    def get_accuracy(self):
        return self.accuracy

    def get_values(self):
        return [self.cluster_id, self.get_accuracy(), self.hparams]

    def set_values(self, values):
        self.hparams = values[2]

    # ---------------------------------------------------------- state transfer
    def export_state(self):
        """Flat tensor holding the member's full training state."""
        raise NotImplementedError

    def import_state(self, flat) -> None:
        raise NotImplementedError

    def state_numel(self) -> int:
        return int(self.export_state().numel())

    def state_device(self):
        return self.export_state().device

    def save_checkpoint(self) -> None:
        """Write ``savedata/model_<id>/model.ckpt`` (+ ``checkpoint`` state file)."""
        import torch
        d = self.ensure_save_dir()
        state = self.export_state().detach().to("cpu")
        torch.save({"state": state, "epoches_trained": self.epoches_trained,
                    "hparams": self.hparams}, os.path.join(d, "model.ckpt"))
        with open(os.path.join(d, "checkpoint"), "w") as f:
            f.write('model_checkpoint_path: "model.ckpt"\n')

    def has_checkpoint(self) -> bool:
        return os.path.isfile(os.path.join(self.save_dir, "model.ckpt"))

    def load_checkpoint(self) -> bool:
        import torch
        path = os.path.join(self.save_dir, "model.ckpt")
        if not os.path.isfile(path):
            return False
        blob = torch.load(path, map_location="cpu", weights_only=True)
        self.import_state(blob["state"])
        return True
