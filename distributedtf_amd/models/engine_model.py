"""``EngineModel``: a ``ModelBase`` whose state lives in a shared ``PopulationEngine``.

All members of one model family on one rank/device share one engine, so
``TrainingWorker.train`` -> ``train_population`` runs them TOGETHER: each step
is one population-wide forward/backward + one fused optimizer launch, and
members with different batch sizes / epoch lengths simply drop out of the active
set when their epoch is done.  (The reference trains members one after another,
each rebuilding its graph and restoring a checkpoint: ``training_worker.py:64``.)
"""

from __future__ import annotations

import csv
import math
import os
import time
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from .model_base import ModelBase
from ..data import datasets
from ..engine.population import PopulationEngine


def default_device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class EngineModel(ModelBase):
    _engines: Dict[tuple, PopulationEngine] = {}
    _datasets: Dict[tuple, object] = {}

    # subclass hooks ----------------------------------------------------------
    def make_arch(self):
        raise NotImplementedError

    def make_dataset(self, device):
        raise NotImplementedError

    def learning_rate(self, step: int) -> float:
        raise NotImplementedError

    def steps_per_epoch(self) -> int:
        raise NotImplementedError

    def csv_row(self, accuracy: float):
        raise NotImplementedError

    # ------------------------------------------------------------------------
    def __init__(self, cluster_id, hparams, save_base_dir, seed=None, device=None, backend="auto",
                 capacity=8, use_synthetic_data=None, data_dir=None, max_train_steps=None,
                 checkpoint_every_round=True, eval_every_round=True, dp=None, tf_checkpoint=False, **kw):
        super().__init__(cluster_id, hparams, save_base_dir, seed=seed)
        self.dp = dp  # parallel.dataparallel.DPContext: this member is one replica of a data-parallel group
        self.options = dict(kw)
        self.device = torch.device(device) if device is not None else default_device()
        self.data_dir = data_dir
        self.use_synthetic_data = use_synthetic_data
        self.max_train_steps = max_train_steps
        self.checkpoint_every_round = checkpoint_every_round
        self.tf_checkpoint = tf_checkpoint  # also export the reference's TF tensor-bundle format every round
        self.eval_every_round = eval_every_round
        self.arch = self.make_arch()
        key = (type(self).__name__, str(self.device), self.arch.name, backend)
        eng = EngineModel._engines.get(key)
        if eng is None or not eng.free_slots:
            eng = self._grow_or_create(key, eng, capacity, backend)
        self.engine = eng
        if dp is not None:
            eng.set_data_parallel(dp)
        self._engine_key = key
        init_seed = (seed if seed is not None else int(time.time() * 1000) % 100000) * 1009 + self.cluster_id
        self.slot = eng.add_member(self, self.hparams, init_seed)
        self.last_loss = float("nan")
        self.images_trained = 0

    def _grow_or_create(self, key, eng, capacity, backend):
        if eng is None:
            eng = PopulationEngine(self.arch, capacity, self.device, backend=backend)
        else:
            new = PopulationEngine(self.arch, eng.capacity * 2, self.device, backend=backend)
            new.state[:eng.capacity].copy_(eng.state)
            new.members = dict(eng.members)
            new.free_slots = [s for s in range(new.capacity) if s not in new.members]
            new.host_step[:eng.capacity] = eng.host_step
            for slot, m in new.members.items():
                m.engine = new
            new.backend.on_params_changed(list(new.members))
            eng = new
        EngineModel._engines[key] = eng
        return eng

    @classmethod
    def reset_engines(cls):
        EngineModel._engines.clear()
        EngineModel._datasets.clear()

    def dataset(self):
        key = (type(self).__name__, str(self.device), self.data_dir, self.use_synthetic_data)
        ds = EngineModel._datasets.get(key)
        if ds is None:
            ds = self.make_dataset(self.device)
            EngineModel._datasets[key] = ds
        return ds

    # ------------------------------------------------------------- state API
    def state_view(self):
        return self.engine.state_row(self.slot)

    def export_state(self):
        return self.engine.state_row(self.slot)

    def import_state(self, flat):
        self.engine.state_row(self.slot).copy_(flat.to(self.engine.state.device, torch.float32))
        self.on_state_imported()

    def on_state_imported(self, step=None):
        self.engine.on_state_imported(self.slot, step)

    def tf_variables(self):
        """This member's state as the reference's TF1 checkpoint variables (name -> numpy array)."""
        e, s = self.engine, self.slot
        row = e.state[s].detach().float().cpu().numpy()
        P, Pp, R = e.P, e.Pp, e.R
        return self.arch.tf_variables(row[:P], row[Pp:Pp + P], row[2 * Pp:2 * Pp + P], row[3 * Pp:3 * Pp + R],
                                      self.hparams["opt_case"]["optimizer"], int(self.global_step))

    def import_tf_checkpoint(self, prefix: str) -> int:
        """Load a TF tensor bundle written under the reference's variable names (ours or TF's own ``Saver``)
        into this member: weights, BN moving statistics, the optimizer slots present in the bundle, global_step.
        The name -> state-row mapping is ``tf_variables`` evaluated on position indices, so every layout
        transform is inverted exactly.  Returns the number of tensors applied."""
        import numpy as np
        from ..utils.tf_bundle import load_bundle
        e, s = self.engine, self.slot
        P, Pp, R = e.P, e.Pp, e.R
        ar = np.arange(max(P, R), dtype=np.float64)
        pos = self.arch.tf_variables(ar[:P], Pp + ar[:P], 2 * Pp + ar[:P], 3 * Pp + ar[:R],
                                     self.hparams["opt_case"]["optimizer"], 0, dtype="float64")
        tensors = load_bundle(prefix)
        row = e.state[s].detach().cpu().numpy().copy()
        used = 0
        for name, where in pos.items():
            if name in ("global_step", "beta1_power", "beta2_power") or name not in tensors:
                continue
            val = np.asarray(tensors[name], dtype=np.float32)
            if val.shape != where.shape:
                raise ValueError("%s: checkpoint shape %s != model %s" % (name, val.shape, where.shape))
            row[where.astype(np.int64).ravel()] = val.ravel()
            used += 1
        step = int(np.asarray(tensors.get("global_step", 0)).reshape(-1)[0]) if "global_step" in tensors else 0
        row[3 * Pp + R] = float(step)
        e.state[s].copy_(torch.from_numpy(row).to(e.state.device))
        self.on_state_imported(step)
        return used

    def release(self):
        self.engine.remove_member(self.slot)

    @property
    def global_step(self) -> int:
        return self.engine.host_step[self.slot]

    def set_values(self, values):
        super().set_values(values)

    # ------------------------------------------------------------- training
    @property
    def is_dp_follower(self) -> bool:
        """Replicas other than the group's first one train and evaluate but write no files."""
        return self.dp is not None and self.dp.rank != 0

    def save_checkpoint(self, wait: bool = False) -> None:
        if not self.is_dp_follower:
            super().save_checkpoint(wait)

    def _batch(self, ds, gen):
        b = int(self.hparams["batch_size"])
        if self.dp is not None:
            b = max(1, self.dp.local_batch(b))  # this replica's shard of the member's batch
        if hasattr(ds, "batch_slice"):
            return ds.batch_slice(b)
        if not hasattr(self, "_perm") or self._perm_pos + b > self._perm.numel():
            self._perm = torch.randperm(ds.num_train, device=ds.train_x.device, generator=gen)
            self._perm_pos = 0
        idx = self._perm[self._perm_pos:self._perm_pos + b]
        self._perm_pos += b
        if getattr(ds, "hip_augment", False):
            return datasets.IndexBatch(ds, idx)
        return ds.batch(idx, gen)

    def n_steps(self, num_epoch: int) -> int:
        n = num_epoch * self.steps_per_epoch()
        if self.max_train_steps:
            n = min(n, int(self.max_train_steps))
        return max(1, n)

    @classmethod
    def train_population(cls, members: List["EngineModel"], num_epoch: int, total_epochs: int):
        failed = {}
        groups: Dict[int, List[EngineModel]] = {}
        for m in members:
            groups.setdefault(id(m.engine), []).append(m)
        for ms in groups.values():
            eng = ms[0].engine
            ds = ms[0].dataset()
            gen = None
            if ds.device.type == "cuda":
                gen = torch.Generator(device=ds.device)
                # replicas of a data-parallel group draw different shards (the member rng stays in lockstep)
                gen.manual_seed(int(ms[0].rng.random() * 1e9) + (7919 * ms[0].dp.rank if ms[0].dp else 0))
            todo = {m.slot: m.n_steps(num_epoch) for m in ms}
            by_slot = {m.slot: m for m in ms}
            done = 0
            loss_acc = {m.slot: None for m in ms}
            while True:
                active = [s for s in sorted(todo) if todo[s] > done]
                if not active:
                    break
                batches = [by_slot[s]._batch(ds, gen) for s in active]
                hps = [by_slot[s].hparams for s in active]
                lrs = [by_slot[s].learning_rate(eng.host_step[s]) for s in active]
                losses = eng.train_step(active, batches, hps, lrs)
                for i, s in enumerate(active):
                    by_slot[s].images_trained += datasets.batch_len(batches[i])
                for i, s in enumerate(active):
                    loss_acc[s] = losses[i]  # view, no host sync
                done += 1
            dp = ms[0].dp
            if dp is not None:
                # same NaN verdict and the same BatchNorm running statistics on every replica
                eng.dp_sync_running([m.slot for m in ms])
                for m in ms:
                    if loss_acc[m.slot] is not None:
                        t = loss_acc[m.slot].detach().float().reshape(1).clone()
                        dp.allreduce_mean_(t)
                        loss_acc[m.slot] = t[0]
            for m in ms:
                try:
                    if loss_acc[m.slot] is not None:
                        m.last_loss = float(loss_acc[m.slot].item())
                    m.finish_round(num_epoch)
                except Exception as e:  # member-level culling
                    failed[m.cluster_id] = e
        return failed

    def finish_round(self, num_epoch):
        if math.isnan(self.last_loss) or math.isinf(self.last_loss):
            self.accuracy = float("nan")
        elif self.eval_every_round:
            x, y = self.dataset().eval_set()
            self.accuracy = self.engine.evaluate(self.slot, x, y)
        self.write_learning_curve(self.accuracy)
        self.epoches_trained += num_epoch
        if self.checkpoint_every_round:
            self.save_checkpoint()
            if self.tf_checkpoint and not self.is_dp_follower:
                self.export_tf_checkpoint()

    def train(self, num_epoch, total_epochs):
        failed = type(self).train_population([self], num_epoch, total_epochs)
        if self.cluster_id in failed:
            raise failed[self.cluster_id]

    def write_learning_curve(self, accuracy):
        if self.is_dp_follower:
            return
        fields, row = self.csv_row(accuracy)
        d = self.ensure_save_dir()
        path = os.path.join(d, "learning_curve.csv")
        exists = os.path.isfile(path)
        with open(path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=fields)
            if not exists:
                w.writeheader()
            w.writerow(row)
