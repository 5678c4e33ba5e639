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
from ..utils.profiling import timed_phase


def default_device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class _LazyValues(dict):
    """Hook values: host scalars up front, device-derived ones (``cross_entropy``, ``train_accuracy``: one
    readback) only when a hook asks for them."""

    def __init__(self, fetch, base, extra=None):
        super().__init__(base)
        self._fetch = fetch
        self._extra = dict(extra or {})  # key -> fetch() for other device-derived values (``probabilities``)

    def _device(self):
        if not dict.__contains__(self, "cross_entropy"):
            h = self._fetch()
            dict.__setitem__(self, "cross_entropy", h["ce"])
            if h.get("acc") is not None:
                dict.__setitem__(self, "train_accuracy", h["acc"])

    def _other(self, key):
        f = self._extra.pop(key, None)
        if f is not None:
            v = f()
            if v is not None:
                dict.__setitem__(self, key, v)

    def __missing__(self, key):
        if key in ("cross_entropy", "train_accuracy"):
            self._device()
        else:
            self._other(key)
        if dict.__contains__(self, key):
            return dict.__getitem__(self, key)
        raise KeyError(key)

    def __contains__(self, key):
        if key in ("cross_entropy", "train_accuracy"):
            self._device()
        else:
            self._other(key)
        return dict.__contains__(self, key)

    def get(self, key, default=None):
        return self[key] if key in self else default


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
                 checkpoint_every_round=True, eval_every_round=True, dp=None, tf_checkpoint=False, ready_steps=None,
                 stop_threshold=None, batch_size=None, dtype="bf16", loss_scale=1.0, epochs_between_evals=1, **kw):
        super().__init__(cluster_id, hparams, save_base_dir, seed=seed)
        from ..utils.flags import get_dtype
        self.compute_dtype = get_dtype(dtype)  # --dtype: bf16 (HIP kernels) | fp32 / fp16 (PyTorch backend)
        self.loss_scale = float(loss_scale or 1.0)
        self.ready_steps = int(ready_steps) if ready_steps else None  # PBT ready interval in steps (--ready_steps)
        self.stop_threshold = stop_threshold  # --stop_threshold: end a member's train call once eval passes it
        # --epochs_between_evals: epochs per train -> eval cycle (reference _base.py:74-79, resnet_run_loop.py:446-447)
        self.epochs_between_evals = max(1, int(epochs_between_evals or 1))
        self.batch_size_override = int(batch_size) if batch_size else None  # --batch_size
        self._pin_batch_size()
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
        key = (type(self).__name__, str(self.device), self.arch.name, backend, self.compute_dtype, self.loss_scale)
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
        kw = dict(backend=backend, compute_dtype=self.compute_dtype, loss_scale=self.loss_scale)
        if eng is None:
            eng = PopulationEngine(self.arch, capacity, self.device, **kw)
        else:
            new = PopulationEngine(self.arch, eng.capacity * 2, self.device, **kw)
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

    def import_state(self, flat, step=None):
        """Overwrite this member's state row with ``flat`` (a host or device row).  ``step``: the source's step
        counter; if omitted it is taken from ``flat``'s step column (a host read for a host row)."""
        e = self.engine
        if step is None:
            step = int(round(float(flat[3 * e.Pp + e.R])))
        e.state_row(self.slot).copy_(flat.to(e.state.device, torch.float32))
        self.on_state_imported(step)

    def on_state_imported(self, step):
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

    def _pin_batch_size(self):
        if self.batch_size_override:
            self.hparams["batch_size"] = self.batch_size_override

    def set_values(self, values):
        super().set_values(values)
        self._pin_batch_size()

    def perturb_hparams(self):
        super().perturb_hparams()
        self._pin_batch_size()  # --batch_size fixes every member's batch (explore would move it)

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
            if b < self.dp.size:
                # an empty shard would still train on one image and the replica weights (local / member batch)
                # would sum to more than 1, scaling the all-reduced gradient up
                raise ValueError("member %d: batch_size %d < --dp_size %d (every replica needs >= 1 image)"
                                 % (self.cluster_id, b, self.dp.size))
            b = self.dp.local_batch(b)  # this replica's shard of the member's batch
        if hasattr(ds, "batch_slice"):
            return ds.batch_slice(b)
        gen = self._data_gen(ds, gen)
        if not hasattr(self, "_perm") or self._perm_pos + b > self._perm.numel():
            self._perm_gen_state = gen.get_state() if gen is not None else None  # (stream_state: exact resume)
            self._perm = torch.randperm(ds.num_train, device=ds.train_x.device, generator=gen)
            self._perm_pos = 0
        idx = self._perm[self._perm_pos:self._perm_pos + b]
        self._perm_pos += b
        if getattr(ds, "hip_augment", False):
            return datasets.IndexBatch(ds, idx)
        return ds.batch(idx, gen)

    def stream_state(self):
        """Explore rng + the member's data stream (its generator state when the current epoch permutation was drawn,
        the position in it, and the generator's current state): JSON-able, for the whole-run resume table."""
        d = super().stream_state()
        g = getattr(self, "_gen", None)
        if g is not None and getattr(self, "_perm_gen_state", None) is not None:
            d["data"] = {"perm_gen": self._perm_gen_state.cpu().numpy().tobytes().hex(), "perm_pos": self._perm_pos,
                         "gen": g.get_state().cpu().numpy().tobytes().hex()}
        return d

    def restore_stream_state(self, d) -> None:
        super().restore_stream_state(d)
        data = (d or {}).get("data")
        if data is None:
            return
        ds = self.dataset()
        if getattr(ds, "num_train", None) is None:
            return
        # the generator is created here only to receive the saved state: its seed draw must not advance the
        # just-restored explore rng (the uninterrupted run drew that seed rounds ago, before the saved rng state)
        rs = self.rng.getstate()
        g = self._data_gen(ds)
        self.rng.setstate(rs)
        if g is None:
            return
        st = lambda h: torch.frombuffer(bytearray(bytes.fromhex(h)), dtype=torch.uint8)  # noqa: E731
        g.set_state(st(data["perm_gen"]))
        self._perm_gen_state = g.get_state()
        self._perm = torch.randperm(ds.num_train, device=ds.train_x.device, generator=g)
        self._perm_pos = int(data["perm_pos"])
        g.set_state(st(data["gen"]))

    def _data_gen(self, ds, shared=None):
        """This member's own data-order / augmentation generator (seeded once from the member's rng): a member's
        batches do not depend on which members share its rank or plan, so a PBT run reads the same data at any
        placement of the population (tests/test_gpu_placement.py).  Replicas of a data-parallel group draw
        different shards."""
        if ds.device.type != "cuda":
            return shared
        g = getattr(self, "_gen", None)
        if g is None or g.device != ds.device:
            g = torch.Generator(device=ds.device)
            g.manual_seed(int(self.rng.random() * 1e9) + (7919 * self.dp.rank if self.dp else 0))
            self._gen = g
        return g

    def n_steps(self, num_epoch: int) -> int:
        """Steps of one ``train`` call: ``ready_steps`` when set (a fixed PBT ready interval in steps), else
        ``num_epoch`` epochs capped by ``max_train_steps``."""
        if self.ready_steps:
            return int(self.ready_steps)
        n = num_epoch * self.steps_per_epoch()
        if self.max_train_steps:
            n = min(n, int(self.max_train_steps))
        return max(1, n)

    def cycle_steps(self, num_epoch: int) -> List[int]:
        """Steps of each train -> eval cycle of one call.  The reference evaluates (and appends a CSV row, checks
        the stop threshold) after every ``epochs_between_evals`` epochs -- 1 in the PBT runs
        (``resnet_run_loop.py:446-508``: ``train_epochs // epochs_between_evals`` cycles; ``mnist_model.py:161-172``);
        with ``ready_steps`` the whole call is one cycle."""
        total = self.n_steps(num_epoch)
        ebe = self.epochs_between_evals
        if self.ready_steps or num_epoch <= ebe:
            return [total]
        per = ebe * self.steps_per_epoch()
        out = []
        for _ in range(num_epoch // ebe):
            n = min(per, total - sum(out))
            out.append(max(0, n))
        out[-1] += max(0, total - sum(out))  # a remainder of epochs (num_epoch % ebe) joins the last cycle
        return out

    @classmethod
    def _hooks(cls, eng, m):
        """Training hooks of this engine's population (``--hooks``; reference hooks_helper.get_train_hooks,
        resnet_run_loop.py:423-426), created once and kept across rounds."""
        hs = getattr(eng, "train_hooks", None)
        if hs is None:
            from ..utils.hooks import get_train_hooks
            names = m.options.get("hooks") or ""
            n = int(m.options.get("hook_every_n") or 100)
            pn = int(getattr(m, "probabilities_every_n", 0) or 0)
            if pn > 0 and "probabilities" not in names.lower():
                names = ",".join(x for x in (names, "probabilities") if x)  # MNIST default (mnist_model.py:149-151)
            hs = get_train_hooks(names, batch_size=int(m.hparams["batch_size"]), every_n_iter=n, every_n_steps=n,
                                 every_n_secs_steps=n, warm_steps=min(5, n), probabilities_every_n=pn or 50,
                                 model_dir=m.options.get("model_dir") or os.path.dirname(m.save_dir) or ".")
            for h in hs:
                h.begin()
            if any(getattr(h, "needs_probabilities", False) for h in hs) and hasattr(eng.backend, "keep_probs"):
                eng.backend.keep_probs = True  # before the first step: plans then keep the head's logits
            eng.train_hooks = hs
            eng.hook_step = 0
        return hs

    @classmethod
    def train_population(cls, members: List["EngineModel"], num_epoch: int, total_epochs: int):
        from ..utils.model_helpers import past_stop_threshold
        failed = {}
        groups: Dict[int, List[EngineModel]] = {}
        for m in members:
            groups.setdefault(id(m.engine), []).append(m)
        for ms in groups.values():
            eng = ms[0].engine
            ds = ms[0].dataset()
            gen = None  # each member draws from its own generator (_data_gen)
            hooks = cls._hooks(eng, ms[0])
            plan = {m.slot: m.cycle_steps(num_epoch) for m in ms}
            by_slot = {m.slot: m for m in ms}
            live = list(ms)  # members still training in this call (NaN / stop threshold end a member's call)
            for cycle in range(max(len(v) for v in plan.values())):
                todo = {m.slot: plan[m.slot][cycle] for m in live if cycle < len(plan[m.slot])}
                cyc = [by_slot[s] for s in todo]
                if not cyc:
                    break
                cls._train_cycle(eng, ds, gen, by_slot, todo, hooks)
                # eval of every finite member of this engine together (one batched forward per chunk)
                ev = [m for m in cyc if m.eval_every_round and math.isfinite(m.last_loss)]
                accs = {}
                if ev:
                    with timed_phase("eval"):
                        x, y = ms[0].dataset().eval_set()
                        accs = eng.evaluate_population([m.slot for m in ev], x, y)
                for m in cyc:
                    try:
                        m.end_cycle(accs.get(m.slot))
                    except Exception as e:  # member-level culling
                        failed[m.cluster_id] = e
                live = [m for m in cyc if m.cluster_id not in failed and math.isfinite(m.accuracy)
                        and not past_stop_threshold(m.stop_threshold, m.accuracy)]
            for m in ms:
                if m.cluster_id in failed:
                    continue
                try:
                    m.finish_round(num_epoch)
                except Exception as e:  # member-level culling
                    failed[m.cluster_id] = e
        return failed

    @classmethod
    def _train_cycle(cls, eng, ds, gen, by_slot, todo, hooks):
        """``todo[slot]`` population steps of every listed member (members drop out of the active set when their
        count is reached), then one readback of the members' last losses."""
        from ..utils.profiling import PHASES
        done = 0
        loss_acc = {s: None for s in todo}
        ms = [by_slot[s] for s in todo]
        t_enq = t_prep = 0.0  # host time enqueueing steps / preparing their inputs (metrics.jsonl phases_s)
        with timed_phase("train_steps"):
            while True:
                t0 = time.perf_counter()
                active = [s for s in sorted(todo) if todo[s] > done]
                if not active:
                    break
                batches = [by_slot[s]._batch(ds, gen) for s in active]
                hps = [by_slot[s].hparams for s in active]
                lrs = [by_slot[s].learning_rate(eng.host_step[s]) for s in active]
                t1 = time.perf_counter()
                losses = eng.train_step(active, batches, hps, lrs)
                t_enq += time.perf_counter() - t1
                t_prep += t1 - t0
                n_img = 0
                for i, s in enumerate(active):
                    b = datasets.batch_len(batches[i])
                    by_slot[s].images_trained += b
                    n_img += b
                    # a view (no host sync); a member's LAST step is copied: the view may be a LossRing row that later
                    # steps of the still-active members overwrite
                    loss_acc[s] = losses[i] if todo[s] > done + 1 else losses[i].clone()
                done += 1
                if hooks:
                    eng.hook_step += 1
                    cls._run_hooks(eng, hooks, [by_slot[s] for s in active], losses, lrs, n_img)
            dp = ms[0].dp
            if dp is not None:
                # same NaN verdict and the same BatchNorm running statistics on every replica
                eng.dp_sync_running([m.slot for m in ms])
                for m in ms:
                    if loss_acc[m.slot] is not None:
                        t = loss_acc[m.slot].detach().float().reshape(1).clone()
                        dp.allreduce_mean_(t)
                        loss_acc[m.slot] = t[0]
            present = [m for m in ms if loss_acc[m.slot] is not None]
            if present:
                # every member's last loss in one readback (also where the host waits for the queued steps)
                t2 = time.perf_counter()
                vals = torch.stack([loss_acc[m.slot].float().reshape(()) for m in present]).cpu().tolist()
                PHASES.total["train_drain"] += time.perf_counter() - t2
                for m, v in zip(present, vals):
                    m.last_loss = float(v)
        PHASES.total["host_step_enqueue"] += t_enq
        PHASES.total["host_step_prep"] += t_prep
        PHASES.total["train_step_count"] += done

    @staticmethod
    def _run_hooks(eng, hooks, active, losses, lrs, n_img):
        """Drive the step hooks; device values (cross entropy, train accuracy) are read back only when a hook
        wants this step (the reference's LoggingTensorHook every 100 steps)."""
        step = eng.hook_step
        due = [h for h in hooks if h.wants(step)]
        if not due:
            return
        host = {}

        def device_values():
            if not host:
                host["ce"] = losses.float().cpu().tolist()
                corr = getattr(eng.backend, "train_correct", None)
                c = corr([m.slot for m in active]) if corr is not None else None
                host["acc"] = None if c is None else [float(v) / max(1, int(m.hparams["batch_size"]))
                                                      for v, m in zip(c.cpu().tolist(), active)]
            return host

        def probabilities():
            fn = getattr(eng.backend, "train_probabilities", None)
            pr = fn([m.slot for m in active]) if fn is not None else None
            return None if pr is None else [None if t is None else t.cpu().numpy() for t in pr]

        values = _LazyValues(device_values, {"images": n_img, "model_ids": [m.cluster_id for m in active],
                                             "learning_rate": list(lrs), "sync": eng.device.type == "cuda"},
                             extra={"probabilities": probabilities})
        for h in due:
            h.after_step(step, values)

    def end_cycle(self, accuracy=None):
        """After one train -> eval cycle: accuracy, benchmark-logger eval record, a ``learning_curve.csv`` row."""
        if math.isnan(self.last_loss) or math.isinf(self.last_loss):
            self.accuracy = float("nan")
        elif accuracy is not None:
            self.accuracy = accuracy
        elif self.eval_every_round:
            x, y = self.dataset().eval_set()
            self.accuracy = self.engine.evaluate(self.slot, x, y)
        if not self.is_dp_follower:
            from ..utils.logger import get_benchmark_logger
            get_benchmark_logger().log_evaluation_result(
                {"accuracy": float(self.accuracy), "loss": float(self.last_loss), "global_step": int(self.global_step),
                 "model_id": int(self.cluster_id)})
        self.write_learning_curve(self.accuracy)

    def finish_round(self, num_epoch):
        self.epoches_trained += num_epoch
        if self.checkpoint_every_round:
            with timed_phase("checkpoint"):
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
