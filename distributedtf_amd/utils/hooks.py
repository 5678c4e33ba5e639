"""Training-step hooks and the hook registry.

Reference: ``official/utils/logs/hooks.py`` (ExamplesPerSecondHook),
``hooks_helper.py`` (name -> factory registry: LoggingTensorHook every 100
steps for lr / cross_entropy / train_accuracy, ProfilerHook chrome trace every
1000 steps, ExamplesPerSecondHook, LoggingMetricHook) and ``metric_hook.py``.

Hooks here are plain Python objects driven by the population training loop:
``begin()``, ``after_step(step, values)`` (values: dict of host scalars such as
``lr``, ``cross_entropy``, ``train_accuracy``, ``images``), ``end()``.  Host
values are only materialised on logging steps, so hooks never add a device sync
to ordinary steps.
"""

from __future__ import annotations

import json
import os
import time
from typing import Any, Callable, Dict, List, Optional

from .logger import get_benchmark_logger, log

_TENSORS_TO_LOG = ("learning_rate", "cross_entropy", "train_accuracy")


class StepHook:
    every_n_steps = 1

    def begin(self):
        pass

    def wants(self, step: int) -> bool:
        return self.every_n_steps and step % self.every_n_steps == 0

    def after_step(self, step: int, values: Dict[str, Any]):
        pass

    def end(self):
        pass


class ExamplesPerSecondHook(StepHook):
    """Average and current examples/sec after ``warm_steps`` (the north-star metric)."""

    def __init__(self, batch_size: int, every_n_steps: Optional[int] = None, every_n_secs: Optional[float] = None,
                 warm_steps: int = 0, metric_logger=None):
        if (every_n_steps is None) == (every_n_secs is None):
            raise ValueError("exactly one of every_n_steps and every_n_secs should be provided.")
        self.batch_size = batch_size
        self.every_n_steps = every_n_steps
        self.every_n_secs = every_n_secs
        self.warm_steps = warm_steps
        self.logger = metric_logger or get_benchmark_logger()
        self.total_steps = 0
        self.total_time = 0.0
        self.total_images = 0
        self._images = 0  # since the last report
        self._last_t = None
        self._last_step = None
        self.current = None
        self.average = None

    def wants(self, step):
        return True

    def begin(self):
        self._last_t = time.perf_counter()
        self._last_step = 0

    def after_step(self, step, values=None):
        """``values["images"]``: images of this step (a population step trains every active member's batch;
        default ``batch_size``); ``values["sync"]``: drain the device before reading the clock on report steps
        (steps are queued asynchronously, so host time alone would count queueing, not work)."""
        values = values or {}
        if step <= self.warm_steps:
            self._last_t = time.perf_counter()
            self._last_step = step
            self._images = 0
            return
        self._images += int(values.get("images", self.batch_size))
        nsteps = step - self._last_step
        if self.every_n_steps and nsteps < self.every_n_steps:
            return
        if values.get("sync"):
            import torch
            torch.cuda.synchronize()
        now = time.perf_counter()
        elapsed = now - self._last_t
        if not self.every_n_steps and elapsed < self.every_n_secs:
            return
        self.total_steps += nsteps
        self.total_time += elapsed
        self.total_images += self._images
        self.current = self._images / elapsed if elapsed > 0 else 0.0
        self.average = self.total_images / self.total_time if self.total_time > 0 else 0.0
        self._images = 0
        self.logger.log_metric("average_examples_per_sec", self.average, global_step=step)
        self.logger.log_metric("current_examples_per_sec", self.current, global_step=step)
        self._last_t, self._last_step = now, step


class LoggingHook(StepHook):
    """LoggingTensorHook equivalent: prints selected scalars every N steps."""

    def __init__(self, tensors=_TENSORS_TO_LOG, every_n_steps: int = 100, printer: Callable = None):
        self.tensors = tuple(tensors)
        self.every_n_steps = every_n_steps
        self.printer = printer or (lambda s: print(s, flush=True))
        self.records: List[Dict[str, Any]] = []

    def after_step(self, step, values):
        rec = {k: values[k] for k in self.tensors if k in values}
        ids = values.get("model_ids")
        rec["step"] = step
        self.records.append(rec)
        if ids is None:
            self.printer(", ".join("%s = %s" % (k, rec[k]) for k in rec))
            return
        # population step: one line per member (each value is a per-member list)
        for i, mid in enumerate(ids):
            self.printer("step = %d, model_id = %d, " % (step, mid) +
                         ", ".join("%s = %.6g" % (k, rec[k][i]) for k in self.tensors if k in rec))


class LoggingMetricHook(LoggingHook):
    """Routes the same scalars to the benchmark logger (metric.log)."""

    def __init__(self, tensors=_TENSORS_TO_LOG, every_n_steps: int = 100, metric_logger=None):
        super().__init__(tensors, every_n_steps)
        self.logger = metric_logger or get_benchmark_logger()

    def after_step(self, step, values):
        ids = values.get("model_ids")
        for k in self.tensors:
            if k not in values:
                continue
            v = values[k]
            if ids is None:
                self.logger.log_metric(k, float(v), global_step=step)
            else:
                for mid, x in zip(ids, v):
                    self.logger.log_metric(k, float(x), global_step=step, extras={"model_id": mid})


class ProbabilitiesHook(StepHook):
    """The MNIST ``LoggingTensorHook(tensors={"probabilities": "softmax_tensor"}, every_n_iter=50)`` of the reference
    (``mnist_model.py:149-151``): every ``every_n_steps`` steps, each member's softmax over its last training batch
    (dropout on, as in the reference's training graph) is printed -- numpy's summarised repr, as TF prints a tensor.
    The backend keeps the logits only while this hook is registered (one [batch, 10] fp32 store in the head kernel);
    they are read back on logging steps only."""

    needs_probabilities = True

    def __init__(self, every_n_steps: int = 50, printer: Callable = None):
        self.every_n_steps = every_n_steps
        self.printer = printer or (lambda s: print(s, flush=True))
        self.records: List[Dict[str, Any]] = []

    def after_step(self, step, values):
        probs = values.get("probabilities")
        ids = values.get("model_ids") or [None]
        if probs is None:
            return
        if not isinstance(probs, list):
            probs = [probs]
        for mid, pr in zip(ids, probs):
            if pr is None:
                continue
            self.records.append({"step": step, "model_id": mid, "probabilities": pr})
            head = "step = %d, " % step + ("model_id = %d, " % mid if mid is not None else "")
            self.printer(head + "probabilities = %s" % (pr,))


class ProfilerHook(StepHook):
    """Chrome-trace window every ``save_steps`` steps via ``torch.profiler``.

    The trace includes the HIP kernels (CUPTI-equivalent roctracer activity on
    ROCm).  For kernel counters use rocprofv3 on the whole run instead.
    """

    def __init__(self, save_steps: int = 1000, output_dir: str = ".", window: int = 2):
        self.every_n_steps = save_steps
        self.output_dir = output_dir
        self.window = window
        self._prof = None
        self._stop_at = None
        self.traces: List[str] = []

    def wants(self, step):
        return True

    def after_step(self, step, values=None):
        if self._prof is not None and step >= self._stop_at:
            self._prof.__exit__(None, None, None)
            path = os.path.join(self.output_dir, "timeline-%d.json" % step)
            self._prof.export_chrome_trace(path)
            self.traces.append(path)
            self._prof = None
        elif self._prof is None and step % self.every_n_steps == 0:
            import torch
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts)
            self._prof.__enter__()
            self._stop_at = step + self.window

    def end(self):
        if self._prof is not None:
            self._prof.__exit__(None, None, None)
            self._prof = None


def _logging(**kw):
    return LoggingHook(every_n_steps=kw.get("every_n_iter", 100), printer=kw.get("printer"))


def _probabilities(**kw):
    return ProbabilitiesHook(every_n_steps=kw.get("probabilities_every_n", 50), printer=kw.get("printer"))


def _profiler(**kw):
    return ProfilerHook(save_steps=kw.get("save_steps", 1000), output_dir=kw.get("model_dir", "."))


def _eps(**kw):
    return ExamplesPerSecondHook(batch_size=kw.get("batch_size", 128), every_n_steps=kw.get("every_n_steps", 100),
                                 warm_steps=kw.get("warm_steps", 5))


def _metric(**kw):
    return LoggingMetricHook(every_n_steps=kw.get("every_n_secs_steps", 100))


HOOKS = {
    "loggingtensorhook": _logging,
    "logging": _logging,
    "profilerhook": _profiler,
    "profiler": _profiler,
    "examplespersecondhook": _eps,
    "examples_per_second": _eps,
    "loggingmetrichook": _metric,
    "metric": _metric,
    "probabilities": _probabilities,
}


def get_train_hooks(name_list, **kwargs) -> List[StepHook]:
    """Build hooks by (case-insensitive) name; unknown names raise ValueError."""
    if not name_list:
        return []
    if isinstance(name_list, str):
        name_list = [n for n in name_list.split(",") if n.strip()]
    out = []
    for name in name_list:
        key = name.strip().lower()
        if key not in HOOKS:
            raise ValueError("Unrecognized training hook requested: {}".format(name))
        out.append(HOOKS[key](**kwargs))
    return out
