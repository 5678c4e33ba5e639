"""Tracing / profiling helpers.

* ``Timer`` / ``PhaseTimers`` -- wall-clock accumulators for the PBT phases
  (train / exploit / explore per rank, reference ``training_worker.py:21-22``,
  ``pbt_cluster.py:36,130,166``);
* ``GpuStepTimer`` -- HIP-event timing of device work without a sync per step;
* ``roctx_range`` -- named ranges visible in rocprofv3 ``--marker-trace`` when
  ``libroctx64.so`` is present (no-op otherwise).
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        for p in ("/opt/rocm/lib/libroctx64.so", "libroctx64.so"):
            try:
                lib = ctypes.CDLL(p)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                _ROCTX = lib
                break
            except OSError:
                continue
    return _ROCTX or None


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _roctx() if os.environ.get("DTF_ROCTX", "0") == "1" else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


class PhaseTimers:
    def __init__(self):
        self.total = defaultdict(float)
        self.count = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        t0 = time.perf_counter()
        with roctx_range(name):
            try:
                yield
            finally:
                self.total[name] += time.perf_counter() - t0
                self.count[name] += 1

    def summary(self):
        return {k: {"seconds": v, "calls": self.count[k]} for k, v in self.total.items()}

    def snapshot(self):
        return dict(self.total)

    def since(self, snap):
        """Seconds per phase accumulated after ``snapshot()`` returned ``snap``."""
        return {k: v - snap.get(k, 0.0) for k, v in self.total.items() if v - snap.get(k, 0.0) > 0.0}


# Process-wide phase timers of the member-level work inside a PBT round (train steps, eval, checkpoint writes,
# hooks); the round loop reports their per-round deltas in metrics.jsonl.
PHASES = PhaseTimers()


def timed_phase(name: str):
    return PHASES.phase(name)


class GpuStepTimer:
    """Records a HIP event pair around each step; resolves lazily (no per-step sync)."""

    def __init__(self):
        import torch
        self.torch = torch
        self.pairs = []

    @contextlib.contextmanager
    def step(self):
        t = self.torch
        a, b = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        a.record()
        yield
        b.record()
        self.pairs.append((a, b))

    def millis(self):
        self.torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in self.pairs]
