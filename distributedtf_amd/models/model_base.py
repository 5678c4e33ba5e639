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

import atexit
import copy
import os
import queue
import random
import threading
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

    # PBT round whose state the next checkpoint holds (set by the round loop); None: untagged
    ckpt_round: Optional[int] = None
    # the TF tensor bundle (``--tf_checkpoint``) owns the ``checkpoint`` state file when set
    tf_checkpoint = False

    def stream_state(self):
        """JSON-able state of the member's random streams (the explore rng), saved in the whole-run resume table
        so a resumed run draws the same perturbations as an uninterrupted one."""
        v, st, gauss = self.rng.getstate()
        return {"rng": [v, list(st), gauss]}

    def restore_stream_state(self, d) -> None:
        if d and "rng" in d:
            v, st, gauss = d["rng"]
            self.rng.setstate((v, tuple(st), gauss))

    def save_checkpoint(self, wait: bool = False) -> None:
        """Write ``savedata/model_<id>/model.ckpt`` (+ ``checkpoint`` state file).

        With a round tag (``ckpt_round``) the file is ``model.ckpt-r<round>`` and ``model.ckpt`` is a hard link to
        it; the last two rounds are kept, so a whole-run resume can load exactly the round the population table
        names even when a crash left some members one round ahead (``load_checkpoint(round_tag=...)``).
        The state leaves the GPU through one device->host copy into a pinned buffer (ordered on the current
        stream, so training can continue immediately); serialisation and the file write run on the background
        ``CheckpointWriter`` thread.  ``wait=True`` (or ``flush_checkpoints()``) blocks
        until the file is on disk."""
        d = self.ensure_save_dir()
        blob = {"epoches_trained": self.epoches_trained, "hparams": copy.deepcopy(self.hparams),
                "round": self.ckpt_round}
        CheckpointWriter.get().submit(self.export_state().detach(), blob, d, tag=self.ckpt_round,
                                      state_file=not self.tf_checkpoint)
        if wait:
            flush_checkpoints()

    def tf_variables(self) -> Dict[str, Any]:
        """name -> numpy array under the reference's TF1 variable names (families that map onto TF layers)."""
        raise NotImplementedError("%s has no TensorFlow variable mapping" % type(self).__name__)

    def export_tf_checkpoint(self, directory: Optional[str] = None) -> str:
        """Write the member in the reference's on-disk format: a TF tensor bundle ``model.ckpt-<step>.index`` /
        ``.data-00000-of-00001`` (byte-compatible with TF 1.x ``Saver``; utils/tf_bundle.py) plus the
        ``checkpoint`` state file naming it.  Returns the checkpoint prefix."""
        from ..utils.tf_bundle import write_bundle
        flush_checkpoints()
        d = directory or self.ensure_save_dir()
        tensors = self.tf_variables()
        step = int(tensors["global_step"]) if "global_step" in tensors else 0
        prefix = os.path.join(d, "model.ckpt-%d" % step)
        write_bundle(prefix, tensors)
        with open(os.path.join(d, "checkpoint"), "w") as f:
            f.write('model_checkpoint_path: "model.ckpt-%d"\nall_model_checkpoint_paths: "model.ckpt-%d"\n'
                    % (step, step))
        return prefix

    def has_checkpoint(self) -> bool:
        flush_checkpoints()
        return os.path.isfile(os.path.join(self.save_dir, "model.ckpt"))

    def load_checkpoint(self, round_tag: Optional[int] = None) -> bool:
        """Load ``model.ckpt`` (latest) or, with ``round_tag``, exactly ``model.ckpt-r<round_tag>``."""
        import torch
        flush_checkpoints()  # a pending write of this member must land first
        name = "model.ckpt" if round_tag is None else "model.ckpt-r%d" % int(round_tag)
        path = os.path.join(self.save_dir, name)
        if not os.path.isfile(path):
            return False
        blob = torch.load(path, map_location="cpu", weights_only=True)
        self.import_state(blob["state"])
        return True


class CheckpointWriter:
    """One background thread per process that writes member checkpoints.

    ``submit`` snapshots the state into a pinned host buffer with a non-blocking copy and records a GPU
    event; the thread waits for that event, then ``torch.save``s the blob and writes the TF-style
    ``checkpoint`` state file.  Writes of one directory stay in submission order (single thread)."""

    _inst: Optional["CheckpointWriter"] = None
    _lock = threading.Lock()

    def __init__(self):
        self.q: "queue.Queue" = queue.Queue()
        self.error: Optional[BaseException] = None
        self.t = threading.Thread(target=self._run, name="dtf-ckpt-writer", daemon=True)
        self.t.start()
        atexit.register(self.q.join)  # the daemon thread finishes pending writes before the interpreter exits

    @classmethod
    def get(cls) -> "CheckpointWriter":
        with cls._lock:
            if cls._inst is None:
                cls._inst = CheckpointWriter()
            return cls._inst

    def submit(self, state, blob: Dict[str, Any], directory: str, tag: Optional[int] = None,
               state_file: bool = True) -> None:
        import torch
        if state.is_cuda:
            host = torch.empty(state.shape, dtype=state.dtype, pin_memory=True)
            host.copy_(state, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = state.clone(), None
        # the cwd may change before the write: absolute directory
        self.q.put((host, ev, blob, os.path.abspath(directory), tag, state_file))

    @staticmethod
    def _write(host, blob, d, tag, state_file):
        import torch
        blob = dict(blob)
        blob["state"] = host
        tmp = os.path.join(d, "model.ckpt.tmp")
        torch.save(blob, tmp)
        latest = os.path.join(d, "model.ckpt")
        if tag is None:
            os.replace(tmp, latest)
        else:
            tagged = os.path.join(d, "model.ckpt-r%d" % int(tag))
            os.replace(tmp, tagged)
            link = os.path.join(d, "model.ckpt.lnk")
            try:
                if os.path.lexists(link):
                    os.remove(link)
                os.link(tagged, link)
            except OSError:  # no hard links on this filesystem: copy
                import shutil
                shutil.copyfile(tagged, link)
            os.replace(link, latest)
            for f in os.listdir(d):  # keep this round and the previous one
                if f.startswith("model.ckpt-r") and f[len("model.ckpt-r"):].isdigit() \
                        and int(f[len("model.ckpt-r"):]) < int(tag) - 1:
                    os.remove(os.path.join(d, f))
        if state_file:
            with open(os.path.join(d, "checkpoint"), "w") as f:
                f.write('model_checkpoint_path: "model.ckpt"\n')

    def _run(self):
        while True:
            item = self.q.get()
            try:
                host, ev, blob, d, tag, state_file = item
                if ev is not None:
                    ev.synchronize()
                self._write(host, blob, d, tag, state_file)
            except BaseException as e:  # surfaced by flush()
                self.error = e
            finally:
                self.q.task_done()

    def flush(self) -> None:
        self.q.join()
        if self.error is not None:
            e, self.error = self.error, None
            raise RuntimeError("checkpoint write failed") from e


def flush_checkpoints() -> None:
    """Block until every submitted checkpoint is on disk (no-op when nothing was written)."""
    if CheckpointWriter._inst is not None:
        CheckpointWriter._inst.flush()
