"""``TrainingWorker``: hosts this rank's population members.

Compatible with reference ``training_worker.py:12-105`` (instruction loop,
``add_graphs``, ``train``, ``get_all_values``, ``set_values``,
``explore_necessary_graphs``, NaN / exception culling, train / explore timers).

Differences (MI355X-first):
  * ``train`` hands ALL resident members to ``target_model_class.train_population``
    so a model family can run them together on the GPU (population-batched
    kernels) instead of one after another;
  * exploit weight copies arrive over the data plane (RCCL send/recv or an
    on-device copy), not through ``cp`` on a shared filesystem; the reference's
    file-copy path is still available (``exploit_transport="files"``).
"""

from __future__ import annotations

import math
import shutil
import time
from typing import Any, Dict, List, Optional

from .hparams import WorkerInstruction


from ..models.model_base import flush_checkpoints

class TrainingWorker:
    def __init__(self, comm, master_rank: int, target_model_class, save_base_dir: str = "./savedata/model_",
                 seed: Optional[int] = None, model_kwargs: Optional[Dict[str, Any]] = None,
                 dataplane=None, verbose: bool = True):
        self.worker_graphs: List[Any] = []
        self.is_expolore_only = False
        self.comm = comm
        self.rank = comm.Get_rank()
        self.master_rank = master_rank
        self.target_model_class = target_model_class
        self.save_base_dir = save_base_dir
        self.seed = seed
        self.model_kwargs = dict(model_kwargs or {})
        self.dataplane = dataplane
        self.verbose = verbose
        self.train_time = 0.0
        self.explore_time = 0.0
        self.removed_ids: List[int] = []
        self.reseed_dead = False  # SPMD --reseed_dead: NaN members stay and are re-seeded at the next exploit

    def log(self, *a):
        if self.verbose:
            print(*a, flush=True)

    # ------------------------------------------------------ reference protocol
    def _handle_add(self, d):
        """(ADD_GRAPHS, hparams, begin[, explore_only[, reseed_dead]]) -- the trailing fields are extensions."""
        if len(d) > 4:
            self.reseed_dead = bool(d[4])
        self.add_graphs(d[1], d[2], d[3] if len(d) > 3 else False)

    def main_loop(self):
        handlers = {
            WorkerInstruction.ADD_GRAPHS: lambda d: self._handle_add(d),
            WorkerInstruction.TRAIN: lambda d: self.train(d[1], d[2]),
            WorkerInstruction.GET: lambda d: self.comm.send(self.get_all_values(), self.master_rank),
            WorkerInstruction.SET: lambda d: self._handle_set(d),
            WorkerInstruction.EXPLORE: lambda d: self.explore_necessary_graphs(),
            WorkerInstruction.GET_PROFILING_INFO: lambda d: self.comm.send(
                [self.train_time, self.explore_time], self.master_rank),
        }
        while True:
            data = self.comm.recv(self.master_rank)
            inst = data[0]
            if inst == WorkerInstruction.EXIT:
                break
            handler = handlers.get(inst)
            if handler is None:
                self.log("Invalid instruction!!!!")
                continue
            handler(data)

    def _handle_set(self, data):
        values = data[1]
        transfers = data[2] if len(data) > 2 else None
        reload_from_disk = data[3] if len(data) > 3 else False
        if transfers and self.dataplane is not None:
            self.dataplane.execute(transfers, self.members_by_id())
        self.set_values(values, reload_from_disk=reload_from_disk)

    # ------------------------------------------------------------- operations
    def members_by_id(self) -> Dict[int, Any]:
        return {g.cluster_id: g for g in self.worker_graphs}

    def add_graphs(self, hparam_list, id_begin, is_explore_only: bool = False):
        self.is_expolore_only = bool(is_explore_only)
        self.log("[{}]Got {} hparams".format(self.rank, len(hparam_list)))
        for i, hp in enumerate(hparam_list):
            g = self.target_model_class(id_begin + i, hp, self.save_base_dir, seed=self.seed, **self.model_kwargs)
            self.worker_graphs.append(g)

    def add_members(self, id_hparams):
        """Instantiate members with explicit ids (whole-run resume: ids need not be contiguous)."""
        for mid, hp in id_hparams:
            self.worker_graphs.append(self.target_model_class(int(mid), hp, self.save_base_dir, seed=self.seed,
                                                              **self.model_kwargs))

    def _cull(self, g, why: str):
        flush_checkpoints()  # no pending write may recreate the directory removed below
        self.worker_graphs.remove(g)
        self.removed_ids.append(g.cluster_id)
        shutil.rmtree(self.save_base_dir + str(g.cluster_id), ignore_errors=True)
        release = getattr(g, "release", None)
        if release is not None:
            release()
        self.log("Error occured , graph {} removed ({})".format(g.cluster_id, why))

    def train(self, num_epoches, total_epochs):
        t0 = time.time()
        if self.worker_graphs:
            failed = self.target_model_class.train_population(list(self.worker_graphs), num_epoches, total_epochs)
            for g in list(self.worker_graphs):
                if g.cluster_id in failed:
                    self._cull(g, repr(failed[g.cluster_id]))
                    continue
                self.log("Model {} epoch = {},  acc = {}".format(g.cluster_id, g.epoches_trained, g.get_accuracy()))
                acc = g.get_accuracy()
                if (acc is None or (isinstance(acc, float) and math.isnan(acc))) and not self.reseed_dead:
                    self._cull(g, "nan accuracy")
        self.train_time += time.time() - t0

    def get_all_values(self):
        # GET is the end-of-train barrier of the reference protocol: checkpoints are on disk before the master
        # may copy member directories (exploit_transport="files")
        flush_checkpoints()
        return [g.get_values() for g in self.worker_graphs]

    def set_values(self, values_to_set, reload_from_disk: bool = False):
        by_id = self.members_by_id()
        for v in values_to_set:
            g = by_id.get(int(v[0]))
            if g is None:
                continue
            g.set_values(v)
            if reload_from_disk:
                g.load_checkpoint()
            g.need_explore = True

    def explore_necessary_graphs(self):
        t0 = time.time()
        for g in self.worker_graphs:
            if g.need_explore or self.is_expolore_only:
                self.log("[{}]Exploring graph {}".format(self.rank, g.cluster_id))
                g.perturb_hparams()
                on_change = getattr(g, "on_hparams_changed", None)
                if on_change is not None:
                    on_change()
                g.need_explore = False
        self.explore_time += time.time() - t0
