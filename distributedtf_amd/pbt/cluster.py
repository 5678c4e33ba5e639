"""PBT control plane.

Two drivers share the worker, the exploit planner and the report writers:

``PBTCluster`` -- reference-compatible master (``pbt_cluster.py:27-470``).  Rank
``master_rank`` owns the population and drives ``TrainingWorker.main_loop`` on
the other ranks with the ``WorkerInstruction`` protocol (ADD_GRAPHS / TRAIN /
GET / SET / EXPLORE / GET_PROFILING_INFO / EXIT).  The master trains nothing.
Exploit weight copies go over the data plane between the two worker ranks
(``exploit_transport="dataplane"``, default) or through the shared filesystem
exactly like the reference (``"files"``).

``SPMDPopulation`` -- the MI355X-native driver: every rank (one per GPU) trains
its slice of the population; scores are all-gathered and every rank computes
the same exploit plan, so there is no idle master and no SET / EXPLORE traffic;
weights move GPU->GPU over RCCL (or D2D when winner and loser share a GPU).
"""

from __future__ import annotations

import copy
import datetime
import math
import os
import random
import shutil
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

from .exploit import apply_plan_to_values, plan_exploit, plan_reseed
from .hparams import WorkerInstruction, generate_random_hparam
from . import reports
from ..models.model_base import flush_checkpoints
from ..utils.profiling import roctx_range


def partition(pop_size: int, n_slots: int) -> List[Tuple[int, int]]:
    """Contiguous id blocks of ``ceil(pop / n)`` per slot (``pbt_cluster.py:56,66-75``).

    Returns ``[(begin, count), ...]`` of length ``n_slots``; trailing slots may be
    empty when ``pop < n`` (Appendix A15 handled explicitly).
    """
    if n_slots <= 0:
        raise ValueError("need at least one slot")
    per = int(math.ceil(pop_size / float(n_slots))) if pop_size else 0
    out, begin, left = [], 0, pop_size
    for _ in range(n_slots):
        cnt = max(0, min(per, left))
        out.append((begin, cnt))
        begin += cnt
        left -= cnt
    return out


def sample_population(pop_size: int, seed: Optional[int] = None) -> List[Dict[str, Any]]:
    import random
    rng = random.Random(seed) if seed is not None else random
    return [generate_random_hparam(rng) for _ in range(pop_size)]


EXCLUDE_ON_COPY = ("learning_curve.csv", "theta.csv")


def _excluded(name: str) -> bool:
    return name in EXCLUDE_ON_COPY or name.startswith("events.out") or name.startswith(".nfs")


def copy_member_files(src_dir: str, dest_dir: str) -> bool:
    """Reference ``copyfiles`` rules: replace dest's checkpoint files by src's,
    keeping dest's own learning curves / event files."""
    if os.path.abspath(src_dir) == os.path.abspath(dest_dir):
        print("Warning, src_dir and dest_dir are the same")
        return False
    os.makedirs(dest_dir, exist_ok=True)
    for name in os.listdir(dest_dir):
        p = os.path.join(dest_dir, name)
        if os.path.isfile(p) and not _excluded(name):
            os.remove(p)
    if os.path.isdir(src_dir):
        for name in os.listdir(src_dir):
            p = os.path.join(src_dir, name)
            if os.path.isfile(p) and not _excluded(name):
                shutil.copy2(p, dest_dir)
    return True


class _ReportMixin:
    savedata = "savedata"
    do_exploit = True
    do_explore = True

    def dump_all_models_to_json(self, filename):
        reports.dump_population_json(self.get_all_values(), filename)
        print("Saving all models to {}".format(filename))

    def report_best_model(self):
        path = os.path.join(self.savedata, "best_model.json")
        rep = reports.write_best_model(self.get_all_values(), path)
        print("Saving best model to {}".format(path))
        return rep

    def export_best_model(self, export_dir):
        """``--export_dir`` in master/worker mode: the master owns no member, so it exports the best member's
        flushed checkpoint from the shared savedata (``model.ckpt`` + ``model.json`` metadata)."""
        import json
        import shutil
        vals = self.get_all_values()
        if not vals:
            return None
        best = reports.best_member(vals)
        os.makedirs(export_dir, exist_ok=True)
        src = os.path.join(self.savedata, "model_%d" % int(best[0]), "model.ckpt")
        if os.path.isfile(src):
            shutil.copyfile(src, os.path.join(export_dir, "model.ckpt"))
        with open(os.path.join(export_dir, "model.json"), "w") as f:
            json.dump({"model_id": int(best[0]), "accuracy": float(best[1]), "hparams": best[2]}, f, indent=2,
                      sort_keys=True)
        return export_dir

    def report_plot_for_toy_model(self):
        return reports.plot_toy(self.savedata, self.do_exploit, self.do_explore)

    def report_accuracy_plot(self):
        return reports.plot_curves(self.savedata, "acc", self.do_exploit, self.do_explore)

    def report_lr_plot(self):
        return reports.plot_curves(self.savedata, "lr", self.do_exploit, self.do_explore)

    def report_best3_plot(self):
        return reports.plot_best3(self.savedata, self.do_exploit, self.do_explore)


class PBTCluster(_ReportMixin):
    """Reference-compatible master (runs on ``master_rank`` only)."""

    def __init__(self, pop_size, comm, master_rank, epochs_per_round, do_exploit=True, do_explore=True,
                 seed=None, exploit_transport="dataplane", savedata="savedata", hparams=None, reseed_dead=False):
        self.pop_size = pop_size
        self.reseed_dead = bool(reseed_dead)  # workers learn it with ADD_GRAPHS (keep NaN members for re-seeding)
        self.comm = comm
        self.master_rank = master_rank
        self.epochs_per_round = epochs_per_round
        self.do_exploit = do_exploit
        self.do_explore = do_explore
        self.exploit_transport = exploit_transport
        self.savedata = savedata
        self.seed = seed
        self.exploit_time = 0.0
        self.round_times: List[float] = []
        self.last_plan = []
        self._initial_hparams = hparams
        self.dispatch_hparams_to_workers()

    def workers(self) -> List[int]:
        return [r for r in range(self.comm.Get_size()) if r != self.master_rank]

    def _bcast(self, msg, ranks=None):
        for r in (self.workers() if ranks is None else ranks):
            self.comm.isend(msg, r).wait()

    def dispatch_hparams_to_workers(self):
        hps = self._initial_hparams or sample_population(self.pop_size, self.seed)
        self.pop_size = len(hps)
        print("Population size = {}".format(self.pop_size))
        explore_only = self.do_explore and not self.do_exploit
        ws = self.workers()
        self.id_owner: Dict[int, int] = {}
        for r, (begin, cnt) in zip(ws, partition(self.pop_size, len(ws))):
            self.comm.isend((WorkerInstruction.ADD_GRAPHS, hps[begin:begin + cnt], begin, explore_only,
                             self.reseed_dead), r).wait()
            for i in range(begin, begin + cnt):
                self.id_owner[i] = r

    def kill_all_workers(self):
        self._bcast((WorkerInstruction.EXIT,))

    def train(self, round_num):
        start = time.time()
        for rnd in range(round_num):
            t0 = time.time()
            print("\nRound {}".format(rnd))
            self._bcast((WorkerInstruction.TRAIN, self.epochs_per_round, self.epochs_per_round * round_num))
            if self.do_exploit:
                self.exploit()
            if self.do_explore:
                self.explore()
            self.round_times.append(time.time() - t0)
            print("Round elapsed time: {}\n".format(datetime.timedelta(seconds=self.round_times[-1])))
        self.flush_all_instructions()
        total = time.time() - start
        print("Total elapsed time: {}".format(datetime.timedelta(seconds=total)))
        return total

    def _gather(self):
        self._bcast((WorkerInstruction.GET,))
        values, owner = [], {}
        for r in self.workers():
            data = self.comm.recv(r)
            values += data
            for d in data:
                owner[int(d[0])] = r
        return values, owner

    def exploit(self):
        values, owner = self._gather()  # the recv is the end-of-TRAIN barrier
        t0 = time.time()
        self.pop_size = len(values)
        plan = plan_reseed(values) if getattr(self, "reseed_dead", False) else plan_exploit(values)
        self.last_plan = plan
        updates = apply_plan_to_values(values, plan)
        per_rank: Dict[int, list] = {r: [] for r in self.workers()}
        transfers = []
        for p in plan:
            print("Copied: {} -> {}".format(p.src_id, p.dst_id))
            per_rank[owner[p.dst_id]].append(updates[p.dst_id])
            if self.exploit_transport == "files":
                copy_member_files(os.path.join(self.savedata, "model_%d" % p.src_id),
                                  os.path.join(self.savedata, "model_%d" % p.dst_id))
            else:
                transfers.append((p.src_id, owner[p.src_id], p.dst_id, owner[p.dst_id]))
        from_disk = self.exploit_transport == "files"
        involved = set(per_rank) if transfers else {r for r, v in per_rank.items() if v}
        for r in self.workers():
            if r in involved or per_rank[r]:
                self.comm.isend((WorkerInstruction.SET, per_rank[r], transfers, from_disk), r).wait()
        self.exploit_time += time.time() - t0

    def explore(self):
        self._bcast((WorkerInstruction.EXPLORE,))

    def flush_all_instructions(self):
        self.get_all_values()

    def get_all_values(self):
        return self._gather()[0]

    def get_profiling_info(self):
        self._bcast((WorkerInstruction.GET_PROFILING_INFO,))
        return [self.comm.recv(r) for r in self.workers()]

    def print_profiling_info(self):
        infos = self.get_profiling_info()
        n = max(1, len(infos))
        tr = sum(i[0] for i in infos) / n
        ex = sum(i[1] for i in infos) / n
        print("")
        print("=======Profiling Information========")
        print("Total train time: {}".format(datetime.timedelta(seconds=tr)))
        print("Total exploit time: {}".format(datetime.timedelta(seconds=self.exploit_time)))
        print("Total explore time: {}\n".format(datetime.timedelta(seconds=ex)))
        return {"train": tr, "exploit": self.exploit_time, "explore": ex}


class SPMDPopulation(_ReportMixin):
    """Every rank trains; exploit plans are computed identically everywhere."""

    def __init__(self, pop_size, comm, target_model_class, epochs_per_round=1, do_exploit=True, do_explore=True,
                 seed=None, savedata="savedata", model_kwargs=None, dataplane=None, hparams=None,
                 verbose=True, inject_nan=None, resume=False, dp_size=1, reseed_dead=False):
        from .worker import TrainingWorker
        self.comm = comm
        self.rank = comm.Get_rank()
        self.world = comm.Get_size()
        self.epochs_per_round = epochs_per_round
        self.do_exploit = do_exploit
        self.do_explore = do_explore
        self.savedata = savedata
        self.verbose = verbose
        self.exploit_time = 0.0
        self.round_times: List[float] = []
        self.inject_nan = inject_nan or {}  # {round: [member ids]} fault injection
        if dataplane is None:
            from ..parallel.dataplane import DataPlane
            dataplane = DataPlane(comm)
        self.dataplane = dataplane
        # intra-member data parallelism (parallel/dataparallel.py): world / dp_size member groups
        from ..parallel.dataparallel import make_dp_context
        self.dp_size = max(1, int(dp_size))
        self.dp = make_dp_context(comm, self.dp_size)
        self.group_index = self.rank // self.dp_size
        self.n_groups = self.world // self.dp_size
        if self.dp is not None:
            if seed is None:  # replicas must draw identical inits and explore steps
                seed = comm.bcast(random.randrange(1 << 30) if self.rank == 0 else None, 0)
            model_kwargs = dict(model_kwargs or {}, dp=self.dp)
        self.worker = TrainingWorker(comm, 0, target_model_class, save_base_dir=os.path.join(savedata, "model_"),
                                     seed=seed, model_kwargs=model_kwargs, dataplane=dataplane, verbose=verbose)
        self.worker.reseed_dead = bool(reseed_dead)
        self.reseed_dead = bool(reseed_dead)
        self.start_round = 0
        state = None
        if resume:
            ok = os.path.isfile(os.path.join(savedata, reports.POPULATION_STATE)) if self.rank == 0 else None
            if comm.bcast(ok, 0):
                state = comm.bcast(reports.read_population_state(savedata) if self.rank == 0 else None, 0)
        if state is None:
            hps = hparams if hparams is not None else (
                sample_population(pop_size, seed) if self.rank == 0 else None)
            hps = comm.bcast(hps, 0)
            self.initial_pop_size = len(hps)
            rows = [(i, None, hp, 0) for i, hp in enumerate(hps)]
        else:
            # whole-run resume: surviving members keep their ids (and owners); state from their checkpoints
            self.initial_pop_size = int(state["population_size"])
            self.start_round = int(state["next_round"])
            rows = [(m["model_id"], m["accuracy"], m["hparams"], m["epoches_trained"]) for m in state["members"]]
            csv_lines = {int(m["model_id"]): m.get("csv_lines", {}) for m in state["members"]}
            streams = {int(m["model_id"]): m.get("stream_state") for m in state["members"]}
        self.pop_size = len(rows)
        blocks = partition(self.initial_pop_size, self.n_groups)
        self.id_owner = {}  # member id -> member group (= rank when dp_size == 1)
        for r, (b, c) in enumerate(blocks):
            for i in range(b, b + c):
                self.id_owner[i] = r
        mine = [r for r in rows if self.id_owner[int(r[0])] == self.group_index]
        self.worker.is_expolore_only = bool(do_explore and not do_exploit)
        self.worker.add_members([(r[0], copy.deepcopy(r[2])) for r in mine])
        if state is not None:
            by_id = self.worker.members_by_id()
            tag = state.get("ckpt_round")  # exactly the round the table describes (members may be one ahead)
            for mid, acc, _, epochs in mine:
                g = by_id[int(mid)]
                if not g.load_checkpoint(round_tag=tag):
                    raise RuntimeError("resume: member %d has no checkpoint%s in %s"
                                       % (mid, "" if tag is None else " of round %d" % tag, g.save_dir))
                g.accuracy, g.epoches_trained = float(acc), int(epochs)
                if streams.get(int(mid)) is not None and hasattr(g, "restore_stream_state"):
                    g.restore_stream_state(streams[int(mid)])
                # drop learning-curve rows a crashed round appended after the table was written
                reports.truncate_member_csvs(g.save_dir, csv_lines.get(int(mid), {}))
            self.log("Resumed %d members at round %d" % (len(rows), self.start_round))
        self.last_plan = []

    def log(self, *a):
        if self.verbose and self.rank == 0:
            print(*a, flush=True)

    @property
    def is_group_leader(self) -> bool:
        return self.dp is None or self.dp.rank == 0

    def _values(self):
        """This rank's share of the population table (replicas other than a group's first report nothing)."""
        vals = self.worker.get_all_values()
        return vals if self.is_group_leader else []

    def get_all_values(self):
        parts = self.comm.allgather(self._values())
        return [v for part in parts for v in part]

    def train_one_round(self, rnd, total_rounds):
        # the batch sizes this round trains with (explore may change them before the round's metrics line)
        self._round_bs = [[int(getattr(g, "cluster_id", -1)), int(g.hparams.get("batch_size", 0))]
                          for g in self.worker.worker_graphs if self.is_group_leader and hasattr(g, "hparams")]
        self.worker.train(self.epochs_per_round, self.epochs_per_round * total_rounds)
        for mid in self.inject_nan.get(rnd, []):
            for g in list(self.worker.worker_graphs):
                if g.cluster_id == mid:
                    g.accuracy = float("nan")
                    if not self.reseed_dead:
                        self.worker._cull(g, "injected nan")

    def _steps(self):
        """member id -> host step counter of this rank's members (sent with the scores: an exploit destination
        learns its new step without reading the imported device row back)."""
        return {int(g.cluster_id): int(getattr(g, "global_step", 0) or 0) for g in self.worker.worker_graphs}

    def exploit(self):
        gathered = self.comm.allgather([self._values(), self._steps()])  # also the end-of-train barrier
        t0 = time.time()
        parts = [g[0] for g in gathered]
        steps = {}
        for g in gathered:
            steps.update(g[1])
        values = [v for part in parts for v in part]
        owner = {int(v[0]): r // self.dp_size for r, part in enumerate(parts) for v in part}  # member group
        self.pop_size = len(values)
        plan = plan_reseed(values) if getattr(self, "reseed_dead", False) else plan_exploit(values)
        self.last_plan = plan
        for p in plan:
            self.log("Copied: {} -> {}".format(p.src_id, p.dst_id))
        d = self.dp_size  # replica r of the winner's group -> replica r of the loser's group
        transfers = [(p.src_id, owner[p.src_id] * d + r, p.dst_id, owner[p.dst_id] * d + r)
                     for p in plan for r in range(d)]
        if transfers:
            self.dataplane.execute(transfers, self.worker.members_by_id(), steps=steps)
        updates = apply_plan_to_values(values, plan)
        mine = [u for mid, u in updates.items() if owner[mid] == self.group_index]
        self.worker.set_values(mine)
        self.exploit_time += time.time() - t0

    def explore(self):
        self.worker.explore_necessary_graphs()

    def _counters(self):
        dp = self.dataplane
        return [sum(int(getattr(g, "images_trained", 0)) for g in self.worker.worker_graphs), self.worker.train_time,
                self.worker.explore_time, float(dp.bytes_moved), dp.seconds, dp.transfers_done]

    def _graph_state(self):
        from ..engine.hip_resnet import graph_state
        for g in self.worker.worker_graphs:
            eng = getattr(g, "engine", None)
            if eng is not None:
                return graph_state(eng.backend)
        return None

    def log_round_metrics(self, rnd, round_s):
        """Append one JSON line per round to ``savedata/metrics.jsonl``: throughput (images/s of
        the whole job), per-phase times (train / exploit / explore, max over ranks), exploit data-plane bytes and
        latency, population accuracy summary."""
        from ..utils.profiling import PHASES
        cur = self._counters()
        prev = getattr(self, "_prev_counters", None) or [0, 0.0, 0.0, 0.0, 0.0, 0]
        self._prev_counters = cur
        delta = [c - p for c, p in zip(cur, prev)]
        phases = PHASES.since(getattr(self, "_prev_phases", {}))
        self._prev_phases = PHASES.snapshot()
        parts = self.comm.allgather([delta, [float(v[1]) for v in self._values()], phases, self._graph_state(),
                                     getattr(self, "_round_bs", [])])
        if self.rank != 0:
            return
        d = [p[0] for p in parts]
        phase_s = {}
        for p in parts:  # member-level phases inside the round (train steps, eval, checkpoint, hooks): max over ranks
            for k, v in p[2].items():
                phase_s[k] = max(phase_s.get(k, 0.0), v)
        accs = [a for p in parts for a in p[1] if a == a]
        images = sum(x[0] for x in d)
        rec = {"round": rnd, "round_s": round_s, "images": images,
               "images_per_s": images / round_s if round_s > 0 else None,
               "train_s": max(x[1] for x in d), "explore_s": max(x[2] for x in d),
               "exploit_s": self.exploit_time - getattr(self, "_prev_exploit", 0.0),
               "exploit_transfers": int(max(x[5] for x in d)), "exploit_bytes": int(sum(x[3] for x in d)),
               "exploit_dataplane_s": max(x[4] for x in d), "population": len(accs),
               "best_acc": max(accs) if accs else None, "mean_acc": sum(accs) / len(accs) if accs else None,
               "world_size": self.world, "phases_s": phase_s,
               # how the HIP step ran on each rank ("captured" graph replay / "eager_fallback" when a data-parallel
               # capture was refused / "disabled" / None for torch backends): a silent eager cliff shows up here
               "step_graph": sorted({str(p[3]) for p in parts}),
               # member id -> batch size trained this round (bench.py --ragged --batch_sizes reproduces the mix)
               "batch_sizes": {str(i): b for p in parts for i, b in sorted(p[4])}}
        self._prev_exploit = self.exploit_time
        import json
        os.makedirs(self.savedata, exist_ok=True)
        with open(os.path.join(self.savedata, "metrics.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")

    def save_round_state(self, next_round):
        """Resume point: re-save the members whose state changed after their end-of-train checkpoint (exploit
        destinations), then rank 0 writes the population table."""
        dsts = {p.dst_id for p in self.last_plan} if self.do_exploit else set()
        for g in self.worker.worker_graphs:
            if g.cluster_id in dsts and getattr(g, "checkpoint_every_round", True):
                g.save_checkpoint()
                if getattr(g, "tf_checkpoint", False) and self.is_group_leader:
                    # the reference's directory holds the winner's TF checkpoint after the copy: re-export the
                    # bundle of the imported state and drop the loser's stale one
                    reports.remove_tf_bundles(g.save_dir)
                    g.export_tf_checkpoint()
        flush_checkpoints()  # every rank's checkpoints are on disk before the table that names them
        rows = self.comm.allgather([[g.cluster_id, g.get_accuracy(), g.hparams, g.epoches_trained,
                                     reports.member_csv_lines(g.save_dir),
                                     g.stream_state() if hasattr(g, "stream_state") else None]
                                    for g in self.worker.worker_graphs] if self.is_group_leader else [])
        if self.rank == 0:
            reports.write_population_state(self.savedata, next_round, self.initial_pop_size,
                                           [r for part in rows for r in part], ckpt_round=next_round - 1)

    def train(self, round_num):
        """Run rounds ``start_round .. round_num - 1`` (``start_round`` > 0 after a resume)."""
        start = time.time()
        for rnd in range(self.start_round, round_num):
            t0 = time.time()
            self.log("\nRound {}".format(rnd))
            for g in self.worker.worker_graphs:
                g.ckpt_round = rnd  # checkpoints written in this round are tagged with it
            # roctx ranges (rocprofv3 --marker-trace, DTF_ROCTX=1) around the PBT phases
            with roctx_range("pbt/round%d/train" % rnd):
                self.train_one_round(rnd, round_num)
            if self.do_exploit:
                with roctx_range("pbt/round%d/exploit" % rnd):
                    self.exploit()
            if self.do_explore:
                with roctx_range("pbt/round%d/explore" % rnd):
                    self.explore()
            with roctx_range("pbt/round%d/checkpoint" % rnd):
                self.save_round_state(rnd + 1)
            self.round_times.append(time.time() - t0)
            self.log_round_metrics(rnd, self.round_times[-1])
            self.log("Round elapsed time: {}\n".format(datetime.timedelta(seconds=self.round_times[-1])))
        self.comm.barrier()
        total = time.time() - start
        self.log("Total elapsed time: {}".format(datetime.timedelta(seconds=total)))
        return total

    def get_profiling_info(self):
        return self.comm.allgather([self.worker.train_time, self.worker.explore_time])

    def print_profiling_info(self):
        infos = self.get_profiling_info()
        n = max(1, len(infos))
        tr = sum(i[0] for i in infos) / n
        ex = sum(i[1] for i in infos) / n
        if self.rank == 0:
            print("")
            print("=======Profiling Information========")
            print("Total train time: {}".format(datetime.timedelta(seconds=tr)))
            print("Total exploit time: {}".format(datetime.timedelta(seconds=self.exploit_time)))
            print("Total explore time: {}\n".format(datetime.timedelta(seconds=ex)))
            print("Exploit data plane: {} transfers, {:.1f} KB, {:.3f}s".format(
                self.dataplane.transfers_done, self.dataplane.bytes_moved / 1024.0, self.dataplane.seconds))
        return {"train": tr, "exploit": self.exploit_time, "explore": ex}

    # report writers run on rank 0 but need everyone for the gather
    def dump_all_models_to_json(self, filename):
        vals = self.get_all_values()
        if self.rank == 0:
            reports.dump_population_json(vals, filename)

    def report_best_model(self):
        vals = self.get_all_values()
        if self.rank == 0:
            return reports.write_best_model(vals, os.path.join(self.savedata, "best_model.json"))

    def export_best_model(self, export_dir):
        """``--export_dir`` (reference resnet_run_loop.py:510-514 SavedModel export): the rank that owns the best
        member writes its inference weights + metadata (utils/export.export_member)."""
        vals = self.get_all_values()
        if not vals:
            return None
        best = int(reports.best_member(vals)[0])
        g = self.worker.members_by_id().get(best)
        if g is not None and self.is_group_leader:
            from ..utils.export import export_member
            export_member(g, export_dir)
        self.comm.barrier()
        return export_dir

    def kill_all_workers(self):
        self.comm.barrier()
