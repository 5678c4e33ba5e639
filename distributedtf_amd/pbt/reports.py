"""Run artefacts: JSON population snapshots, PNG plots, ``test_results.txt``.

File names and CSV column contracts follow the reference
(``pbt_cluster.py:240-470``, ``main_manager.py:60-61``):

* ``savedata/initial_hp.json`` / ``dump_population_json`` -- ``[{model_id,
  accuracy, hparams}]`` sorted ascending by accuracy;
* ``savedata/best_model.json`` -- ``{best_model_id, best_acc, best_hparams}``;
* ``{acc,lr,best3,toy}_{PBT,exploit_only,explore_only,grid_search}.png``.
  Plots read ``learning_curve.csv`` columns 0 (x), 1 (accuracy), 3 (lr) and
  ``theta.csv`` columns 0/1.
"""

from __future__ import annotations

import csv
import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np


def mode_name(do_exploit: bool, do_explore: bool) -> Tuple[str, str]:
    """(plot title, file suffix) for the four PBT modes."""
    if do_exploit and do_explore:
        return "PBT", "PBT"
    if do_exploit:
        return "Exploit only", "exploit_only"
    if do_explore:
        return "Explore only", "explore_only"
    return "Grid search", "grid_search"


def _ranked(values):
    return sorted((list(v) for v in values), key=lambda v: float(v[1]))


def dump_population_json(values: Sequence, filename: str) -> None:
    report = [{"model_id": int(v[0]), "accuracy": float(v[1]), "hparams": v[2]} for v in _ranked(values)]
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    with open(filename, "w") as fp:
        json.dump(report, fp, indent=4, sort_keys=True)


def best_member(values: Sequence):
    """The ``[id, acc, hparams]`` row best_model.json reports (last of the ascending ranking)."""
    return _ranked(values)[-1]


def write_best_model(values: Sequence, filename: str) -> Dict:
    best = best_member(values)
    report = {"best_model_id": int(best[0]), "best_acc": float(best[1]), "best_hparams": best[2]}
    os.makedirs(os.path.dirname(filename) or ".", exist_ok=True)
    with open(filename, "w") as fp:
        json.dump(report, fp, indent=4, sort_keys=True)
    return report


POPULATION_STATE = "population_state.json"


def write_population_state(savedata: str, next_round: int, population_size: int, rows: Sequence,
                           ckpt_round: Optional[int] = None) -> str:
    """Whole-run resume table (opt-in ``--resume``): the round to run next, the round
    tag of the member checkpoints it pairs with (``model.ckpt-r<ckpt_round>``) and, per surviving member,
    ``[id, accuracy, hparams, epoches_trained(, csv line counts)]``.  Written atomically (tmp + rename) at the end
    of every round, after the members' checkpoints."""
    path = os.path.join(savedata, POPULATION_STATE)
    members = []
    for r in sorted(rows, key=lambda r: int(r[0])):
        m = {"model_id": int(r[0]), "accuracy": float(r[1]), "hparams": r[2], "epoches_trained": int(r[3])}
        if len(r) > 4:
            m["csv_lines"] = dict(r[4])
        if len(r) > 5 and r[5] is not None:
            m["stream_state"] = r[5]  # explore rng (+ data stream) of the member: a resumed run replays the same draws
        members.append(m)
    blob = {"next_round": int(next_round), "population_size": int(population_size), "members": members}
    if ckpt_round is not None:
        blob["ckpt_round"] = int(ckpt_round)
    os.makedirs(savedata, exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as fp:
        json.dump(blob, fp, indent=2, sort_keys=True)
    os.replace(tmp, path)
    return path


def member_csv_lines(save_dir: str) -> Dict[str, int]:
    """Line count of every CSV in a member directory (learning_curve.csv, theta.csv)."""
    out = {}
    if os.path.isdir(save_dir):
        for f in sorted(os.listdir(save_dir)):
            if f.endswith(".csv"):
                with open(os.path.join(save_dir, f)) as fp:
                    out[f] = sum(1 for _ in fp)
    return out


def truncate_member_csvs(save_dir: str, lines: Dict[str, int]) -> None:
    """Cut each CSV back to the line count recorded with the population table (resume after a crashed round)."""
    for f, n in lines.items():
        path = os.path.join(save_dir, f)
        if not os.path.isfile(path):
            continue
        with open(path) as fp:
            keep = fp.readlines()
        if len(keep) > int(n):
            with open(path, "w") as fp:
                fp.writelines(keep[:int(n)])


def remove_tf_bundles(save_dir: str) -> None:
    """Delete the TF tensor bundles (``model.ckpt-<step>.index`` / ``.data-*``) of a member directory."""
    if not os.path.isdir(save_dir):
        return
    for f in os.listdir(save_dir):
        if f.startswith("model.ckpt-") and (f.endswith(".index") or ".data-" in f) and not f.startswith("model.ckpt-r"):
            os.remove(os.path.join(save_dir, f))


def read_population_state(savedata: str) -> Dict:
    with open(os.path.join(savedata, POPULATION_STATE)) as fp:
        return json.load(fp)


def append_test_result(world_size: int, pop_size: int, seconds: float, path: str = "test_results.txt") -> None:
    with open(path, "a") as f:
        f.write("n = {}, pop_size = {}, time = {}s\n".format(world_size, pop_size, seconds))


def _member_csvs(savedata: str, name: str) -> List[str]:
    if not os.path.isdir(savedata):
        return []
    out = []
    for d in sorted(os.listdir(savedata)):
        p = os.path.join(savedata, d, name)
        if d.startswith("model_") and os.path.isfile(p):
            out.append(p)
    return out


def read_columns(path: str, cols: Sequence[int], casts: Sequence) -> List[List]:
    rows = []
    with open(path) as f:
        reader = csv.reader(f)
        header = next(reader, None)
        if header is None:
            return rows
        for r in reader:
            if not r:
                continue
            rows.append([c(float(r[i])) if c is int else c(r[i]) for i, c in zip(cols, casts)])
    return rows


def _pyplot():
    import matplotlib
    matplotlib.use("Agg")
    from matplotlib import pyplot
    return pyplot


def _finish(plt, savedata, kind, do_exploit, do_explore):
    title, suffix = mode_name(do_exploit, do_explore)
    plt.title(title)
    out = os.path.join(savedata, f"{kind}_{suffix}.png")
    plt.savefig(out)
    plt.close()
    return out


def plot_curves(savedata: str, kind: str, do_exploit: bool, do_explore: bool) -> str:
    """kind in {'acc', 'lr'}: one line per member from learning_curve.csv."""
    plt = _pyplot()
    col = 1 if kind == "acc" else 3
    plt.figure()
    for path in _member_csvs(savedata, "learning_curve.csv"):
        rows = read_columns(path, [0, col], [int, float])
        if rows:
            xs, ys = zip(*rows)
            plt.plot(xs, ys)
    plt.xlabel("Train epochs")
    plt.ylabel("Accuracy" if kind == "acc" else "Learning rate")
    if kind == "lr":
        plt.ylim(0, 1)
    plt.grid(True)
    return _finish(plt, savedata, kind, do_exploit, do_explore)


def top3_average(curves: List[List[Tuple[int, float]]]) -> List[Tuple[int, float]]:
    """Per record index: mean of the 3 best accuracies (fewer if <3 members)."""
    longest = max((len(c) for c in curves), default=0)
    out = []
    for i in range(longest):
        col = sorted(c[i][1] for c in curves if len(c) > i)
        x = next((c[i][0] for c in curves if len(c) > i), 0)
        best = col[-3:]
        out.append((x, sum(best) / len(best) if best else 0.0))
    return out


def plot_best3(savedata: str, do_exploit: bool, do_explore: bool) -> str:
    plt = _pyplot()
    curves = [read_columns(p, [0, 1], [int, float]) for p in _member_csvs(savedata, "learning_curve.csv")]
    curves = [c for c in curves if c]
    plt.figure()
    for c in curves:
        xs, ys = zip(*c)
        plt.plot(xs, ys, color=(0.0, 0.0, 0.5, 0.3))
    avg = top3_average(curves)
    if avg:
        xs, ys = zip(*avg)
        plt.plot(xs, ys, "r")
    plt.xlabel("Train epochs")
    plt.ylabel("Accuracy")
    plt.ylim(0, 1)
    plt.grid(True)
    return _finish(plt, savedata, "best3", do_exploit, do_explore)


def plot_toy(savedata: str, do_exploit: bool, do_explore: bool) -> str:
    plt = _pyplot()
    plt.figure()
    plt.xlabel(r"$\theta_0$")
    plt.ylabel(r"$\theta_1$")
    plt.xlim(0, 1)
    plt.ylim(0, 1)
    for p in _member_csvs(savedata, "theta.csv"):
        rows = read_columns(p, [0, 1], [float, float])
        if rows:
            xs, ys = zip(*rows)
            plt.plot(xs, ys, ".")
    g = np.linspace(0, 1, 100)
    x, y = np.meshgrid(g, g)
    plt.contour(x, y, 1.2 - (x ** 2 + y ** 2), colors="lightgray")
    return _finish(plt, savedata, "toy", do_exploit, do_explore)
