"""Placement invariance of a whole PBT run over real RCCL.

The same population -- ``main_manager.py 8 --model cifar10 --resnet_size 20 --deterministic`` (pop 8, seed 1,
3 rounds) -- runs at world 1, 2, 4 and 8 under torchrun on the 1-GPU box (``DTF_SHARE_GPU=1``: each rank its own
RCCL "node", parallel/comm.py configure_shared_gpu), i.e. with 8, 4, 2 and 1 members per rank.  World 8 is the
headline topology: an 8-rank communicator, and each k = 2 exploit moves two disjoint cross-rank pairs in one
``batch_isend_irecv``.  The data is ``--use_synthetic_data learnable`` (class-template images
through the real input path), so the population LEARNS -- best accuracy climbs well above chance over the rounds
and the exploit plan ranks real differences, not noise.  Every rank
trains (SPMD), exploit copies cross ranks in both directions in one ``batch_isend_irecv`` (parallel/dataplane.py),
and the deterministic kernel build makes every per-member reduction order independent of the other members of a
plan.  Asserted BITWISE across world sizes:

  * ``best_model.json`` and ``initial_hp.json``;
  * every member's final checkpoint state row (weights, optimizer slots, BN moving statistics, step counter) and
    hyper-parameters (``model_<id>/model.ckpt``);
  * the per-round population accuracies of ``metrics.jsonl`` (best / mean) and the exploit plans (``Copied:`` lines).

Then a resume: world 2 runs rounds 0-1, stops, and ``--resume`` runs round 2 -- the final states must equal the
uninterrupted runs' (reference: main_manager.py:46-73, pbt_cluster.py:113-166; whole-run resume is this
framework's addition).
"""
import json
import os
import re
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["8", "--model", "cifar10", "--resnet_size", "20", "--deterministic", "--max_train_steps", "25",
        "--seed", "1", "--use_synthetic_data", "learnable"]
WORLDS = (1, 2, 4, 8)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, savedata, rounds, extra=(), timeout=240):
    env = dict(os.environ, DTF_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "main_manager.py"] + ARGS + \
        ["--rounds", str(rounds), "--savedata", str(savedata), "--results_file", os.path.join(str(savedata), "r.txt")] \
        + list(extra)
    logdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else str(savedata)
    path = os.path.join(logdir, "placement_w%d_%s.log" % (world, os.path.basename(str(savedata))))
    with open(path, "w") as f:
        try:
            rc = subprocess.run(cmd, cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT, timeout=timeout).returncode
        except subprocess.TimeoutExpired:
            rc = "timeout"
    log = open(path).read()
    assert rc == 0, "world %d rc %s\n%s" % (world, rc, log[-5000:])
    return log


def _outcome(savedata, log):
    out = {"best": json.load(open(os.path.join(savedata, "best_model.json"))),
           "initial": json.load(open(os.path.join(savedata, "initial_hp.json"))),
           "copies": re.findall(r"Copied: (\d+) -> (\d+)", log), "states": {}, "hparams": {}, "rounds": []}
    for line in open(os.path.join(savedata, "metrics.jsonl")):
        r = json.loads(line)
        out["rounds"].append((r["round"], r["population"], r["best_acc"], r["mean_acc"]))
    for d in sorted(os.listdir(savedata)):
        if d.startswith("model_"):
            blob = torch.load(os.path.join(savedata, d, "model.ckpt"), map_location="cpu", weights_only=True)
            out["states"][d] = blob["state"]
            out["hparams"][d] = json.dumps(blob["hparams"], sort_keys=True)
    return out


def _same(a, b, what):
    assert a["best"] == b["best"], (what, a["best"], b["best"])
    assert a["initial"] == b["initial"], what
    assert a["rounds"] == b["rounds"], (what, a["rounds"], b["rounds"])
    assert sorted(a["states"]) == sorted(b["states"]), what
    diff = [k for k in a["states"] if not torch.equal(a["states"][k], b["states"][k])]
    assert not diff, (what, "state rows differ", diff)
    assert a["hparams"] == b["hparams"], what


@pytest.mark.timeout(1150)
def test_pbt_run_is_placement_invariant_and_resumable(tmp_path):
    res = {}
    for w in WORLDS:
        sd = tmp_path / ("w%d" % w)
        res[w] = _outcome(str(sd), _run(w, sd, 3, timeout=300))
        print("world %d: rounds %s copies %s" % (w, res[w]["rounds"], res[w]["copies"]))
    assert len(res[1]["states"]) == 8 and len(res[1]["rounds"]) == 3
    assert res[1]["copies"], "exploit must have copied members"
    # a learning population: the best member is far above chance (0.1) by the last round, and improves
    best = [r[2] for r in res[1]["rounds"]]
    assert best[-1] >= 0.3 and best[-1] > best[0], best
    # the copies cross ranks at world 2 / 4 / 8 (pop 8: rank r owns members 8r/w ..)
    for w in WORLDS[1:]:
        per = 8 // w
        assert any(int(s) // per != int(d) // per for s, d in res[w]["copies"]), (w, res[w]["copies"])
        assert res[w]["copies"] == res[1]["copies"], (w, res[w]["copies"], res[1]["copies"])
        _same(res[1], res[w], "world 1 vs %d" % w)
    # whole-run resume: rounds 0-1, then --resume for round 2, at world 2
    sd = tmp_path / "resume"
    log1 = _run(2, sd, 2)
    log2 = _run(2, sd, 3, extra=["--resume"])
    assert "Resumed 8 members at round 2" in log2, log2[-3000:]
    r = _outcome(str(sd), log1 + log2)
    _same(res[1], r, "uninterrupted vs resumed")
