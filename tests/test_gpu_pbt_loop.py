"""The product PBT loop on the GPU: ``SPMDPopulation`` -> ``EngineModel.train_population`` (HIP step graph) ->
population eval -> checkpoint -> exploit (D2D state copy) -> explore, and the ``main_manager`` entry point.

Reference: ``pbt_cluster.py:87-166`` (round loop, exploit copying the winner's checkpoint: weights, optimizer slots
and global step), ``training_worker.py:60-95``, ``main_manager.py:48-70``.
"""
import json
import math
import os

import pytest
import torch

from distributedtf_amd.models.cifar10_model import Cifar10Model
from distributedtf_amd.models.engine_model import EngineModel
from distributedtf_amd.parallel.comm import SingleComm
from distributedtf_amd.pbt.cluster import SPMDPopulation

pytestmark = pytest.mark.gpu


def _kw(**extra):
    kw = dict(resnet_size=20, backend="hip", use_synthetic_data=True, max_train_steps=6, device="cuda:0")
    kw.update(extra)
    return kw


def test_spmd_population_exploit_is_bit_exact_and_loser_follows_winner(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    EngineModel.reset_engines()
    from distributedtf_amd.pbt.cluster import sample_population
    hps = sample_population(4, 5)
    for i, h in enumerate(hps):  # sane optimizers (no divergence -> no culling); batch sizes stay ragged
        h["opt_case"] = {"optimizer": "Momentum", "lr": 0.02 * (i + 1), "momentum": 0.9}
    pop = SPMDPopulation(4, SingleComm(), Cifar10Model, epochs_per_round=1, seed=5, savedata="savedata",
                         verbose=False, model_kwargs=_kw(), hparams=hps)
    members = pop.worker.members_by_id()
    eng = next(iter(members.values())).engine
    assert eng.backend.name == "hip"
    pop.train_one_round(0, 2)
    for g in members.values():
        assert math.isfinite(g.get_accuracy()) and 0.0 <= g.get_accuracy() <= 1.0
        assert g.global_step == 6
    pop.exploit()
    plan = pop.last_plan
    assert len(plan) == 1  # k = ceil(4 / 4)
    p = plan[0]
    win, lose = members[p.src_id], members[p.dst_id]
    torch.cuda.synchronize()
    # the loser's whole state row (weights, optimizer slots, BN moving statistics, step) is the winner's
    assert torch.equal(eng.state[win.slot], eng.state[lose.slot])
    assert lose.global_step == win.global_step
    assert lose.hparams == win.hparams  # (ModelBase.set_values copies only the hparams: model_base.py:112-113)
    # next step on the same batch with the same hyper-parameters: the loser follows the winner
    ds = win.dataset()
    b = int(win.hparams["batch_size"])
    batch = ds.batch_slice(b)
    lrs = [win.learning_rate(win.global_step)] * 2
    losses = eng.train_step([win.slot, lose.slot], [batch, batch], [win.hparams, lose.hparams], lrs).cpu()
    torch.cuda.synchronize()
    assert abs(float(losses[0]) - float(losses[1])) <= 1e-3 * max(1.0, abs(float(losses[0]))), losses
    # parameters after the step: equal up to the reduction-order noise of two members of one population step
    # (fp32 atomics in the BN statistics, bf16 activations).  At random init the BN-gamma / stem gradients are sums
    # with heavy cancellation, so even identical twins differ there by ~10% relative (tools/twin_check.py); the
    # whole parameter row moves by ~1e-3 -- a stale weight / hyper / step refresh would show in the loss above.
    P = eng.P
    a, b = eng.state[win.slot, :P].double(), eng.state[lose.slot, :P].double()
    rel = float((a - b).norm() / a.norm())
    assert rel <= 5e-3, rel
    assert lose.global_step == win.global_step
    pop.explore()
    pop.save_round_state(1)
    # second round through the whole loop (checkpoint, metrics)
    pop.train_one_round(1, 2)
    pop.exploit()
    pop.explore()
    pop.save_round_state(2)
    for g in members.values():
        lines = open(os.path.join(g.save_dir, "learning_curve.csv")).read().strip().splitlines()
        assert len(lines) == 3, lines  # header + 2 rounds
        assert os.path.isfile(os.path.join(g.save_dir, "model.ckpt"))


def test_main_manager_cifar10_hip_end_to_end(tmp_path, monkeypatch):
    """``main_manager.py 4 --model cifar10 ...`` on one GPU: every reference output file plus metrics.jsonl with the
    round's phases itemised (train steps / eval / checkpoint)."""
    import main_manager
    monkeypatch.chdir(tmp_path)
    EngineModel.reset_engines()
    rc = main_manager.main(["4", "--model", "cifar10", "--resnet_size", "20", "--use_synthetic_data", "true",
                            "--max_train_steps", "8", "--rounds", "2", "--seed", "3", "--backend", "hip"])
    assert rc == 0
    sd = "savedata"
    for f in ("initial_hp.json", "best_model.json", "metrics.jsonl", "acc_PBT.png", "lr_PBT.png", "best3_PBT.png"):
        assert os.path.isfile(os.path.join(sd, f)), f
    recs = [json.loads(l) for l in open(os.path.join(sd, "metrics.jsonl"))]
    assert [r["round"] for r in recs] == [0, 1]
    init = json.load(open(os.path.join(sd, "initial_hp.json")))
    assert recs[0]["images"] == 8 * sum(int(d["hparams"]["batch_size"]) for d in init)
    for r in recs:
        assert r["images_per_s"] > 0
        assert "eval" in r["phases_s"] and "train_steps" in r["phases_s"] and "checkpoint" in r["phases_s"]
    best = json.load(open(os.path.join(sd, "best_model.json")))
    assert 0.0 <= best["best_acc"] <= 1.0
    assert open("test_results.txt").read().startswith("n = 1, pop_size = 4")
