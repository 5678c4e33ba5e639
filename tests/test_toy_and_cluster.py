"""Toy model resume semantics + the PBT drivers on the in-process LocalComm backend."""
import json
import os
import threading

import pytest

from distributedtf_amd.models import toy_model
from distributedtf_amd.models.toy_model import ToyModel
from distributedtf_amd.parallel.comm import LocalComm
from distributedtf_amd.parallel.dataplane import DataPlane
from distributedtf_amd.pbt import generate_random_hparam
from distributedtf_amd.pbt.cluster import PBTCluster, SPMDPopulation, copy_member_files
from distributedtf_amd.pbt.worker import TrainingWorker


@pytest.fixture
def hp():
    h = generate_random_hparam()
    h["h_0"], h["h_1"] = 1.0, 0.0
    return h


def test_toy_basic(tmp_cwd, hp):
    step, obj = toy_model.main(hp, 0, "savedata/model_", "", 1)
    assert step == 1


def test_toy_model_class_train(tmp_cwd, hp):
    m = ToyModel(0, hp, "savedata/model_")
    acc1, e1 = m.get_accuracy(), m.epoches_trained
    m.train(1, 1)
    assert m.get_accuracy() != acc1 and m.epoches_trained == e1 + 1


def test_toy_save_load(tmp_cwd, hp):
    """Port of reference test_toy_model.py:38-50."""
    import shutil
    s1, _ = toy_model.main(hp, 0, "savedata/model_", "", 10)
    s2, _ = toy_model.main(hp, 0, "savedata/model_", "", 10)
    s3, _ = toy_model.main(hp, 1, "savedata/model_", "", 10)
    assert (s1, s2, s3) == (10, 20, 10)
    shutil.rmtree("savedata")
    os.mkdir("savedata")
    s4, _ = toy_model.main(hp, 0, "savedata/model_", "", 10)
    assert s4 == 10


def test_toy_csv_contract(tmp_cwd, hp):
    m = ToyModel(3, hp, "savedata/model_")
    m.train(4, 4)
    lines = open("savedata/model_3/learning_curve.csv").read().strip().splitlines()
    assert lines[0] == "global_step,accuracy,optimizer,lr"
    assert len(lines) == 5
    assert open("savedata/model_3/theta.csv").read().startswith("theta_0,theta_1")


def test_copy_member_files_rules(tmp_path):
    src, dst = tmp_path / "model_1", tmp_path / "model_2"
    src.mkdir(); dst.mkdir()
    (src / "model.ckpt").write_text("W")
    (src / "learning_curve.csv").write_text("src-curve")
    (dst / "model.ckpt").write_text("old")
    (dst / "stale.bin").write_text("x")
    (dst / "learning_curve.csv").write_text("dst-curve")
    (dst / "events.out.tfevents.1").write_text("ev")
    assert copy_member_files(str(src), str(dst))
    assert (dst / "model.ckpt").read_text() == "W"
    assert not (dst / "stale.bin").exists()
    assert (dst / "learning_curve.csv").read_text() == "dst-curve"
    assert (dst / "events.out.tfevents.1").exists()
    assert not copy_member_files(str(src), str(src))


def _run_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except Exception as e:  # pragma: no cover
            errs.append(e)
            raise
    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs


@pytest.mark.parametrize("transport", ["dataplane", "files"])
def test_master_worker_protocol_localcomm(tmp_cwd, transport):
    comms = LocalComm.create(3)
    out = {}

    def master():
        c = PBTCluster(6, comms[0], 0, epochs_per_round=4, seed=7, exploit_transport=transport)
        c.dump_all_models_to_json("savedata/initial_hp.json")
        out["t"] = c.train(4)
        out["vals"] = c.get_all_values()
        out["prof"] = c.get_profiling_info()
        c.report_best_model()
        c.report_plot_for_toy_model()
        c.report_accuracy_plot()
        c.report_lr_plot()
        c.report_best3_plot()
        c.kill_all_workers()

    def worker(r):
        TrainingWorker(comms[r], 0, ToyModel, seed=7, dataplane=DataPlane(comms[r]), verbose=False).main_loop()

    _run_threads([master, lambda: worker(1), lambda: worker(2)])
    assert len(out["vals"]) == 6
    assert sorted(v[0] for v in out["vals"]) == list(range(6))
    init = json.load(open("savedata/initial_hp.json"))
    assert len(init) == 6 and all(d["accuracy"] == 0.0 for d in init)
    best = json.load(open("savedata/best_model.json"))
    assert set(best) == {"best_model_id", "best_acc", "best_hparams"}
    for f in ["toy_PBT.png", "acc_PBT.png", "lr_PBT.png", "best3_PBT.png"]:
        assert os.path.isfile(os.path.join("savedata", f))


def test_spmd_localcomm_matches_and_culls(tmp_cwd):
    comms = LocalComm.create(2)
    res = {}

    def rank(r):
        pop = SPMDPopulation(8, comms[r], ToyModel, epochs_per_round=3, seed=11, verbose=False,
                             inject_nan={1: [5]})
        pop.train(3)
        res[r] = pop.get_all_values()
        res["plan%d" % r] = [(p.src_id, p.dst_id) for p in pop.last_plan]

    _run_threads([lambda: rank(0), lambda: rank(1)])
    assert res[0] == res[1]
    assert sorted(v[0] for v in res[0]) == [0, 1, 2, 3, 4, 6, 7]  # member 5 culled after round 1
    assert res["plan0"] == res["plan1"]
    assert not os.path.exists("savedata/model_5")


def test_modes_file_suffix():
    from distributedtf_amd.pbt.reports import mode_name
    assert mode_name(True, True)[1] == "PBT"
    assert mode_name(True, False)[1] == "exploit_only"
    assert mode_name(False, True)[1] == "explore_only"
    assert mode_name(False, False)[1] == "grid_search"
