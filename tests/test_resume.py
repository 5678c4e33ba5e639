"""Opt-in whole-run resume: a run stopped after some rounds continues from
``savedata/population_state.json`` + the members' checkpoints -- round counter, surviving ids, weights
(step counters), accuracies and hyper-parameters carry over; culled members stay dead."""
import json
import os

import pytest

from distributedtf_amd.models.toy_model import ToyModel
from distributedtf_amd.parallel.comm import LocalComm
from distributedtf_amd.pbt.cluster import SPMDPopulation
from distributedtf_amd.pbt.reports import POPULATION_STATE

from test_toy_and_cluster import _run_threads


def _run(world, rounds, resume, out, inject=None):
    comms = LocalComm.create(world)

    def body(r):
        pop = SPMDPopulation(6, comms[r], ToyModel, epochs_per_round=2, seed=5, verbose=False, resume=resume,
                             inject_nan=inject or {})
        out.setdefault("start", {})[r] = pop.start_round
        pop.train(rounds)
        vals = pop.get_all_values()
        steps = {g.cluster_id: int(g.export_state()[2]) for g in pop.worker.worker_graphs}
        out.setdefault("vals", {})[r] = vals
        out.setdefault("steps", {}).update(steps)
        out.setdefault("epochs", {}).update({g.cluster_id: g.epoches_trained for g in pop.worker.worker_graphs})

    _run_threads([lambda r=r: body(r) for r in range(world)])


@pytest.mark.parametrize("world", [1, 2])
def test_resume_continues_rounds(tmp_cwd, world):
    first, second = {}, {}
    _run(world, 2, False, first, inject={0: [4]})
    st = json.load(open(os.path.join("savedata", POPULATION_STATE)))
    assert st["next_round"] == 2 and st["population_size"] == 6
    assert sorted(m["model_id"] for m in st["members"]) == [0, 1, 2, 3, 5]  # member 4 was culled
    assert all(m["epoches_trained"] == 4 for m in st["members"])
    assert set(first["steps"].values()) == {4}
    # a "new job" resumes and runs rounds 2..4
    _run(world, 5, True, second)
    assert set(second["start"].values()) == {2}
    assert sorted(second["steps"]) == [0, 1, 2, 3, 5]
    assert set(second["steps"].values()) == {10}  # 5 rounds x 2 epochs, continued from the checkpoints
    assert set(second["epochs"].values()) == {10}
    st = json.load(open(os.path.join("savedata", POPULATION_STATE)))
    assert st["next_round"] == 5
    # learning curves were appended to, not restarted
    rows = open("savedata/model_0/learning_curve.csv").read().strip().splitlines()
    assert len(rows) == 1 + 10


def test_resume_without_state_starts_fresh(tmp_cwd):
    out = {}
    _run(1, 1, True, out)
    assert set(out["start"].values()) == {0}
    assert set(out["steps"].values()) == {2}


def test_round_metrics_jsonl(tmp_cwd):
    out = {}
    _run(2, 3, False, out)
    recs = [json.loads(l) for l in open(os.path.join("savedata", "metrics.jsonl"))]
    assert [r["round"] for r in recs] == [0, 1, 2]
    for r in recs:
        assert r["population"] == 6 and r["world_size"] == 2
        assert r["exploit_transfers"] == 2  # ceil(6/4) = 2 bottom members per round
        assert r["exploit_bytes"] > 0 and r["round_s"] > 0


def test_resume_after_crash_between_checkpoints_and_table(tmp_cwd):
    """members finish round r+1 (checkpoints + learning-curve rows written) but the job dies before the
    population table of round r+1 is written.  Resume must load exactly the round-r checkpoints the table pairs
    with (round-tagged files) and drop the crashed round's CSV rows -- no extra round of training, no duplicate
    learning-curve rows."""
    first = {}
    _run(1, 2, False, first)
    assert os.path.isfile("savedata/model_0/model.ckpt-r1")

    def crash(self, next_round):
        raise RuntimeError("simulated crash before the round-%d table" % next_round)

    orig = SPMDPopulation.save_round_state
    SPMDPopulation.save_round_state = crash
    try:
        with pytest.raises(RuntimeError):
            comms = LocalComm.create(1)
            pop = SPMDPopulation(6, comms[0], ToyModel, epochs_per_round=2, seed=5, verbose=False, resume=True)
            pop.train(3)
    finally:
        SPMDPopulation.save_round_state = orig
    from distributedtf_amd.models.model_base import flush_checkpoints
    flush_checkpoints()
    assert os.path.isfile("savedata/model_0/model.ckpt-r2")  # the crashed round's checkpoints exist ...
    assert len(open("savedata/model_0/learning_curve.csv").read().strip().splitlines()) == 1 + 6
    second = {}
    _run(1, 5, True, second)  # ... but the resume pairs the table (round 2 next) with the round-1 files
    assert set(second["start"].values()) == {2}
    assert set(second["steps"].values()) == {10}
    assert set(second["epochs"].values()) == {10}
    rows = open("savedata/model_0/learning_curve.csv").read().strip().splitlines()
    assert len(rows) == 1 + 10
    assert not os.path.exists("savedata/model_0/model.ckpt-r2")  # only the last two round tags are kept
