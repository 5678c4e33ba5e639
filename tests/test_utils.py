"""Ports of the vendored utils tests (flags_test, logger_test, hooks_test, hooks_helper_test,
model_helpers_test, distribution_utils_test, export_test) onto the new utils."""
import json
import os

import pytest
import torch

from distributedtf_amd.utils import hooks, logger, model_helpers
from distributedtf_amd.utils.export import serving_input_spec
from distributedtf_amd.utils.flags import MemberConfig, get_loss_scale, parse_main_args


class _MockLogger(logger.BaseBenchmarkLogger):
    def __init__(self):
        self.logged = []

    def log_metric(self, name, value, unit=None, global_step=None, extras=None):
        self.logged.append({"name": name, "value": value, "global_step": global_step})


def test_flags_defaults_and_positional():
    a = parse_main_args(["7", "--model", "toy"])
    assert a.population_size == 7 and a.model == "toy" and a.train_round == 20 and a.mode == "spmd"
    assert get_loss_scale("fp16", None) == 128 and get_loss_scale("bf16", None) == 1
    assert get_loss_scale("fp32", 5) == 5


def test_flags_validators():
    with pytest.raises(SystemExit):
        parse_main_args(["--loss_scale", "-1"])
    with pytest.raises(SystemExit):
        parse_main_args(["--resnet_version", "1", "--dtype", "fp16"])
    with pytest.raises(SystemExit):
        parse_main_args(["--dtype", "int8"])


def test_member_config():
    hp = {"opt_case": {"optimizer": "RMSProp", "lr": 1e-4, "momentum": 0.5, "grad_decay": 0.8},
          "decay_steps": 20, "decay_rate": 0.5, "weight_decay": 1e-3, "regularizer": "None",
          "initializer": "he_init", "batch_size": 99}
    m = MemberConfig.from_hparams(hp, 3)
    assert m.optimizer == "RMSProp" and m.regularizer is None and m.batch_size == 99 and m.model_id == 3


def test_file_logger(tmp_path):
    fl = logger.BenchmarkFileLogger(str(tmp_path))
    fl.log_metric("accuracy", 0.5, global_step=3, extras={"a": "b"})
    fl.log_metric("bad", "not-a-number")
    lines = open(tmp_path / "metric.log").read().strip().splitlines()
    assert len(lines) == 1
    m = json.loads(lines[0])
    assert m["name"] == "accuracy" and m["value"] == 0.5 and m["global_step"] == 3
    assert m["extras"] == [{"name": "a", "value": "b"}]
    fl.log_run_info("resnet", "cifar10", {"batch_size": 32})
    info = json.load(open(tmp_path / "benchmark_run.log"))
    assert info["model_name"] == "resnet" and info["dataset"]["name"] == "cifar10"


def test_benchmark_context_status(tmp_path):
    class F:
        benchmark_logger_type = "BenchmarkFileLogger"
        benchmark_log_dir = str(tmp_path)
    with logger.benchmark_context(F()):
        pass
    assert json.load(open(tmp_path / "benchmark_run.log"))["status"] == "success"
    with pytest.raises(RuntimeError):
        with logger.benchmark_context(F()):
            raise RuntimeError("x")
    assert json.load(open(tmp_path / "benchmark_run.log"))["status"] == "failure"


def test_examples_per_second_hook():
    ml = _MockLogger()
    h = hooks.ExamplesPerSecondHook(batch_size=256, every_n_steps=2, warm_steps=1, metric_logger=ml)
    h.begin()
    for step in range(1, 8):
        h.after_step(step, {})
    names = [m["name"] for m in ml.logged]
    assert names.count("average_examples_per_sec") == 3 and names.count("current_examples_per_sec") == 3
    assert h.average > 0
    with pytest.raises(ValueError):
        hooks.ExamplesPerSecondHook(batch_size=1)


def test_hooks_helper_registry():
    hs = hooks.get_train_hooks("LoggingTensorHook,ExamplesPerSecondHook", batch_size=8)
    assert isinstance(hs[0], hooks.LoggingHook) and isinstance(hs[1], hooks.ExamplesPerSecondHook)
    assert hooks.get_train_hooks("") == []
    with pytest.raises(ValueError):
        hooks.get_train_hooks(["nope"])


def test_logging_metric_hook():
    ml = _MockLogger()
    h = hooks.LoggingMetricHook(every_n_steps=10, metric_logger=ml)
    h.after_step(10, {"cross_entropy": 2.0, "learning_rate": 0.1})
    assert {m["name"] for m in ml.logged} == {"cross_entropy", "learning_rate"}


def test_past_stop_threshold():
    assert model_helpers.past_stop_threshold(None, 1.5) is False
    assert model_helpers.past_stop_threshold(0.5, 0.6) is True
    assert model_helpers.past_stop_threshold(0.5, 0.4) is False
    with pytest.raises(ValueError):
        model_helpers.past_stop_threshold("x", 1.0)
    with pytest.raises(ValueError):
        model_helpers.past_stop_threshold(0.5, "x")


def test_member_dp_batch_split():
    """Intra-member DP splits a member's batch over its ranks (uneven sizes allowed, unlike
    distribution_utils.per_device_batch_size): the shards always add up to the member's batch."""
    from distributedtf_amd.parallel.dataparallel import DPContext
    for b in (64, 65, 127):
        shards = [DPContext(group=None, size=4, rank=r, group_index=0, n_groups=1).local_batch(b) for r in range(4)]
        assert sum(shards) == b and max(shards) - min(shards) <= 1


def test_serving_spec():
    s = serving_input_spec((32, 32, 3), batch_size=8)
    assert s["shape"] == [8, 32, 32, 3]


def test_curve_check_bounds():
    """The trajectory test's per-window bound (utils/curves.py): the round-5 driver failure (Momentum window 2, HIP
    1.105 vs oracle 0.819, neighbours 1.668 / 0.422) passes as a one-window lag; a curve that stays 0.5 above the
    oracle on a flat stretch fails; a window where torch bf16 itself sits far from fp32 widens the bound."""
    import torch
    from distributedtf_amd.utils.curves import curve_check, windowed_means
    ref = torch.tensor([[2.273], [1.668], [0.819], [0.422], [0.220]])
    hip = torch.tensor([[2.269], [1.798], [1.105], [0.588], [0.255]])
    ok, rows = curve_check(ref, ref, hip)
    assert ok.all(), rows
    assert "shift" in rows[2]
    flat_ref = torch.full((6, 1), 0.05)
    ok, rows = curve_check(flat_ref, flat_ref, flat_ref + 0.5)
    assert not ok.any(), rows
    yard = torch.full((6, 1), 0.45)
    ok, rows = curve_check(flat_ref, yard, flat_ref + 0.5)
    assert ok.all() and all("bf16" in r for r in rows), rows
    w = windowed_means([torch.tensor([1.0, 2.0]), torch.tensor([3.0, 4.0]), torch.tensor([5.0, 6.0])], 2)
    assert w.shape == (1, 2) and w.tolist() == [[2.0, 3.0]]
