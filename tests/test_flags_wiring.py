"""Every main_manager flag reaches the training loop (CPU, PyTorch backend, ResNet-8 on synthetic data).

Reference wiring: ``resnet_run_loop.py:419-426`` (run info + train hooks), ``:466`` (log_evaluation_result),
``:469-503`` (one learning-curve row per eval cycle), ``:505-508`` (stop threshold), ``:510-514`` (export),
``official/utils/logs/hooks_helper.py:33-35,97-132`` (hook registry).
"""
import csv
import json
import os

import pytest

import main_manager
from distributedtf_amd.models.engine_model import EngineModel
from distributedtf_amd.utils import logger as bench_logger

BASE = ["2", "--model", "cifar10", "--resnet_size", "8", "--use_synthetic_data", "true", "--seed", "4",
        "--backend", "torch"]


def _run(tmp_path, monkeypatch, *extra):
    monkeypatch.chdir(tmp_path)
    EngineModel.reset_engines()
    assert main_manager.main(BASE + list(extra)) == 0


def _curves(sd="savedata"):
    out = {}
    for d in sorted(os.listdir(sd)):
        p = os.path.join(sd, d, "learning_curve.csv")
        if os.path.isfile(p):
            out[d] = list(csv.DictReader(open(p)))
    return out


def test_hooks_logger_and_export(tmp_path, monkeypatch, capsys):
    _run(tmp_path, monkeypatch, "--max_train_steps", "4", "--rounds", "2", "--hooks",
         "logging,examples_per_second,metric", "--log_every_n_steps", "2", "--benchmark_logger_type",
         "BenchmarkFileLogger", "--benchmark_log_dir", "bench_logs", "--export_dir", "exported")
    out = capsys.readouterr().out
    assert "cross_entropy" in out and "learning_rate" in out and "model_id" in out  # LoggingHook lines
    metrics = [json.loads(l) for l in open("bench_logs/metric.log")]
    names = {m["name"] for m in metrics}
    assert {"accuracy", "loss", "average_examples_per_sec", "current_examples_per_sec", "cross_entropy"} <= names
    acc = [m for m in metrics if m["name"] == "accuracy"]
    assert len(acc) == 4  # 2 members x 2 rounds (log_evaluation_result per eval)
    run = json.load(open("bench_logs/benchmark_run.log"))
    assert run["status"] == "success" and run["model_name"] == "resnet8"
    assert os.path.isfile("exported/model.safetensors")
    meta = json.load(open("exported/model.json"))
    best = json.load(open("savedata/best_model.json"))
    assert meta["model_id"] == best["best_model_id"]


def test_epoch_cycles_and_stop_threshold(tmp_path, monkeypatch):
    """epochs_per_round 2 -> two train/eval cycles (two CSV rows) per round; a stop threshold every eval passes
    ends each member's call after its first cycle."""
    monkeypatch.setattr("distributedtf_amd.models.cifar10_model.Cifar10Model.steps_per_epoch", lambda self: 2)
    _run(tmp_path, monkeypatch, "--rounds", "1", "--epochs_per_round", "2")
    rows = _curves()
    assert all(len(r) == 2 for r in rows.values()), rows
    assert all(r[0]["epochs"] == r[1]["epochs"] == "0" for r in rows.values())  # epoch_index of the call
    os.chdir(tmp_path)
    import shutil
    shutil.rmtree("savedata")
    _run(tmp_path, monkeypatch, "--rounds", "1", "--epochs_per_round", "2", "--stop_threshold", "0.0")
    rows = _curves()
    assert all(len(r) == 1 for r in rows.values()), rows


def test_ready_steps_and_batch_size(tmp_path, monkeypatch):
    _run(tmp_path, monkeypatch, "--rounds", "2", "--ready_steps", "3", "--batch_size", "16")
    recs = [json.loads(l) for l in open("savedata/metrics.jsonl")]
    assert [r["images"] for r in recs] == [2 * 3 * 16, 2 * 3 * 16]  # explore cannot move the pinned batch
    for r in _curves().values():
        assert all(row["batch_size"] == "16" for row in r)


def test_dtype_routing():
    from distributedtf_amd.utils.flags import parse_main_args
    a = parse_main_args(["--model", "cifar10", "--dtype", "fp32"])
    assert a.backend == "auto" and a.model_kwargs()["dtype"] == "fp32"  # the fp32 HIP step on a GPU
    assert parse_main_args(["--model", "cifar10", "--dtype", "fp32", "--backend", "hip"]).backend == "hip"
    assert parse_main_args(["--model", "cifar10", "--dtype", "fp32", "--loss_scale", "8"]).backend == "torch"
    with pytest.raises(SystemExit):
        parse_main_args(["--model", "cifar10", "--dtype", "fp32", "--loss_scale", "8", "--backend", "hip"])
    # ImageNet fp32 too (engine/hip_imagenet_f32.py); MNIST fp16 has no half build -> torch
    assert parse_main_args(["--model", "imagenet", "--dtype", "fp32", "--backend", "hip"]).backend == "hip"
    with pytest.raises(SystemExit):
        parse_main_args(["--model", "mnist", "--dtype", "fp16", "--backend", "hip"])
    # MNIST fp32 stays on HIP (engine/hip_mnist_f32.py: the generic fp32 MFMA conv kernels)
    assert parse_main_args(["--model", "mnist", "--dtype", "fp32"]).backend == "auto"
    assert parse_main_args(["--model", "mnist", "--dtype", "fp32", "--backend", "hip"]).backend == "hip"
    with pytest.raises(SystemExit):
        parse_main_args(["--model", "cifar10", "--loss_scale", "8"])  # bf16 HIP path: no loss scaling
    a = parse_main_args(["--model", "cifar10", "--dtype", "fp16"])
    # fp16 ResNet v2: the half build of the HIP kernels (DTF_HALF, set by apply_runtime_modes) with loss scale 128
    assert a.backend == "auto" and a.model_kwargs()["loss_scale"] == 128
    assert parse_main_args(["--model", "imagenet", "--dtype", "fp16", "--backend", "hip"]).backend == "hip"
    assert parse_main_args(["--model", "mnist", "--dtype", "fp16"]).backend == "torch"  # no fp16 MNIST kernels
    with pytest.raises(SystemExit):  # the reference's validator: fp16 is not supported with ResNet v1
        parse_main_args(["--model", "cifar10", "--dtype", "fp16", "--resnet_version", "1"])
    # fp16 + --deterministic: the deterministic half build (libdtf_kernels_f16_det.so)
    assert parse_main_args(["--model", "cifar10", "--dtype", "fp16", "--deterministic",
                            "--backend", "hip"]).backend == "hip"
    with pytest.raises(SystemExit):  # no debug fp16 kernel build
        parse_main_args(["--model", "cifar10", "--dtype", "fp16", "--debug_kernels", "--backend", "hip"])
    with pytest.raises(SystemExit):
        parse_main_args(["--benchmark_logger_type", "BenchmarkFileLogger"])


def test_fp16_loss_scaled_training_is_finite(tmp_path, monkeypatch):
    _run(tmp_path, monkeypatch, "--rounds", "1", "--max_train_steps", "2", "--dtype", "fp32", "--loss_scale", "64")
    best = json.load(open("savedata/best_model.json"))
    assert best["best_acc"] == best["best_acc"]


def test_deterministic_flag_selects_det_build(monkeypatch):
    """--deterministic keeps the HIP backend for the CIFAR ResNet v1/v2 and MNIST steps (deterministic kernel build,
    selected by DTF_DETERMINISTIC) and moves the families whose HIP kernels keep atomic reductions to the torch
    backend; an explicit --backend hip for those is an error."""
    from distributedtf_amd import ops
    from distributedtf_amd.ops import build as kb
    from distributedtf_amd.utils.flags import parse_main_args
    monkeypatch.delenv("DTF_DETERMINISTIC", raising=False)
    a = parse_main_args(["--model", "cifar10", "--deterministic"])
    a.apply_runtime_modes()
    try:
        assert os.environ.get("DTF_DETERMINISTIC") == "1" and ops.deterministic_mode()
        assert a.backend == "auto" and a.seed == 0
        b = parse_main_args(["--model", "mnist", "--deterministic"])
        b.apply_runtime_modes()
        assert b.backend == "auto"  # MNIST has a deterministic HIP build too
        v1 = parse_main_args(["--model", "cifar10", "--resnet_version", "1", "--deterministic", "--backend", "hip"])
        assert v1.backend == "hip"  # so does ResNet v1 (per-image BN-backward rows added in image order)
        c = parse_main_args(["--model", "imagenet", "--deterministic"])
        c.apply_runtime_modes()
        assert c.backend == "auto"  # ImageNet: fixed-point (int64) accumulation in the deterministic build
        assert parse_main_args(["--model", "imagenet", "--deterministic", "--backend", "hip"]).backend == "hip"
        # the fp32 CIFAR step has a deterministic build too (int64 fixed-point accumulation, f32conv.hip)
        assert parse_main_args(["--model", "cifar10", "--dtype", "fp32", "--deterministic",
                                "--backend", "hip"]).backend == "hip"
        assert parse_main_args(["--model", "mnist", "--dtype", "fp32", "--deterministic",
                                "--backend", "hip"]).backend == "hip"
        assert parse_main_args(["--model", "imagenet", "--dtype", "fp32", "--deterministic",
                                "--backend", "hip"]).backend == "hip"
        with pytest.raises(SystemExit):  # an explicit --backend hip must not silently lose the guarantee
            parse_main_args(["--model", "mnist", "--dtype", "fp16", "--deterministic", "--backend", "hip"])
        with pytest.raises(SystemExit):  # the debug kernel build is not the deterministic one
            parse_main_args(["--model", "cifar10", "--deterministic", "--debug_kernels"])
        assert kb.LIB_DET.endswith("libdtf_kernels_det.so") and "-DDTF_NREP=64" in kb.DET_FLAGS
        assert kb.LIB_HALF_DET.endswith("libdtf_kernels_f16_det.so")
    finally:
        os.environ.pop("DTF_DETERMINISTIC", None)
        import torch
        torch.use_deterministic_algorithms(False)


def test_reference_base_flags_train_epochs_ebe_model_dir(tmp_path, monkeypatch):
    """--train_epochs / --epochs_between_evals / --model_dir (reference official/utils/flags/_base.py:56-80):
    train_epochs is the epochs a member trains per round, the round runs train_epochs // epochs_between_evals
    train -> eval cycles (resnet_run_loop.py:446-447), model_dir is the member-directory base."""
    from distributedtf_amd.utils.flags import parse_main_args
    a = parse_main_args(["--model", "cifar10", "--train_epochs", "4", "--epochs_between_evals", "2",
                         "--model_dir", "md"])
    assert a.epochs_per_round == 4 and a.savedata == "md" and a.model_kwargs()["epochs_between_evals"] == 2
    with pytest.raises(SystemExit):
        parse_main_args(["--epochs_between_evals", "0"])
    monkeypatch.setattr("distributedtf_amd.models.cifar10_model.Cifar10Model.steps_per_epoch", lambda self: 2)
    _run(tmp_path, monkeypatch, "--rounds", "1", "--train_epochs", "4", "--epochs_between_evals", "2",
         "--model_dir", "md")
    rows = _curves("md")
    assert len(rows) == 2 and all(len(r) == 2 for r in rows.values()), rows  # 4 // 2 cycles per round
    recs = [json.loads(l) for l in open("md/metrics.jsonl")]
    assert recs[0]["images"] > 0


def test_mnist_probabilities_hook(tmp_path, monkeypatch, capsys):
    """The reference logs MNIST's training softmax every 50 iterations (mnist_model.py:149-151): on by default,
    rows are probability distributions over the 10 classes, one line per member."""
    from distributedtf_amd.utils.hooks import ProbabilitiesHook, get_train_hooks
    monkeypatch.chdir(tmp_path)
    EngineModel.reset_engines()
    assert main_manager.main(["2", "--model", "mnist", "--use_synthetic_data", "true", "--seed", "3",
                              "--backend", "torch", "--rounds", "1", "--max_train_steps", "5",
                              "--log_probabilities_every_n", "2", "--batch_size", "16"]) == 0
    out = capsys.readouterr().out
    lines = [l for l in out.splitlines() if "probabilities = " in l]
    assert len(lines) == 2 * 2, out[-2000:]  # steps 2 and 4, two members
    assert "model_id = 0" in out and "model_id = 1" in out
    h = [h for h in get_train_hooks("probabilities", probabilities_every_n=3)][0]
    assert isinstance(h, ProbabilitiesHook) and h.every_n_steps == 3
    eng = next(iter(EngineModel._engines.values()))
    hk = [x for x in eng.train_hooks if isinstance(x, ProbabilitiesHook)][0]
    import numpy as np
    pr = hk.records[-1]["probabilities"]
    assert pr.shape == (16, 10) and np.allclose(pr.sum(axis=1), 1.0, atol=1e-5)
    # off switch
    EngineModel.reset_engines()
    monkeypatch.chdir(tmp_path / "..")
    (tmp_path / "off").mkdir()
    monkeypatch.chdir(tmp_path / "off")
    assert main_manager.main(["2", "--model", "mnist", "--use_synthetic_data", "true", "--seed", "3",
                              "--backend", "torch", "--rounds", "1", "--max_train_steps", "5",
                              "--log_probabilities_every_n", "0", "--batch_size", "16"]) == 0
    assert "probabilities = " not in capsys.readouterr().out
