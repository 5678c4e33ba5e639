"""--debug_kernels / --deterministic switches and deterministic replay of a CPU PBT run."""
import os

import torch

from distributedtf_amd.utils.flags import parse_main_args


def test_debug_kernels_sets_hip_serialisation(monkeypatch):
    for k in ("AMD_SERIALIZE_KERNEL", "HIP_LAUNCH_BLOCKING", "DTF_HIP_GRAPH", "DTF_DEBUG"):
        monkeypatch.delenv(k, raising=False)
    a = parse_main_args(["4", "--model", "cifar10", "--debug_kernels"])
    a.apply_runtime_modes()
    assert os.environ["AMD_SERIALIZE_KERNEL"] == "3"
    assert os.environ["HIP_LAUNCH_BLOCKING"] == "1"
    assert os.environ["DTF_HIP_GRAPH"] == "0"
    assert os.environ["DTF_DEBUG"] == "1"
    for k in ("AMD_SERIALIZE_KERNEL", "HIP_LAUNCH_BLOCKING", "DTF_HIP_GRAPH", "DTF_DEBUG"):
        monkeypatch.delenv(k, raising=False)


def test_deterministic_mode_seeds_and_selects_backend(monkeypatch):
    """--deterministic seeds every RNG; CIFAR ResNet v2 and MNIST keep the HIP backend (deterministic kernel builds),
    families whose HIP kernels keep atomic reductions fall back to deterministic torch algorithms."""
    monkeypatch.delenv("DTF_DETERMINISTIC", raising=False)
    try:
        a = parse_main_args(["4", "--model", "cifar10", "--deterministic"])
        a.apply_runtime_modes()
        assert a.seed == 0 and a.backend == "auto"
        assert os.environ["DTF_DETERMINISTIC"] == "1"
        assert torch.are_deterministic_algorithms_enabled()
        b = parse_main_args(["4", "--model", "mnist", "--deterministic"])
        b.apply_runtime_modes()
        assert b.backend == "auto"
        c = parse_main_args(["4", "--model", "imagenet", "--deterministic"])
        c.apply_runtime_modes()
        assert c.backend == "auto" and c.model_kwargs()["backend"] == "auto"
    finally:
        torch.use_deterministic_algorithms(False)
        os.environ.pop("DTF_DETERMINISTIC", None)


def test_seeded_pbt_runs_replay_exactly(tmp_cwd):
    from distributedtf_amd.models.toy_model import ToyModel
    from distributedtf_amd.parallel.comm import LocalComm
    from distributedtf_amd.pbt.cluster import SPMDPopulation

    def run(tag):
        pop = SPMDPopulation(6, LocalComm.create(1)[0], ToyModel, epochs_per_round=2, seed=3, verbose=False,
                             savedata="savedata_%s" % tag)
        pop.train(4)
        return sorted((v[0], v[1], sorted(v[2].items(), key=str)) for v in pop.get_all_values())

    assert run("a") == run("b")
