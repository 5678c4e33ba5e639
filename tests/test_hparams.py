"""Search space sampling and the explore rule (reference constants.py, model_base.py:30-104)."""
import copy
import random

from hypothesis import given, settings, strategies as st

from distributedtf_amd.pbt.hparams import (decimal_places_of, generate_random_hparam, get_hp_range_definition,
                                           perturb_hparams)

R = get_hp_range_definition()


def test_sample_ranges_many():
    rng = random.Random(0)
    seen_opts = set()
    for _ in range(2000):
        hp = generate_random_hparam(rng)
        opt = hp["opt_case"]
        seen_opts.add(opt["optimizer"])
        assert opt["lr"] in R["lr"][opt["optimizer"]]
        if opt["optimizer"] in ("Momentum", "RMSProp"):
            assert 0.0 <= opt["momentum"] <= 0.9
        else:
            assert "momentum" not in opt
        if opt["optimizer"] == "RMSProp":
            assert 0.0 <= opt["grad_decay"] <= 0.9
        assert hp["decay_steps"] in R["decay_steps"]
        assert 0.1 <= hp["decay_rate"] <= 1.0
        assert 1e-8 <= hp["weight_decay"] <= 1e-2
        assert hp["regularizer"] in R["regularizer"]
        assert hp["initializer"] in R["initializer"]
        assert isinstance(hp["batch_size"], int) and 65 <= hp["batch_size"] <= 255
    assert seen_opts == set(R["optimizer_list"])


def test_sampler_deterministic_with_seed():
    a = [generate_random_hparam(random.Random(5)) for _ in range(3)]
    b = [generate_random_hparam(random.Random(5)) for _ in range(3)]
    assert a == b


def test_decimal_places():
    assert decimal_places_of(0.001) == 3
    assert decimal_places_of(0.1) == 1
    assert decimal_places_of(1e-08) == 8
    assert decimal_places_of(1e-05) == 5
    assert decimal_places_of(0.0001) == 4
    assert decimal_places_of(0.0) == 1


@settings(max_examples=200, deadline=None)
@given(seed=st.integers(0, 10 ** 6))
def test_perturb_stays_in_range(seed):
    rng = random.Random(seed)
    hp = generate_random_hparam(rng)
    before = copy.deepcopy(hp)
    perturb_hparams(hp, rng)
    opt = hp["opt_case"]
    grid = R["lr"][opt["optimizer"]]
    assert opt["optimizer"] == before["opt_case"]["optimizer"]
    assert grid[0] <= opt["lr"] <= grid[-1]
    assert hp["initializer"] == before["initializer"] and hp["regularizer"] == before["regularizer"]
    assert 65 <= hp["batch_size"] <= 256
    assert 0 <= hp["decay_steps"] <= 100
    assert 0.1 <= hp["decay_rate"] <= 1.0
    assert 1e-8 <= hp["weight_decay"] <= 1e-2
    # float perturbation stays within [0.8v, 1.2v] (modulo clamping / rounding)
    v = before["decay_rate"]
    # decay_rate rounds to 1 decimal (str(0.1) has one), so allow +-0.05 of rounding
    assert max(0.1, 0.8 * v) - 0.05 - 1e-9 <= hp["decay_rate"] <= min(1.0, 1.2 * v) + 0.05 + 1e-9


def test_perturb_int_rules():
    rng = random.Random(1)
    hp = {"batch_size": 255, "decay_steps": 0, "opt_case": {"optimizer": "gd", "lr": 1.0}}
    for _ in range(50):
        h = copy.deepcopy(hp)
        perturb_hparams(h, rng)
        assert 204 <= h["batch_size"] <= 256
        assert h["decay_steps"] == 0  # floor(0)=ceil(0)=0 -> min


def test_perturb_rounding_digits():
    rng = random.Random(3)
    for _ in range(100):
        hp = {"weight_decay": 5e-3, "opt_case": {"optimizer": "Adam", "lr": 1e-3}}
        perturb_hparams(hp, rng)
        assert round(hp["weight_decay"], 8) == hp["weight_decay"]
        assert round(hp["opt_case"]["lr"], 4) == hp["opt_case"]["lr"]


def test_string_keys_resampled_except_arch():
    rng = random.Random(2)
    hp = {"activation": "relu", "initializer": "he_init", "regularizer": "l1_regularizer",
          "opt_case": {"optimizer": "Momentum", "lr": 0.1, "momentum": 0.5}}
    perturb_hparams(hp, rng)
    assert hp["activation"] == "relu" and hp["initializer"] == "he_init"
    assert 0.4 <= hp["opt_case"]["momentum"] <= 0.6
