"""Hyper-parameter search space, sampler and the PBT "explore" rule.

Behavioural contract:
  * range table            -- reference ``constants.py:14-43``
  * sampling distributions -- reference ``constants.py:45-100`` (hyperopt space);
    re-implemented here without hyperopt: categorical choices are uniform,
    continuous ranges are ``uniform(lo, hi)``, ``batch_size = randint(191) + 65``.
  * perturbation rule      -- reference ``model_base.py:30-104``.

Every sampler / perturbation takes an explicit ``random.Random`` so a PBT run
can be replayed exactly (the reference never seeds anything, Appendix A14).
"""

from __future__ import annotations

import copy
import enum
import math
import random as _random
from typing import Any, Dict, Optional

__all__ = [
    "WorkerInstruction",
    "get_hp_range_definition",
    "load_hp_space",
    "generate_random_hparam",
    "perturb_hparams",
    "decimal_places_of",
    "ARCH_KEYS",
]


class WorkerInstruction(enum.Enum):
    """Master -> worker opcodes (reference ``constants.py:5-12``)."""

    ADD_GRAPHS = 0
    EXIT = 1
    TRAIN = 2
    GET = 3
    SET = 4
    EXPLORE = 5
    GET_PROFILING_INFO = 6


# Keys whose value defines the architecture: never perturbed
# (reference ``model_base.py:82-85``).
ARCH_KEYS = frozenset(
    ["num_filters_1", "kernel_size_1", "kernel_size_2", "activation", "initializer", "regularizer"]
)

_OPTIMIZERS = ("Adadelta", "Adagrad", "Momentum", "Adam", "RMSProp", "gd")


def get_hp_range_definition() -> Dict[str, Any]:
    """The range table used both for sampling and for clamping perturbations."""
    return {
        "h_0": [0.0, 1.0],
        "h_1": [0.0, 1.0],
        "optimizer_list": list(_OPTIMIZERS),
        "lr": {
            "Adadelta": [0.1, 0.5, 1.0, 1.5, 2.0, 2.5, 3.0, 3.5, 4.0, 4.5, 5.0],
            "Adagrad": [1e-3, 1e-2, 1e-1, 0.5, 1.0],
            "Momentum": [1e-3, 1e-2, 1e-1, 0.5, 1.0],
            "Adam": [1e-4, 1e-3, 1e-2, 1e-1],
            "RMSProp": [1e-5, 1e-4, 1e-3],
            "gd": [1e-2, 1e-1, 0.5, 1.0, 1.5, 2.0, 2.5, 3.0, 3.5, 4.0, 4.5, 5.0],
        },
        "momentum": [0.00, 0.9],
        "grad_decay": [0.00, 0.9],
        "decay_steps": [0, 10, 20, 30, 40, 50, 60, 70, 80, 90, 100],
        "decay_rate": [0.1, 1.0],
        "weight_decay": [1e-8, 1e-2],
        "regularizer": ["l1_regularizer", "l2_regularizer", "l1_l2_regularizer", "None"],
        "initializer": ["glorot_normal", "orthogonal", "he_init", "None"],
        "batch_size": [191],
    }


class _Choice:
    def __init__(self, options):
        self.options = list(options)

    def sample(self, rng):
        return copy.deepcopy(self.options[rng.randrange(len(self.options))])


class _Uniform:
    def __init__(self, lo, hi):
        self.lo, self.hi = float(lo), float(hi)

    def sample(self, rng):
        return rng.uniform(self.lo, self.hi)


class _RandInt:
    def __init__(self, upper, offset=0):
        self.upper, self.offset = int(upper), int(offset)

    def sample(self, rng):
        return rng.randrange(self.upper) + self.offset


def load_hp_space() -> Dict[str, Any]:
    """A declarative description of the search space (hyperopt-free).

    Nested dicts are sampled recursively; leaves are ``_Choice``/``_Uniform``/
    ``_RandInt`` nodes.  ``opt_case`` is a choice over per-optimizer sub-spaces.
    """
    r = get_hp_range_definition()
    mom = _Uniform(*r["momentum"])
    gdec = _Uniform(*r["grad_decay"])
    opt_cases = [
        {"optimizer": "Adadelta", "lr": _Choice(r["lr"]["Adadelta"])},
        {"optimizer": "Adagrad", "lr": _Choice(r["lr"]["Adagrad"])},
        {"optimizer": "Momentum", "lr": _Choice(r["lr"]["Momentum"]), "momentum": mom},
        {"optimizer": "Adam", "lr": _Choice(r["lr"]["Adam"])},
        {"optimizer": "RMSProp", "lr": _Choice(r["lr"]["RMSProp"]), "grad_decay": gdec, "momentum": mom},
        {"optimizer": "gd", "lr": _Choice(r["lr"]["gd"])},
    ]
    return {
        "opt_case": _Choice(opt_cases),
        "decay_steps": _Choice(r["decay_steps"]),
        "decay_rate": _Uniform(*r["decay_rate"]),
        "weight_decay": _Uniform(*r["weight_decay"]),
        "regularizer": _Choice(r["regularizer"]),
        "initializer": _Choice(r["initializer"]),
        "batch_size": _RandInt(r["batch_size"][0], offset=65),
    }


def _sample_node(node, rng):
    if isinstance(node, (_Choice, _Uniform, _RandInt)):
        val = node.sample(rng)
        return _sample_node(val, rng) if isinstance(val, dict) else val
    if isinstance(node, dict):
        return {k: _sample_node(v, rng) for k, v in node.items()}
    return node


def generate_random_hparam(rng: Optional[_random.Random] = None) -> Dict[str, Any]:
    """Draw one hyper-parameter dict (reference ``constants.py:96-100``)."""
    rng = rng if rng is not None else _random
    sample = _sample_node(load_hp_space(), rng)
    sample["batch_size"] = int(sample["batch_size"])
    return sample


# --------------------------------------------------------------------------- explore

def decimal_places_of(limit_min: float) -> int:
    """Rounding precision derived from the textual form of a range's lower limit.

    ``0.001`` -> 3, ``0.1`` -> 1, ``1e-08`` -> 8 (exponent form), ``1.0`` -> 1.
    Mirrors reference ``model_base.py:31-41``.
    """
    text = str(limit_min)
    if "e" in text:
        exponent = int(text.split("e")[1])
        return -exponent if exponent < 0 else exponent
    return text[::-1].find(".")


def _perturb_float(rng, val, lo, hi, factors):
    digits = decimal_places_of(lo)
    a, b = val * factors[0], val * factors[1]
    if a < lo:
        a = lo
        digits += 1
    if b > hi:
        b = hi
    return round(rng.uniform(a, b), digits)


def _perturb_int(rng, val, lo, hi, factors):
    if lo == hi:
        lo = 0
    a = int(math.floor(val * factors[0]))
    b = int(math.ceil(val * factors[1]))
    a = max(a, lo)
    b = min(b, hi)
    if a >= b:
        return a
    return rng.randint(a, b)


def perturb_hparams(hparams: Dict[str, Any], rng: Optional[_random.Random] = None,
                    factors=(0.8, 1.2)) -> Dict[str, Any]:
    """Apply the PBT explore rule in place and return ``hparams``.

    * float  -> ``uniform(0.8v, 1.2v)`` clamped to the range table, rounded;
    * int    -> ``randint(floor(0.8v), ceil(1.2v))`` clamped
      (``batch_size`` clamps to ``[65, 256]``);
    * str    -> architecture keys fixed, others resampled;
    * opt_case -> optimizer fixed; lr (and momentum / grad_decay) perturbed.
    """
    rng = rng if rng is not None else _random
    rdef = get_hp_range_definition()
    # keys in sorted (canonical) order: the draws a key receives must not depend on the dict's insertion order,
    # which a JSON round trip (checkpoint blob, whole-run resume table, all-gathered values) does not keep -- a
    # resumed or differently placed run then perturbs exactly like the original (the reference iterates its
    # hyperopt sample's order with an unseeded rng, so no order is observable there)
    for key in sorted(hparams.keys()):
        value = hparams[key]
        if isinstance(value, bool):
            continue
        if isinstance(value, float):
            lo, hi = rdef[key][0], rdef[key][-1]
            hparams[key] = _perturb_float(rng, value, lo, hi, factors)
        elif isinstance(value, int):
            if key == "batch_size":
                hparams[key] = _perturb_int(rng, value, 65, rdef[key][-1] + 65, factors)
            else:
                hparams[key] = _perturb_int(rng, value, rdef[key][0], rdef[key][-1], factors)
        elif key == "opt_case":
            case = value
            opt = case["optimizer"]
            grid = rdef["lr"][opt]
            case["lr"] = _perturb_float(rng, case["lr"], grid[0], grid[-1], factors)
            if opt in ("Momentum", "RMSProp"):
                case["momentum"] = _perturb_float(
                    rng, case["momentum"], rdef["momentum"][0], rdef["momentum"][-1], factors)
            if opt == "RMSProp":
                case["grad_decay"] = _perturb_float(
                    rng, case["grad_decay"], rdef["grad_decay"][0], rdef["grad_decay"][-1], factors)
        elif key not in ARCH_KEYS:
            choices = rdef[key]
            hparams[key] = copy.deepcopy(choices[rng.randrange(len(choices))])
    return hparams
