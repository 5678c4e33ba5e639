"""Model helpers (reference ``official/utils/misc/model_helpers.py`` and
``distribution_utils.py``).

* ``past_stop_threshold`` -- early stop when an eval metric reaches the flag;
* ``generate_synthetic_data`` -- constant device tensors (reference synthetic mode);
* ``apply_clean`` -- ``--clean`` deletes the model dir;
* ``per_device_batch_size`` -- divisibility check for intra-member data parallelism;
* ``get_distribution_strategy`` -- which parallel layout a member uses.  The
  reference hard-wires one GPU per member (``resnet_run_loop.py:390-392``); here
  ``num_gpus > 1`` selects intra-member data parallelism with an RCCL all-reduce
  of the flat gradient row (``parallel/member_dp.py``).
"""

from __future__ import annotations

import numbers
import os
import shutil

import torch


def past_stop_threshold(stop_threshold, eval_metric) -> bool:
    if stop_threshold is None:
        return False
    if not isinstance(stop_threshold, numbers.Number):
        raise ValueError("Threshold for checking stop conditions must be a number.")
    if not isinstance(eval_metric, numbers.Number):
        raise ValueError("Eval metric being checked against stop conditions must be a number.")
    if eval_metric >= stop_threshold:
        print("Stop threshold of {} was passed with metric value {}.".format(stop_threshold, eval_metric))
        return True
    return False


def generate_synthetic_data(input_shape, input_value=0, input_dtype=torch.float32, label_shape=None, label_value=0,
                            label_dtype=torch.int64, device="cpu"):
    x = torch.full(tuple(input_shape), input_value, dtype=input_dtype, device=device)
    if label_shape is None:
        return x
    y = torch.full(tuple(label_shape), label_value, dtype=label_dtype, device=device)
    return x, y


def apply_clean(flags_obj) -> None:
    if getattr(flags_obj, "clean", False) and os.path.isdir(flags_obj.model_dir):
        print("--clean flag set. Removing existing model dir: {}".format(flags_obj.model_dir))
        shutil.rmtree(flags_obj.model_dir)


def per_device_batch_size(batch_size: int, num_gpus: int) -> int:
    if num_gpus <= 1:
        return batch_size
    remainder = batch_size % num_gpus
    if remainder:
        raise ValueError("When running with multiple GPUs, batch size must be a multiple of the number of available "
                         "GPUs. Found {} GPUs with a batch size of {}; try --batch_size={} instead."
                         .format(num_gpus, batch_size, batch_size - remainder))
    return batch_size // num_gpus


def get_distribution_strategy(num_gpus: int, all_reduce_alg: str = None) -> dict:
    if num_gpus == 0:
        return {"kind": "one_device", "device": "cpu"}
    if num_gpus == 1:
        return {"kind": "one_device", "device": "cuda:0"}
    return {"kind": "member_data_parallel", "num_gpus": num_gpus, "all_reduce": all_reduce_alg or "rccl_ring"}
