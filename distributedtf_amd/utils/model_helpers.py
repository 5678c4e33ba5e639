"""``past_stop_threshold`` (reference ``official/utils/misc/model_helpers.py:26-53``), called by
``EngineModel._train_cycle`` after every eval (``resnet_run_loop.py:505-508``).

The reference's other helpers have product-side equivalents elsewhere: synthetic data is
``data/datasets.py`` (device-resident synthetic pools), intra-member data parallelism and its batch split are
``parallel/dataparallel.py`` (``DPContext.local_batch`` allows uneven splits, so no divisibility check is needed),
and the model directory is cleaned by ``main_manager.py`` at start-up.
"""

from __future__ import annotations

import numbers


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
