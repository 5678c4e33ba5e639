"""Export of a trained member (reference ``official/utils/export/export.py`` +
``resnet_run_loop.py:510-514`` SavedModel export).

``export_member`` writes ``<export_dir>/`` with the member's inference weights
(safetensors: flat params + BN running stats), its hyper-parameters and an
input signature (``serving_input_spec``), loadable without pickle.
"""

from __future__ import annotations

import json
import os
from typing import Dict, Sequence


def serving_input_spec(shape: Sequence[int], dtype: str = "float32", batch_size=None) -> Dict:
    """Reference ``build_tensor_serving_input_receiver_fn``: NHWC input placeholder."""
    return {"name": "input_tensor", "shape": [batch_size] + list(shape), "dtype": dtype}


def export_member(member, export_dir: str) -> str:
    from safetensors.torch import save_file
    os.makedirs(export_dir, exist_ok=True)
    eng = member.engine
    tensors = {"params": eng.params[member.slot].detach().cpu().contiguous(),
               "bn_running": eng.running[member.slot].detach().cpu().contiguous()}
    save_file(tensors, os.path.join(export_dir, "model.safetensors"))
    meta = {"arch": member.arch.name, "model_id": member.cluster_id, "hparams": member.hparams,
            "global_step": member.global_step, "accuracy": member.accuracy,
            "input": serving_input_spec(member.arch.input_shape)}
    with open(os.path.join(export_dir, "model.json"), "w") as f:
        json.dump(meta, f, indent=2, sort_keys=True)
    return export_dir


def load_exported(export_dir: str):
    from safetensors.torch import load_file
    t = load_file(os.path.join(export_dir, "model.safetensors"))
    with open(os.path.join(export_dir, "model.json")) as f:
        meta = json.load(f)
    return t, meta
