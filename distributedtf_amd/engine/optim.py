"""Population optimizer: TF1 optimizer semantics over flat ``[G, P]`` buffers.

The reference builds one of six TF1 optimizers per member
(``resnet_run_loop.py:552-586``, ``mnist_model.py:27-60``) and TF launches one
``Apply*`` kernel per variable.  Here every member's parameters, gradients and
two optimizer slots are rows of flat buffers and ONE fused HIP kernel
(``ops/csrc/optim.hip``) updates the whole population: per-member optimizer
code, learning rate, momentum, decay and regularizer are read from a small
``[G, 8]`` hyper table, so a different lr/optimizer per member costs nothing and
the launch can be captured in a HIP graph.

``apply_reference`` is the plain PyTorch oracle with identical math:

=========  ==================================================================
gd         w -= lr g
Momentum   a = mu a + g ;  w -= lr a
Adam       lr_t = lr sqrt(1-b2^t)/(1-b1^t); m,v EMA; w -= lr_t m/(sqrt(v)+1e-8)
Adagrad    a += g^2 (a0 = 0.1) ;  w -= lr g / sqrt(a)
Adadelta   a = .95a+.05g^2; u = sqrt(au+1e-8)/sqrt(a+1e-8) g; au = .95au+.05u^2; w -= lr u
RMSProp    ms = d ms + (1-d) g^2 (ms0 = 1); m = mu m + lr g/sqrt(ms+1e-10); w -= m
=========  ==================================================================

Regularizer (conv-kernel prefix ``[0, n_reg)`` only): l2 adds ``wd*w``, l1 adds
``wd*sign(w)``, l1_l2 both -- the gradients of TF1's ``l2_loss``-based contrib
regularizers.
"""

from __future__ import annotations

from typing import Dict, Optional

import torch

OPT_CODES = {"gd": 0, "Momentum": 1, "Adam": 2, "Adagrad": 3, "Adadelta": 4, "RMSProp": 5}
REG_CODES = {None: 0, "None": 0, "l1_regularizer": 1, "l2_regularizer": 2, "l1_l2_regularizer": 3}

# columns of the per-member hyper table
H_OPT, H_LR, H_MOM, H_DECAY, H_WD, H_REG, H_STEP, H_ACTIVE = range(8)
N_HYPER = 8

ADAM_B1, ADAM_B2, ADAM_EPS = 0.9, 0.999, 1e-8
ADADELTA_RHO, ADADELTA_EPS = 0.95, 1e-8
RMSPROP_EPS = 1e-10
ADAGRAD_INIT = 0.1


def slot_init_values(optimizer: str):
    """Initial values of (slot1, slot2) for a freshly created member."""
    if optimizer == "Adagrad":
        return ADAGRAD_INIT, 0.0
    if optimizer == "RMSProp":
        return 1.0, 0.0
    return 0.0, 0.0


def hyper_row(hparams: Dict, lr: float, step: int, active: bool = True):
    opt = hparams["opt_case"]
    name = opt["optimizer"]
    return [float(OPT_CODES[name]), float(lr), float(opt.get("momentum", 0.0)), float(opt.get("grad_decay", 0.0)),
            float(hparams.get("weight_decay", 0.0)), float(REG_CODES.get(hparams.get("regularizer"), 0)),
            float(step), 1.0 if active else 0.0]


def _reg_grad(w, g, n_reg, wd, reg):
    if reg == 0 or n_reg == 0:
        return g
    g = g.clone()
    wr = w[:n_reg]
    if reg in (2, 3):
        g[:n_reg] += wd * wr
    if reg in (1, 3):
        g[:n_reg] += wd * torch.sign(wr)
    return g


@torch.no_grad()
def apply_reference(params: torch.Tensor, grads: torch.Tensor, slot1: torch.Tensor, slot2: torch.Tensor,
                    hyper: torch.Tensor, n_reg: int, rows: Optional[list] = None) -> None:
    """In-place update of ``params/slot1/slot2`` rows ([G, P] fp32)."""
    G = params.shape[0]
    hy = hyper.detach().to("cpu", torch.float64)
    for gi in range(G) if rows is None else rows:
        h = hy[gi]
        if h[H_ACTIVE] == 0:
            continue
        code, lr, mu, dec, wd, reg, t = int(h[H_OPT]), h[H_LR].item(), h[H_MOM].item(), h[H_DECAY].item(), \
            h[H_WD].item(), int(h[H_REG]), h[H_STEP].item()
        w, a, b = params[gi], slot1[gi], slot2[gi]
        g = _reg_grad(w, grads[gi].float(), n_reg, wd, reg)
        if code == 0:
            w.sub_(lr * g)
        elif code == 1:
            a.mul_(mu).add_(g)
            w.sub_(lr * a)
        elif code == 2:
            lr_t = lr * (1.0 - ADAM_B2 ** t) ** 0.5 / (1.0 - ADAM_B1 ** t)
            a.mul_(ADAM_B1).add_((1.0 - ADAM_B1) * g)
            b.mul_(ADAM_B2).add_((1.0 - ADAM_B2) * g * g)
            w.sub_(lr_t * a / (b.sqrt() + ADAM_EPS))
        elif code == 3:
            a.add_(g * g)
            w.sub_(lr * g * a.rsqrt())
        elif code == 4:
            a.mul_(ADADELTA_RHO).add_((1.0 - ADADELTA_RHO) * g * g)
            upd = (b + ADADELTA_EPS).sqrt() * (a + ADADELTA_EPS).rsqrt() * g
            b.mul_(ADADELTA_RHO).add_((1.0 - ADADELTA_RHO) * upd * upd)
            w.sub_(lr * upd)
        elif code == 5:
            a.mul_(dec).add_((1.0 - dec) * g * g)
            b.mul_(mu).add_(lr * g * (a + RMSPROP_EPS).rsqrt())
            w.sub_(b)
        else:
            raise ValueError("unknown optimizer code %d" % code)


# TF1 optimizer slot variable names (tf.train.*Optimizer._create_slots): slot1 / slot2 of the flat state
TF_SLOT_NAMES = {
    "gd": (None, None),
    "Momentum": ("Momentum", None),
    "Adam": ("Adam", "Adam_1"),
    "Adagrad": ("Adagrad", None),
    "Adadelta": ("Adadelta", "Adadelta_1"),
    "RMSProp": ("RMSProp", "RMSProp_1"),
}


def tf_optimizer_tensors(optimizer: str, trainable, step: int):
    """Slot tensors (``<var>/<Slot>``) + optimizer non-slot variables of a TF1 checkpoint.

    ``trainable``: iterable of (name, value, slot1_value, slot2_value) with numpy arrays already in TF layout."""
    import numpy as np
    n1, n2 = TF_SLOT_NAMES.get(optimizer, (None, None))
    out = {}
    for name, _, s1, s2 in trainable:
        if n1:
            out["%s/%s" % (name, n1)] = s1
        if n2:
            out["%s/%s" % (name, n2)] = s2
    if optimizer == "Adam":  # AdamOptimizer's beta powers after `step` updates
        out["beta1_power"] = np.array(0.9 ** step, dtype=np.float32)
        out["beta2_power"] = np.array(0.999 ** step, dtype=np.float32)
    out["global_step"] = np.array(step, dtype=np.int64)
    return out
