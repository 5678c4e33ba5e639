"""Python bindings for the hand-written gfx950 kernels (``ops/csrc/*.hip``).

The kernels are compiled in-tree into ``libdtf_kernels.so`` (``ops/build.py``) and
called through ctypes with raw device pointers on PyTorch's current HIP stream,
so they interleave with (and are captured in HIP graphs together with) torch
work.  On a GPU box a missing / unbuildable library is a hard error -- there is
no silent eager fallback for an op that was asked to run on the HIP path.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch

from . import build as _build

_LOCK = threading.Lock()
_LIB = None

c_void_p, c_int, c_long, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float

# name -> argtypes (all return int = hipError_t of the launch)
_SIGNATURES = {
    "dtf_fused_optimizer": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_long, c_long, c_long, c_long, c_int,
                            c_void_p],
    "dtf_shadow_refresh": [c_void_p, c_void_p, c_void_p, c_int, c_long, c_long, c_long, c_void_p],
}


def register(name, argtypes):
    _SIGNATURES[name] = argtypes


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            path = _build.LIB
            if not os.path.isfile(path) or (os.environ.get("DTF_REBUILD") == "1" and _build.needs_build()):
                _build.build(verbose=False)
            if not os.path.isfile(path):
                raise RuntimeError("distributedtf_amd kernel library missing: %s" % path)
            L = ctypes.CDLL(path)
            for name, args in _SIGNATURES.items():
                fn = getattr(L, name, None)
                if fn is None:
                    continue
                fn.argtypes = args
                fn.restype = c_int
            _LIB = L
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


def stream():
    return c_void_p(torch.cuda.current_stream().cuda_stream)


def check(err, name):
    if err != 0:
        raise RuntimeError("%s launch failed: hipError %d" % (name, err))


def fused_optimizer(state, grads, hyper, Pp, P, n_reg, shadow=None, zero_grads=True):
    """One launch: TF1-semantics optimizer step for every member row (see optim.hip)."""
    assert state.is_cuda and state.dtype == torch.float32 and state.is_contiguous()
    assert grads.shape[1] == Pp and hyper.shape[1] == 8
    G = state.shape[0]
    if shadow is not None:
        assert shadow.dtype == torch.bfloat16 and shadow.shape[1] == Pp
    check(lib().dtf_fused_optimizer(ptr(state), ptr(grads), ptr(hyper), ptr(shadow), G, state.shape[1], Pp, P, n_reg,
                                    1 if zero_grads else 0, stream()), "fused_optimizer")


def shadow_refresh(state, shadow, rows, Pp, P):
    rows_t = torch.as_tensor(list(rows), dtype=torch.int32).to(state.device, non_blocking=True)
    check(lib().dtf_shadow_refresh(ptr(state), ptr(shadow), ptr(rows_t), len(rows), state.shape[1], Pp, P, stream()),
          "shadow_refresh")
    return rows_t
