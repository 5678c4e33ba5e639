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
                            c_float, c_void_p],
    "dtf_shadow_refresh": [c_void_p, c_void_p, c_void_p, c_int, c_long, c_long, c_long, c_void_p],
    "dtf_step_advance": [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_int, c_void_p],
    "dtf_step_end": [c_void_p, c_long, c_long, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_int, c_void_p],
}


def register(name, argtypes):
    _SIGNATURES[name] = argtypes


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            # DTF_LIB: an alternative build of the same sources (e.g. timing-only ablation builds of tools/)
            debug = debug_mode()
            det = deterministic_mode()
            half = half_mode()
            if half and debug:
                raise RuntimeError("DTF_HALF=1 (fp16 kernels) has no debug build")
            default = (_build.LIB_DEBUG if debug else
                       (_build.LIB_HALF_DET if half and det else
                        (_build.LIB_DET if det else (_build.LIB_HALF if half else _build.LIB))))
            path = os.environ.get("DTF_LIB") or default
            if path == default and (not os.path.isfile(path) or
                                    (os.environ.get("DTF_REBUILD") == "1" and _build.needs_build(path))):
                if debug:
                    _build.build_debug(verbose=False)
                elif half and det:
                    _build.build_half_det(verbose=False)
                elif det:
                    _build.build_det(verbose=False)
                elif half:
                    _build.build_half(verbose=False)
                else:
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
            _LIB = _DebugLib(L) if debug else L
    return _LIB


def build_nrep() -> int:
    """BatchNorm-statistic replicas compiled into the loaded library (``dtf_nrep``)."""
    fn = lib().dtf_nrep
    fn.argtypes, fn.restype = [], c_int
    return int(fn())


def build_deterministic() -> bool:
    """True if the loaded library is the deterministic build (``dtf_build_deterministic``)."""
    fn = lib().dtf_build_deterministic
    fn.argtypes, fn.restype = [], c_int
    return bool(fn())


def build_half() -> bool:
    """True if the loaded library is the half build (fp16 storage, ``dtf_build_half``)."""
    fn = lib().dtf_build_half
    fn.argtypes, fn.restype = [], c_int
    return bool(fn())


def half_mode() -> bool:
    """DTF_HALF=1 (set by ``--dtype fp16``): load the fp16 build of the kernels (common.h DTF_HALF).  The library is
    one per process, like the deterministic build: a process runs either bf16 or fp16 HIP steps."""
    return os.environ.get("DTF_HALF", "0") == "1"


def act_dtype():
    """torch dtype of the kernels' 16-bit tensors (activations, weight shadows) in this process."""
    import torch
    return torch.float16 if half_mode() else torch.bfloat16


def deterministic_mode() -> bool:
    """DTF_DETERMINISTIC=1 (set by ``--deterministic``): the deterministic kernel build (64 statistic replicas) and
    workgroup caps that make every reduction order fixed (engine/hip_resnet.py)."""
    return os.environ.get("DTF_DETERMINISTIC", "0") == "1"


def debug_mode() -> bool:
    """DTF_DEBUG=1 (set by ``--debug_kernels``): load the debug build and check every launch synchronously."""
    return os.environ.get("DTF_DEBUG", "0") == "1"


class _DebugLib:
    """Debug-mode view of the kernel library.

    Every ``dtf_*`` launcher call is followed by a device synchronisation and a read of the per-source device
    error words (``dtf_debug_error_<tu>``): a failed workgroup check, a failed host-side argument check (return
    code >= 100000) or an asynchronous HIP error is raised as a RuntimeError naming the launcher, at the launch that
    caused it instead of at some later synchronisation.  HIP-graph capture is off in this mode (flags.py).
    """

    def __init__(self, L):
        self._L = L
        self._err_fns = []
        self.launches = 0

    def _error_words(self):
        if not self._err_fns:
            import glob as _glob
            names = [os.path.basename(p)[:-4] for p in _glob.glob(os.path.join(_build.CSRC, "*.hip"))]
            for n in names:
                fn = getattr(self._L, "dtf_debug_error_" + n, None)
                if fn is not None:
                    fn.argtypes = []
                    fn.restype = c_int
                    self._err_fns.append((n, fn))
        return self._err_fns

    def __getattr__(self, name):
        fn = getattr(self._L, name)
        if (not name.startswith("dtf_") or name.startswith("dtf_debug_") or name.endswith("_size")
                or name in ("dtf_crc32c", "dtf_nrep", "dtf_build_deterministic") or not torch.cuda.is_available()):
            return fn
        return _CheckedLaunch(self, name, fn)


def launcher_name(fn) -> str:
    """Symbol name of a library launcher (a ctypes function or a debug-mode _CheckedLaunch)."""
    return fn._o[1] if isinstance(fn, _CheckedLaunch) else fn.__name__


class _CheckedLaunch:
    """A launcher of the debug library: calls through, then synchronises and checks (see _DebugLib).
    ``argtypes`` / ``restype`` read and write the underlying ctypes function."""

    def __init__(self, owner, name, fn):
        object.__setattr__(self, "_o", (owner, name, fn))

    def __getattr__(self, attr):
        return getattr(self._o[2], attr)

    def __setattr__(self, attr, value):
        setattr(self._o[2], attr, value)

    def __call__(self, *args):
        owner, name, fn = self._o
        rc = fn(*args)
        owner.launches += 1
        if isinstance(rc, int) and rc >= 100000:
            raise RuntimeError("%s: host-side argument check failed (csrc line %d)" % (name, rc - 100000))
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError("%s: asynchronous HIP error after launch: %s" % (name, e)) from e
        for tu, ef in owner._error_words():
            v = ef()
            if v > 0:
                raise RuntimeError("%s: device check failed in %s.hip line %d" % (name, tu, v))
        return rc


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


def fused_optimizer(state, grads, hyper, Pp, P, n_reg, shadow=None, zero_grads=True, grad_scale=1.0):
    """One launch: TF1-semantics optimizer step for every member row (see optim.hip).  ``grad_scale`` multiplies every
    gradient first (1 / loss_scale: the fp16 mode's static loss scaling, resnet_run_loop.py:284-294)."""
    assert state.is_cuda and state.dtype == torch.float32 and state.is_contiguous()
    assert grads.shape[1] == Pp and hyper.shape[1] == 8
    G = state.shape[0]
    if shadow is not None:
        assert shadow.dtype in (torch.bfloat16, torch.float16) and shadow.shape[1] == Pp
    check(lib().dtf_fused_optimizer(ptr(state), ptr(grads), ptr(hyper), ptr(shadow), G, state.shape[1], Pp, P, n_reg,
                                    1 if zero_grads else 0, float(grad_scale), stream()), "fused_optimizer")


def shadow_refresh(state, shadow, rows, Pp, P):
    rows_t = torch.as_tensor(list(rows), dtype=torch.int32).to(state.device, non_blocking=True)
    check(lib().dtf_shadow_refresh(ptr(state), ptr(shadow), ptr(rows_t), len(rows), state.shape[1], Pp, P, stream()),
          "shadow_refresh")
    return rows_t


register("dtf_augment_cifar", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_long, c_long, c_void_p])


def augment_cifar(images, labels, idx, rng, augment=True, out16=None, out32=None, lab32=None, lab64=None,
                  member_keys=None):
    """Fused gather + pad/crop/flip + per-image standardization (data.hip).

    images [N,32,32,3] uint8, labels [N] int64, idx [n] int64 (dataset rows), rng [2] int32 (seed, counter; read
    on the device, so graph replays pick up updates).  Writes any of out16 [n,32,32,16] bf16 / out32 [n,32,32,3]
    fp32 / lab32 [n] int32 / lab64 [n] int64.  ``member_keys`` = (img_slot [n] int32, state, row stride, step column):
    crops keyed by each image's member step counter and dataset row instead of the launch counter and batch
    position (placement-invariant population steps, data.hip).
    """
    assert images.dtype == torch.uint8 and tuple(images.shape[1:]) == (32, 32, 3) and images.is_contiguous()
    assert labels.dtype == torch.int64 and idx.dtype == torch.int64 and rng.numel() >= 2
    n = int(idx.numel())
    for t, shp, dt in ((out16, (32, 32, 16), act_dtype()), (out32, (32, 32, 3), torch.float32)):
        if t is not None:
            assert t.dtype == dt and t.shape[0] >= n and tuple(t.shape[1:]) == shp and t.is_contiguous()
    for t, dt in ((lab32, torch.int32), (lab64, torch.int64)):
        if t is not None:
            assert t.dtype == dt and t.numel() >= n
    ks, kst, kstride, kcol = member_keys if member_keys is not None else (None, None, 0, 0)
    if ks is not None:
        assert ks.dtype == torch.int32 and ks.numel() >= n and kst.dtype == torch.float32
    check(lib().dtf_augment_cifar(ptr(images), ptr(labels), ptr(idx), ptr(rng), n, 1 if augment else 0, ptr(out16),
                                  ptr(out32), ptr(lab32), ptr(lab64), ptr(ks), ptr(kst), int(kstride), int(kcol),
                                  stream()), "augment_cifar")
