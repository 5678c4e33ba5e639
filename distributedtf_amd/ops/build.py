"""Build the gfx950 kernel library ``ops/libdtf_kernels.so`` in-tree with hipcc.

The library is a plain C ABI (``extern "C" dtf_*`` launchers taking raw device
pointers and a ``hipStream_t``) loaded with ctypes -- no hipify, no torch
extension headers, no JIT cache outside the repo.  ``python -m
distributedtf_amd.ops.build`` (or ``__graft_entry__.build()``) rebuilds it when a
source is newer than the library.
"""

from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdtf_kernels.so")
# Debug build of the same sources (-DDTF_DEBUG: workgroup-uniform device checks that record and skip instead of
# trapping, host-side launch-argument checks; -g).  Loaded instead of LIB when DTF_DEBUG=1 (ops.lib()).
LIB_DEBUG = os.path.join(HERE, "libdtf_kernels_debug.so")
DEBUG_FLAGS = ["-DDTF_DEBUG=1", "-g"]
# Deterministic build (--deterministic / DTF_DETERMINISTIC=1): 64 BatchNorm-statistic replicas, so that with at
# most 64 workgroups per member per launch (engine/hip_resnet.py caps them) every replica receives at most one
# atomic add onto zero and the consumers sum the replicas in a fixed order -- bitwise-replayable statistics.
LIB_DET = os.path.join(HERE, "libdtf_kernels_det.so")
DET_FLAGS = ["-DDTF_DETERMINISTIC=1", "-DDTF_NREP=64"]
# Half build (--dtype fp16 / DTF_HALF=1): the same kernels for IEEE fp16 activation / weight-shadow storage and
# v_mfma_f32_16x16x32_f16 (common.h DTF_HALF); the static loss scale of the reference's fp16 mode is applied by the
# head (dlogits x S) and removed by the fused optimizer (grads x 1/S)
LIB_HALF = os.path.join(HERE, "libdtf_kernels_f16.so")
HALF_FLAGS = ["-DDTF_HALF=1"]
# Deterministic half build (--dtype fp16 --deterministic): the half kernels with the deterministic build's fixed-order
# reductions (DTF_HALF + DTF_DETERMINISTIC; the two switches are orthogonal in common.h)
LIB_HALF_DET = os.path.join(HERE, "libdtf_kernels_f16_det.so")
ARCH = os.environ.get("DTF_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def needs_build(lib=LIB) -> bool:
    if not os.path.isfile(lib):
        return True
    t = os.path.getmtime(lib)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h"))
    return any(os.path.getmtime(s) > t for s in deps)


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isfile(c) or c == "hipcc"):
            return c
    return "hipcc"


def build(force: bool = False, verbose: bool = True, extra_flags=None, out: str = LIB) -> str:
    if not force and not needs_build(out):
        return out
    objs = []
    procs = []
    for src in sources():
        # per-process and per-library object names: the three libraries may build concurrently
        obj = os.path.join(CSRC, "%s.%d.%s.o" % (os.path.basename(src), os.getpid(), os.path.basename(out)))
        cmd = [hipcc(), "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
               "-Wno-unused-result", "-munsafe-fp-atomics"] + list(extra_flags or [])
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        objs.append(obj)
    failed = False
    for src, p in procs:
        log, _ = p.communicate()
        if p.returncode != 0:
            failed = True
            sys.stderr.write(log.decode(errors="replace"))
            sys.stderr.write("\nhipcc failed on %s\n" % src)
        elif verbose and log.strip():
            sys.stderr.write(log.decode(errors="replace"))
    if failed:
        raise RuntimeError("kernel build failed")
    tmp = out + ".tmp"
    subprocess.check_call([hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs)
    os.replace(tmp, out)
    for o in objs:
        try:
            os.remove(o)
        except OSError:
            pass
    if verbose:
        sys.stderr.write("built %s\n" % out)
    return out


def build_debug(force: bool = False, verbose: bool = True) -> str:
    return build(force=force, verbose=verbose, extra_flags=DEBUG_FLAGS, out=LIB_DEBUG)


def build_det(force: bool = False, verbose: bool = True) -> str:
    return build(force=force, verbose=verbose, extra_flags=DET_FLAGS, out=LIB_DET)


def build_half(force: bool = False, verbose: bool = True) -> str:
    return build(force=force, verbose=verbose, extra_flags=HALF_FLAGS, out=LIB_HALF)


def build_half_det(force: bool = False, verbose: bool = True) -> str:
    return build(force=force, verbose=verbose, extra_flags=HALF_FLAGS + DET_FLAGS, out=LIB_HALF_DET)


if __name__ == "__main__":
    if "--debug" in sys.argv:
        build_debug(force="--force" in sys.argv)
    elif "--half" in sys.argv and "--det" in sys.argv:
        build_half_det(force="--force" in sys.argv)
    elif "--det" in sys.argv:
        build_det(force="--force" in sys.argv)
    elif "--half" in sys.argv:
        build_half(force="--force" in sys.argv)
    else:
        build(force="--force" in sys.argv)
