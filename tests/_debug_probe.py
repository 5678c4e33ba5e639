"""Run under DTF_DEBUG=1 by tests/test_debug_sanitize.py (GPU): the debug kernel library catches a bad launch on
the host, a bad work item on the device (recorded, workgroup skipped -- no trap), and runs a full ResNet-56
population step with every launch checked."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
assert os.environ.get("DTF_DEBUG") == "1"

import torch  # noqa: E402

from distributedtf_amd import ops  # noqa: E402
from distributedtf_amd.engine import hip_resnet as hr  # noqa: E402


def expect_error(fn, text):
    try:
        fn()
    except RuntimeError as e:
        assert text in str(e), str(e)
        return
    raise AssertionError("expected a RuntimeError containing %r" % text)


hr._register()
L = ops.lib()
assert isinstance(L, ops._DebugLib), type(L)
maps = open("/proc/self/maps").read()
assert "libdtf_kernels_debug.so" in maps, "debug library not loaded"

dev = torch.device("cuda:0")
st = ops.stream()
x = torch.zeros(1, 32, 32, 16, dtype=torch.bfloat16, device=dev)
y = torch.zeros_like(x)
w = torch.zeros(16 * 9 * 16, dtype=torch.bfloat16, device=dev)
img_slot = torch.zeros(1, dtype=torch.int32, device=dev)
cnt = torch.ones(1, dtype=torch.float32, device=dev)
# slot -1: an invalid item (an empty item, nit = 0, is legal since elastic plans generate them)
work = torch.tensor([[0, 1, 0, -1]], dtype=torch.int32, device=dev)

a = hr.ConvArgs()
a.x, a.y, a.w = x.data_ptr(), y.data_ptr(), w.data_ptr()
a.img_slot, a.cnt, a.work = img_slot.data_ptr(), cnt.data_ptr(), work.data_ptr()
# 1) host-side argument check: zero spatial dims never reach the GPU
expect_error(lambda: L.dtf_conv_fwd_s1(ctypes.byref(a), 16, 0, 0, 0, 1, 65536, st), "host-side argument check")
# 2) device-side workgroup check: the item is rejected before any tensor access, recorded and reported
a.Hi = a.Wi = a.Ho = a.Wo = 32
a.rows = 8
expect_error(lambda: L.dtf_conv_fwd_s1(ctypes.byref(a), 16, 0, 0, 8, 1, 65536, st), "device check failed in conv.hip")
torch.cuda.synchronize()
# 3) a real population step with every launch checked
import __graft_entry__  # noqa: E402

n0 = L.launches
__graft_entry__.smoke()
assert L.launches - n0 > 50, L.launches - n0
print("debug probe ok: %d checked launches" % (L.launches - n0))
