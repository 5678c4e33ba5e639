"""Timing-only ablation builds of the kernel library (conv_bwd_fused_kernel phases switched off via DTF_ABL).

    python tools/build_ablations.py 1 2 4        -> tools/abl/libdtf_abl{1,2,4}.so
    DTF_LIB=tools/abl/libdtf_abl1.so python bench.py ...   (outputs are WRONG; read the time only)
bits: 1 = no dW slab stores, 2 = no wgrad MFMA loop, 4 = no dgrad MFMAs / epilogue."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedtf_amd.ops import build as kb  # noqa: E402

if __name__ == "__main__":
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "abl")
    os.makedirs(here, exist_ok=True)
    for b in sys.argv[1:]:
        kb.build(force=True, extra_flags=["-DDTF_ABL=%d" % int(b)], out=os.path.join(here, "libdtf_abl%s.so" % b))
