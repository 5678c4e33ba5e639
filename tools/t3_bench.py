"""Microbenchmark of the stride-1 3x3 conv kernel (ops/csrc/convg.hip convg_t3_kernel) at the ResNet-50 shapes.

    python tools/t3_bench.py [--lib tools/abl/libX.so] [--hw 28] [--ci 128] [--dgrad] [--flags 1] [--iters 20]

One launch over pop 8 x 128 images (the product step's batch), weights per member, timed with HIP events (median of
--iters).  Prints us per launch and the achieved dense TFLOP/s.  With --ci above the layer's real width, the time
difference against the real width is the k-loop cost of the extra channels: the rest is per-workgroup overhead
(prologue staging, epilogue, statistics).  --stamps (a -DDTF_STAMP=1 build) prints the per-workgroup phases of
one launch: S0 entry -> S1 first chunk staged -> S2 k loop done -> S3 epilogue done -> S4 stores drained, and the
share of the grid's workgroup-slot time (2 per CU) each phase takes.
"""
import argparse
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--hw", type=int, default=28)
    ap.add_argument("--ci", type=int, default=0, help="input channels (default: the layer's)")
    ap.add_argument("--co", type=int, default=0)
    ap.add_argument("--dgrad", action="store_true")
    ap.add_argument("--flags", type=int, default=1)
    ap.add_argument("--images", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stamps", action="store_true", help="DTF_STAMP build: per-workgroup phases of one launch")
    args = ap.parse_args()
    if args.lib:
        os.environ["DTF_LIB"] = os.path.abspath(args.lib)
    import torch
    from distributedtf_amd import ops
    from distributedtf_amd.engine import hip_imagenet as hi
    hi._register()
    L = ops.lib()
    dev = torch.device("cuda")
    hw = args.hw
    width = {56: 64, 28: 128, 14: 256}[hw]
    ci, co = args.ci or width, args.co or width
    tc = 64 if hw == 56 else 128
    rows = hi._CG_T3[hw]
    n, pop = args.images, 8
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, hw, hw, ci, device=dev, generator=g).bfloat16()
    if args.dgrad:  # A from the forward layout W[o][tap][i]: rows = this launch's outputs (ci of the forward)
        w = (torch.randn(pop, ci, 9, co, device=dev, generator=g) * 0.02).bfloat16()
    else:
        w = (torch.randn(pop, co, 9, ci, device=dev, generator=g) * 0.02).bfloat16()
    xm = torch.randn(n, hw, hw, co, device=dev, generator=g).bfloat16()
    ep = torch.zeros(pop, 4, 512, device=dev)
    ep[:, 0] = 1.0
    ep[:, 3] = 1.0
    y = torch.empty(n, hw, hw, co, dtype=torch.bfloat16, device=dev)
    st = torch.zeros(pop, 2, 512, device=dev, dtype=torch.float64)  # 8 bytes per sum covers either accumulator type
    per = n // pop
    items = []
    for img in range(n):
        for y0 in range(0, hw, rows):
            p0 = (img * hw + y0) * hw
            for o0 in range(0, co, tc):
                items.append([img // per, p0, p0 + rows * hw, o0])
    work = torch.tensor(items, dtype=torch.int32, device=dev)
    a = hi.CgArgs()
    a.x, a.y, a.w, a.work, a.st_out = x.data_ptr(), y.data_ptr(), w.data_ptr(), work.data_ptr(), st.data_ptr()
    a.w_mstride, a.w_off = co * 9 * ci, 0
    a.Hi = a.Wi = a.Ho = a.Wo = hw
    a.Ci, a.Co = ci, co
    a.kh = a.kw = 3
    a.stride, a.pad = 1, 1
    a.cmax = 512
    a.log2ci = ci.bit_length() - 1
    a.flags = args.flags
    if args.dgrad:
        a.xm, a.c_ep = xm.data_ptr(), ep.data_ptr()
    assert ci % 32 == 0 and co % tc == 0 and ci <= 512 and co <= 512

    def launch():
        rc = L.dtf_convg_t3(ctypes.byref(a), tc, 6 if args.dgrad else 4, int(args.dgrad), hw, work.shape[0], 0,
                            ops.stream())
        assert rc == 0, rc

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        launch()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    us = statistics.median(ts)
    flop = 2.0 * n * hw * hw * co * 9 * ci
    print("t3 hw %d ci %d co %d %s flags %d: %.1f us  %.0f TFLOP/s  (%d workgroups)"
          % (hw, ci, co, "dgrad" if args.dgrad else "fwd", args.flags, us, flop / us * 1e-6, work.shape[0]))
    if args.stamps:
        import numpy as np
        nwg = work.shape[0]
        buf = np.zeros((8192, 8), dtype=np.uint64)
        launch()
        torch.cuda.synchronize()
        assert L.dtf_t3_stamp_read(ctypes.c_void_p(buf.ctypes.data), ctypes.c_long(buf.nbytes)) == 0, "not a stamp build"
        st = buf[:min(nwg, 8192)].astype(np.int64)
        t0 = st[:, 0].min()
        span = (st[:, 4].max() - t0) / 100.0
        ph = [(st[:, i + 1] - st[:, i]) / 100.0 for i in range(4)]
        busy = sum(p.sum() for p in ph)
        slots = 512.0
        print("  span %.1f us; phase medians (us) prologue %.2f  k-loop %.2f  epilogue %.2f  drain %.2f" %
              ((span,) + tuple(float(np.median(p)) for p in ph)))
        print("  share of slot time (%d slots x span): prologue %.1f%%  k-loop %.1f%%  epilogue %.1f%%  drain %.1f%%  "
              "idle %.1f%%" % ((slots,) + tuple(100.0 * p.sum() / (slots * span) for p in ph) +
                               (100.0 * (1 - busy / (slots * span)),)))
        # dispatch: when did each round of 512 workgroups start (median entry per round, relative to t0)
        rounds = [float(np.median(st[r:r + 512, 0] - t0)) / 100.0 for r in range(0, len(st), 512)]
        print("  round entry medians (us): " + " ".join("%.1f" % r for r in rounds))
        cu = (st[:, 6].astype(np.int64) << 8) | ((st[:, 5] >> 8) & 0xF) | (((st[:, 5] >> 13) & 0x7) << 4)
        print("  distinct (xcc, se, cu) ids: %d" % len(set(cu.tolist())))


if __name__ == "__main__":
    main()
