"""HBM-byte floor of the HIP ImageNet ResNet-50 v2 training step (engine/hip_imagenet.py launch structure).

Counts, per launch of the population step, the activation bytes it must move through HBM at least once (every
tensor read or written by that launch, NHWC bf16; weights, BN tables and L2 re-reads of a 3x3 halo ignored) and
compares the sum with the measured per-family GPU time of a kernel trace:

    python tools/imagenet_roofline.py [--n 1024] [--bw 6.3] [--top N] [gpurun_out/prof/run_kernel_trace.csv]

``--bw`` is the achievable HBM bandwidth (TB/s; MI355X: 6.3 measured for a float4 copy, 8.0 spec).  The output
lists bytes and floor time per launch family and, with a trace, the measured time per step of the same family.
Reference workload: resnet/resnet_model.py:267-320 (bottleneck v2), imagenet_main.py (ResNet-50, 224x224).
"""

from __future__ import annotations

import argparse
import collections
import csv
import sys

STAGES = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]  # (filters, blocks, first stride)


def launches(N: int, H: int = 224, fold1_maxc: int = 256, compact_pd: bool = True):
    """(family, label, bytes, flops) of every launch of one training step that moves activations, in the plan's
    execution order (engine/hip_imagenet.py _build).  ``fold1_maxc``: blocks without a projection whose conv1 has at
    most that many output channels apply BN1 + ReLU inside conv1 (CG_FOLD1: no "ax" pass); ``compact_pd``: a
    stride-2 projection's data gradient is stored at the dy resolution (CG_COMPACT_PD).  0 / False: the plain path."""
    B = 2 * N  # bytes per (pixel, channel) element over the population batch
    out = []
    H1, H2 = H // 2, H // 4
    out.append(("prep_input", "input", N * H * H * (3 * 4 + 4 * 2), 0))  # fp32 image -> s2d bf16 blocks
    out.append(("conv fwd", "stem 7x7/2 (s2d 4x4)", B * (H1 * H1 * 16 + H1 * H1 * 64), 2 * N * H1 * H1 * 64 * 256))
    out.append(("maxpool fwd", "maxpool", B * (H1 * H1 * 64 + H2 * H2 * 64) + N * H2 * H2 * 64, 0))
    hw, cin = H2, 64
    geo = []
    for si, (f, n, s) in enumerate(STAGES):
        for b in range(n):
            st = s if b == 0 else 1
            geo.append((si, b, hw, hw // st, cin, f, 4 * f, b == 0))
            hw, cin = hw // st, 4 * f
    for si, b, hi, ho, cin, f, fo, proj in geo:
        t = "s%db%d " % (si + 1, b)
        if proj or f > fold1_maxc:
            out.append(("bn_relu_apply", t + "ax", B * 2 * hi * hi * cin, 0))
        if proj:
            out.append(("conv fwd", t + "proj 1x1", B * (ho * ho * cin + ho * ho * fo), 2 * N * ho * ho * cin * fo))
        out.append(("conv fwd", t + "c1 1x1", B * (hi * hi * cin + hi * hi * f), 2 * N * hi * hi * cin * f))
        out.append(("bn_relu_apply", t + "a1", B * 2 * hi * hi * f, 0))
        out.append(("conv fwd", t + "c2 3x3", B * (hi * hi * f + ho * ho * f), 2 * N * ho * ho * 9 * f * f))
        out.append(("bn_relu_apply", t + "a2", B * 2 * ho * ho * f, 0))
        out.append(("conv fwd", t + "c3 1x1", B * (ho * ho * f + 2 * ho * ho * fo), 2 * N * ho * ho * f * fo))
    for si, b, hi, ho, cin, f, fo, proj in reversed(geo):
        t = "s%db%d " % (si + 1, b)
        out.append(("conv dgrad", t + "c3 1x1", B * (ho * ho * fo + 2 * ho * ho * f), 2 * N * ho * ho * f * fo))
        out.append(("bn_bwd_apply", t + "dh2", B * 3 * ho * ho * f, 0))
        out.append(("conv wgrad", t + "c3", B * (ho * ho * f + ho * ho * fo), 2 * N * ho * ho * f * fo))
        out.append(("conv dgrad", t + "c2 3x3", B * (ho * ho * f + 2 * hi * hi * f), 2 * N * ho * ho * 9 * f * f))
        out.append(("bn_bwd_apply", t + "dh1", B * 3 * hi * hi * f, 0))
        out.append(("conv wgrad", t + "c2", B * (hi * hi * f + ho * ho * f), 2 * N * ho * ho * 9 * f * f))
        cpd = proj and compact_pd and ho < hi
        pd = ho * ho * cin if cpd else hi * hi * cin  # the projection data gradient's pixels x channels
        if proj:
            out.append(("conv dgrad", t + "proj 1x1", B * (ho * ho * fo + pd), 2 * N * ho * ho * cin * fo))
            out.append(("conv wgrad", t + "proj", B * (ho * ho * cin + ho * ho * fo), 2 * N * ho * ho * cin * fo))
        out.append(("conv dgrad", t + "c1 1x1", B * (hi * hi * f + 2 * hi * hi * cin + (pd if proj else 0)),
                    2 * N * hi * hi * cin * f))
        out.append(("conv wgrad", t + "c1", B * (hi * hi * cin + hi * hi * f), 2 * N * hi * hi * cin * f))
        out.append(("bn_bwd_apply", t + "g", B * (3 if proj else 4) * hi * hi * cin, 0))
    out.append(("maxpool bwd", "maxpool", B * (H2 * H2 * 64 + H1 * H1 * 64) + N * H2 * H2 * 64, 0))
    # space-to-depth stem (hip_imagenet.py _CG_S2D): a 4x4/1 conv over [H1][H1][16] blocks, K = 256
    out.append(("conv wgrad", "stem", B * (H1 * H1 * 16 + H1 * H1 * 64), 2 * N * H1 * H1 * 64 * 256))
    return out


KERNEL_FAMILY = [("cg_bn_relu_apply", "bn_relu_apply"), ("cg_bn_bwd_apply", "bn_bwd_apply"), ("convg_stem_s2d", "conv fwd"),
                 ("convg_wgrad", "conv wgrad"), ("cg_maxpool_fwd", "maxpool fwd"), ("cg_maxpool_bwd", "maxpool bwd"),
                 ("cg_prep_input", "prep_input")]


def kernel_family(k: str):
    if "convg_fwd_kernel" in k:
        return "conv dgrad" if k.split(",")[4].strip().startswith("true") else "conv fwd"
    if "convg_t3_kernel" in k:  # <TC, EPI, AKM, ...>: AKM = data gradient
        return "conv dgrad" if k.split(",")[2].strip().startswith("true") else "conv fwd"
    if "cg_ew_apply_cf_kernel" in k:  # <RELU_APPLY>: the channel-fixed apply kernels
        return "bn_relu_apply" if "<true>" in k else "bn_bwd_apply"
    for pre, f in KERNEL_FAMILY:
        if pre in k:
            return f
    return None


def per_launch(trace_csv: str, N: int, **kw):
    """Zip the last complete step of the trace with launches(): (family, label, bytes, flops, measured us)."""
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "fused_optimizer_kernel" in r["Kernel_Name"]]
    lo = ends[-2] + 1 if len(ends) >= 2 else 0
    seq = [(kernel_family(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
           for r in rows[lo:ends[-1]]]
    seq = [x for x in seq if x[0] is not None]
    ls = launches(N, **kw)
    assert [x[0] for x in seq] == [x[0] for x in ls], "trace does not match the launch model"
    return [l + (m[1],) for l, m in zip(ls, seq)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="?")
    ap.add_argument("--n", type=int, default=1024, help="images per step over the population (pop 8 x 128)")
    ap.add_argument("--bw", type=float, default=6.3, help="achievable HBM TB/s")
    ap.add_argument("--pf", type=float, default=2.5, help="dense bf16 MFMA peak, PFLOP/s")
    ap.add_argument("--top", type=int, default=25, help="launches listed by excess over their floor")
    ap.add_argument("--fold1-maxc", type=int, default=256, help="CG_FOLD1_MAXC of the traced plan (0: no fold)")
    ap.add_argument("--no-compact-pd", action="store_true", help="the traced plan ran without CG_COMPACT_PD")
    a = ap.parse_args()
    kw = dict(fold1_maxc=a.fold1_maxc, compact_pd=not a.no_compact_pd)
    rows = per_launch(a.trace, a.n, **kw) if a.trace else [l + (0.0,) for l in launches(a.n, **kw)]
    fam = collections.defaultdict(lambda: [0.0, 0.0, 0.0])
    for f, lab, b, fl, m in rows:
        floor = max(b / (a.bw * 1e12), fl / (a.pf * 1e15)) * 1e6
        fam[f][0] += b / 1e9
        fam[f][1] += floor
        fam[f][2] += m
    print("floor = max(activation bytes / %.1f TB/s, FLOPs / %.1f PF/s) per launch, %d images per step" %
          (a.bw, a.pf, a.n))
    print("%-16s %9s %10s %12s %7s" % ("family", "GB", "floor ms", "measured ms", "ratio"))
    T = [0.0, 0.0, 0.0]
    for k, (g, fl, m) in sorted(fam.items(), key=lambda kv: -kv[1][2]):
        print("%-16s %9.1f %10.2f %12.2f %7s" % (k, g, fl / 1e3, m / 1e3, ("%.2f" % (m / fl)) if m else "-"))
        T = [T[0] + g, T[1] + fl, T[2] + m]
    print("%-16s %9.1f %10.2f %12.2f %7s" % ("total", T[0], T[1] / 1e3, T[2] / 1e3,
                                             ("%.2f" % (T[2] / T[1])) if T[2] else "-"))
    if a.trace:
        print("\nlaunches by excess over their floor (us):")
        print("%-14s %-20s %8s %8s %8s %7s %7s" % ("family", "launch", "GB", "TFLOP", "floor", "meas", "TB/s"))
        ex = sorted(rows, key=lambda r: -(r[4] - max(r[2] / (a.bw * 1e12), r[3] / (a.pf * 1e15)) * 1e6))
        for f, lab, b, fl, m in ex[:a.top]:
            floor = max(b / (a.bw * 1e12), fl / (a.pf * 1e15)) * 1e6
            print("%-14s %-20s %8.2f %8.3f %8.1f %7.1f %7.2f" % (f, lab, b / 1e9, fl / 1e12, floor, m,
                                                              b / (m * 1e-6) / 1e12))


if __name__ == "__main__":
    sys.exit(main())
