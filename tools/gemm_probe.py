"""Library GEMM (torch.bmm -> hipBLASLt / rocBLAS) times for the ResNet-50 1x1-conv shapes at pop 8 x 128 images:
what a plain library GEMM would take for each 1x1 conv pass (forward / data gradient / weight gradient), per member
batched (8 weight sets).  Prints us and TFLOP/s per shape.  Diagnostic (GPU)."""
import statistics
import sys

import torch


def t(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    print("blas backend:", getattr(torch.backends.cuda, "preferred_blas_library", lambda: "?")())
    shapes = []  # (label, per-member pixels, cin, cout)
    for st, hw, w in (("s1", 56, 64), ("s2", 28, 128), ("s3", 14, 256), ("s4", 7, 512)):
        P = 128 * hw * hw
        shapes += [(st + " c1", P, 4 * w, w), (st + " c3", P, w, 4 * w)]
    for lab, P, ci, co in shapes:
        x = torch.randn(8, P, ci, device=dev, dtype=torch.bfloat16)
        w = torch.randn(8, ci, co, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(8, P, co, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * 8 * P * ci * co
        f = t(lambda: torch.bmm(x, w))
        d = t(lambda: torch.bmm(dy, w.transpose(1, 2)))
        g = t(lambda: torch.bmm(dy.transpose(1, 2), x))
        print("%-6s P %6d ci %4d co %4d | fwd %7.1f us %5.0f TF | dgrad %7.1f us %5.0f TF | wgrad %7.1f us %5.0f TF"
              % (lab, P, ci, co, f, fl / f * 1e-6, d, fl / d * 1e-6, g, fl / g * 1e-6))
        sys.stdout.flush()
        del x, w, dy


if __name__ == "__main__":
    main()
