"""Per-kernel floor of a graph-replayed launch chain on this box (diagnostic).

Captures N dependent launches of (a) a trivial torch kernel and (b) the library's 1-workgroup step_advance
kernel into one HIP graph, replays it and prints microseconds per launch.  Run under different environment
settings (e.g. HIP_FORCE_DEV_KERNARG) to see what the runtime adds per kernel node.
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def bench_graph(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


def bench_eager(fn, n=200, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps * n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / n * 1e6


def main():
    x = torch.zeros(64, device="cuda")
    print("env HIP_FORCE_DEV_KERNARG=%s" % os.environ.get("HIP_FORCE_DEV_KERNARG"))
    print("torch add_ (1 WG)      graph %.2f us/kernel  eager %.2f" % (bench_graph(lambda: x.add_(1.0)),
                                                                        bench_eager(lambda: x.add_(1.0))))
    y = torch.zeros(1 << 20, device="cuda")
    print("torch add_ (4 MB)      graph %.2f us/kernel" % bench_graph(lambda: y.add_(1.0)))
    from distributedtf_amd import ops
    L = ops.lib()
    state = torch.zeros(4, 64, device="cuda")
    hyper = torch.zeros(4, 8, device="cuda")
    slots = torch.zeros(1, dtype=torch.int32, device="cuda")
    L.dtf_step_advance.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]

    def adv():
        L.dtf_step_advance(state.data_ptr(), 64, 3, hyper.data_ptr(), 2, slots.data_ptr(), 1,
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))

    print("dtf step_advance (1 WG) graph %.2f us/kernel  eager %.2f" % (bench_graph(adv), bench_eager(adv)))


if __name__ == "__main__":
    main()
