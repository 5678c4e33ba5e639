"""Do independent branches of a captured HIP graph run concurrently on this ROCm build? (diagnostic)

Two chains of N spin kernels (torch.cuda._sleep) captured (a) on one stream, (b) forked onto two streams and
joined; prints replay time per kernel for both.  (b) ~ half of (a) means the branches overlap on the GPU.
Also prints the same for small 1-workgroup add kernels (latency-bound chains, like the pop-1 training step).
"""
import time

import torch


def timed(g, reps=10):
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def capture(body):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    return g


def main(n=100, cycles=20000):
    side = torch.cuda.Stream()
    x = torch.zeros(64, device="cuda")
    y = torch.zeros(64, device="cuda")

    for name, op_a, op_b in (("sleep", lambda: torch.cuda._sleep(cycles), lambda: torch.cuda._sleep(cycles)),
                             ("add1wg", lambda: x.add_(1.0), lambda: y.add_(1.0))):
        def serial():
            for _ in range(n):
                op_a()
                op_b()

        def forked():
            main_s = torch.cuda.current_stream()
            side.wait_stream(main_s)
            for _ in range(n):
                op_a()
            with torch.cuda.stream(side):
                for _ in range(n):
                    op_b()
            main_s.wait_stream(side)

        ts = timed(capture(serial))
        tf = timed(capture(forked))
        print("%-7s serial %.1f us  forked %.1f us  ratio %.2f  (%d kernels)" % (name, ts * 1e6, tf * 1e6, tf / ts,
                                                                             2 * n))


if __name__ == "__main__":
    main()
