"""RCCL rehearsal on one GPU: 2+ ranks share the device (``DTF_SHARE_GPU=1``, per-rank NCCL_HOSTID).

    DTF_SHARE_GPU=1 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_shared_probe.py

Checks, on real RCCL kernels: the communicator forms, all_reduce is exact, a batch_isend_irecv of a multi-MB
state row is bit-exact, and an all_reduce captured in a HIP graph replays correctly (the data-parallel step
captures its gradient all-reduce this way).  Prints one JSON line per rank.
"""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from distributedtf_amd.parallel.comm import init_distributed, preconnected

    comm = init_distributed()
    rank, world = comm.Get_rank(), comm.Get_size()
    dev = torch.device("cuda", torch.cuda.current_device())
    out = {"rank": rank, "world": world, "device": str(dev), "preconnected": preconnected()}
    # 1. all_reduce
    t = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    out["allreduce_ok"] = bool(torch.all(t == sum(range(1, world + 1))).item())
    # 2. P2P state-row copy (ring: rank r sends to r+1)
    n = (8 << 20) // 4
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    src = torch.randn(n, generator=g).to(dev)
    dst = torch.empty(n, device=dev)
    peer_to, peer_from = (rank + 1) % world, (rank - 1) % world
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, src, peer_to), dist.P2POp(dist.irecv, dst, peer_from)])
    for r in reqs:
        r.wait()
    torch.cuda.synchronize()
    out["p2p_ms"] = round(1000 * (time.perf_counter() - t0), 3)
    want = torch.randn(n, generator=torch.Generator(device="cpu").manual_seed(1234 + peer_from))
    out["p2p_bitexact"] = bool(torch.equal(dst.cpu(), want))
    # 3. all_reduce captured in a HIP graph, replayed 3 times
    if os.environ.get("DTF_PROBE_GRAPH", "1") != "1":
        out["graph_allreduce_ok"] = True
        return finish(out, comm)
    buf = torch.zeros(4096, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.stream(s):
            dist.all_reduce(buf)  # warm-up outside the capture
            graph.capture_begin(capture_error_mode="thread_local")
            buf.add_(1.0)
            dist.all_reduce(buf)
            graph.capture_end()
        torch.cuda.current_stream().wait_stream(s)
        buf.zero_()
        vals = []
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            vals.append(float(buf[0].item()))
        # buf <- (buf + 1) * world each replay
        exp, e = [], 0.0
        for _ in range(3):
            e = (e + 1.0) * world
            exp.append(e)
        out["graph_allreduce"] = vals
        out["graph_allreduce_ok"] = vals == exp
    except Exception as err:  # report, do not hide
        out["graph_allreduce_error"] = repr(err)[:300]
        out["graph_allreduce_ok"] = False
    del graph
    return finish(out, comm)


def finish(out, comm):
    import faulthandler
    from distributedtf_amd.parallel.comm import shutdown_distributed
    print(json.dumps(out) + "\n", end="", flush=True)
    mark = lambda m: print("rank %d: %s" % (out["rank"], m), file=sys.stderr, flush=True)  # noqa: E731
    faulthandler.dump_traceback_later(25, exit=False)
    mark("barrier")
    comm.barrier()
    mark("shutdown")
    shutdown_distributed()
    mark("shutdown done")
    faulthandler.cancel_dump_traceback_later()
    ok = out["allreduce_ok"] and out["p2p_bitexact"] and out["graph_allreduce_ok"]
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
