"""RCCL paths on real hardware with the 1-GPU test box: 2 torchrun ranks share the device (``DTF_SHARE_GPU=1``
gives each rank its own NCCL_HOSTID, so RCCL forms the communicator and moves data over its socket transport;
parallel/comm.py ``configure_shared_gpu``).  The RCCL kernels, the proxy, the ProcessGroupNCCL stream ordering and
graph capture are the ones an 8-GPU node runs; only the wire differs (loopback instead of xGMI).

Reference: the exploit weight copy (``pbt_cluster.py:145-147,168-181``) and the dead
MirroredStrategy all-reduce (``distribution_utils.py:41-47``, T1).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, tmp, extra_env=None, timeout=150, tag=None, nproc=2):
    env = dict(os.environ)
    env.update(DTF_SHARE_GPU="1", DTF_RCCL_OUT=str(tmp), HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    # the rank logs go to a file (kept under gpurun_out/ on the GPU box) so a hang still leaves its stacks
    # (tests/_rccl_worker.py dumps every thread's stack before the timeout)
    logdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else str(tmp)
    path = os.path.join(logdir, "rccl_%s.log" % (tag or args[-1]))
    with open(path, "w") as f:
        try:
            p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT, timeout=timeout)
            rc = p.returncode
        except subprocess.TimeoutExpired:
            rc = "timeout"
    with open(path) as f:
        log = f.read()
    return rc, log


def _results(tmp):
    out = []
    for r in range(2):
        with open(os.path.join(tmp, "rank%d.json" % r)) as f:
            out.append(json.load(f))
    for o in out:
        assert "error" not in o, o["error"]
    return out


@pytest.mark.timeout(200)
def test_rccl_exploit_copy_bitexact(tmp_path):
    rc, log = _torchrun(["tests/_rccl_worker.py", "exploit"], tmp_path)
    assert rc == 0, log[-4000:]
    r0, r1 = _results(tmp_path)
    # rank 1's member 3 <- member 0 (rank 0); rank 0's member 1 <- member 2 (rank 1)
    assert r1["bitexact"] == {"3": True} and r0["bitexact"] == {"1": True}, (r0["bitexact"], r1["bitexact"])
    la, sa = r0["all_losses_after"], r0["all_steps_after"]
    # the loser continues from the winner: same weights, same step counter, same batch -> the same loss as the
    # winner on this step (BN statistic atomics may reorder: near-equal, not bitwise)
    for dst, src in (("3", "0"), ("1", "2")):
        assert sa[dst] == sa[src] == 4, sa
        assert abs(la[dst] - la[src]) <= 2e-3 * max(1.0, abs(la[src])), la
    assert abs(la["0"] - la["2"]) > 1e-4, "members with different init should differ"
    for r in (r0, r1):
        for mid, st in r["state_steps_after"].items():
            assert st == r["steps_after"][mid]
        assert r["graph_state"] == "captured"


@pytest.mark.timeout(300)
def test_rccl_data_parallel_graph_replicas_identical(tmp_path):
    """--dp_size 2 on the HIP backend: the RCCL gradient all-reduce is captured in the step graph (no eager
    fallback), the two replicas stay bitwise identical, and the process group tears down cleanly (captured graphs
    holding RCCL collectives are released first).  With the deterministic kernel build (--deterministic: fixed-order
    BN statistics) the graph-replayed run and the same steps run eagerly (DTF_HIP_GRAPH=0) are bitwise equal: the
    captured all-reduce is ordered exactly like the eager one."""
    import numpy as np
    det = {"DTF_DETERMINISTIC": "1"}
    rc, log = _torchrun(["tests/_rccl_worker.py", "dp"], tmp_path, extra_env=det, tag="dp_graph")
    assert rc == 0, log[-4000:]
    assert "DTF WARNING" not in log, log[-4000:]
    r0, r1 = _results(tmp_path)
    for r in (r0, r1):
        assert r["graph_state"] == "captured", r
        assert all(r["replicas_identical"].values()), r["replicas_identical"]
        assert r["finite"]
        assert r["steps"] == {"0": 8, "1": 8}, r["steps"]
    g = dict(np.load(os.path.join(tmp_path, "dp_states.npz")))
    eager_dir = tmp_path / "eager"
    eager_dir.mkdir()
    rc, log = _torchrun(["tests/_rccl_worker.py", "dp"], eager_dir, extra_env=dict(det, DTF_HIP_GRAPH="0"),
                        tag="dp_eager")
    assert rc == 0, log[-4000:]
    e0, _ = _results(eager_dir)
    assert e0["graph_state"] == "disabled" and all(e0["replicas_identical"].values())
    e = dict(np.load(os.path.join(eager_dir, "dp_states.npz")))
    for k in g:
        assert np.array_equal(g[k], e[k]), (k, float(np.abs(g[k] - e[k]).max()))


@pytest.mark.timeout(200)
def test_rccl_bench_two_ranks(tmp_path):
    """bench.py's multi-rank path (what the driver's N = 2..8 runs execute): 4 members per rank, cross-rank
    exploit copies over RCCL inside the timed region, one JSON line from rank 0."""
    rc, log = _torchrun(["bench.py", "--gpus", "2", "--steps", "12", "--warmup", "3", "--exploit_every", "4"],
                        tmp_path, tag="bench2")
    assert rc == 0, log[-4000:]
    lines = [json.loads(x) for x in log.splitlines() if x.startswith("{")]
    assert len(lines) == 1, log[-3000:]
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["config"]["exploits_timed"] >= 2 and rec["value"] > 0
    assert rec["config"]["p2p_preconnected"] is True and rec["config"]["step_graph"] == "captured"


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n", [4, 8])
def test_rccl_bench_eight_ranks(tmp_path, n):
    """The driver's N = 4 / 8 headline commands, rehearsed on the 1-GPU box: n ranks, 8 / n
    members each (N = 8: the per-GPU work of the 8-GPU headline), an n-rank RCCL communicator with every pair
    pre-connected, and >= 2 exploit cycles inside the timed region -- at N = 8 each k = 2 cycle moves two disjoint
    cross-rank winner->loser pairs in one batch_isend_irecv (parallel/dataplane.py)."""
    rc, log = _torchrun(["bench.py", "--gpus", str(n), "--steps", "40"], tmp_path, tag="bench%d" % n, nproc=n,
                        timeout=360)
    assert rc == 0, log[-4000:]
    lines = [json.loads(x) for x in log.splitlines() if x.startswith("{")]
    assert len(lines) == 1, log[-3000:]
    rec = lines[0]
    print(json.dumps(rec))
    assert rec["n_gpus"] == n and rec["steps"] == 40 and rec["value"] > 0, rec
    assert rec["config"]["exploits_timed"] >= 2, rec
    assert rec["config"]["p2p_preconnected"] is True and rec["config"]["step_graph"] == "captured", rec
    assert rec["config"]["parallelism"] == "pbt_pop8_%dmembers_per_gpu" % (8 // n), rec
