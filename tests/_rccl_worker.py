"""Rank body of the RCCL GPU tests (tests/test_gpu_rccl_shared.py): launched under torchrun with
``DTF_SHARE_GPU=1`` so that 2 ranks share the test box's one GPU over real RCCL (parallel/comm.py
``configure_shared_gpu``).  Writes one JSON result per rank to ``$DTF_RCCL_OUT/rank<r>.json``.

Modes (argv[1]):
  exploit  2 HIP ResNet-20 members per rank; cross-rank exploit copies of whole state rows over RCCL
           send/recv (parallel/dataplane.py, reference pbt_cluster.py:145-147) -> bit-exact rows, and the next
           captured step of a loser runs on the imported weights and step counter.
  dp       --dp_size 2: one member group of 2 ranks trains 2 members, the gradient all-reduce captured in the
           HIP step graph (engine/hip_resnet.py run_captured); replicas must stay bitwise identical, and the
           step must have run as a graph (no eager fallback).
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _hps(n, seed):
    import random
    from distributedtf_amd.pbt.hparams import generate_random_hparam
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        h = generate_random_hparam(rng)
        h["batch_size"] = 32
        h["opt_case"] = {"optimizer": "Momentum", "lr": 0.05, "momentum": 0.9}
        h["regularizer"] = None
        h["decay_steps"] = 0
        out.append(h)
    return out


def run_exploit(comm, out):
    import torch
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    from distributedtf_amd.parallel.dataplane import DataPlane
    rank = comm.Get_rank()
    hps = _hps(4, 7)
    ids = [2 * rank, 2 * rank + 1]
    members = [Cifar10Model(i, hps[i], "/tmp/dtf_rccl_%d/model_" % rank, seed=11, resnet_size=20, capacity=2,
                            use_synthetic_data=True, checkpoint_every_round=False) for i in ids]
    eng = members[0].engine
    ds = members[0].dataset()
    batch = ds.batch_slice(32)
    slots = [m.slot for m in members]

    def step():
        lrs = [m.learning_rate(eng.host_step[m.slot]) for m in members]
        return eng.train_step(slots, [batch, batch], [m.hparams for m in members], lrs).float().cpu().tolist()

    for _ in range(3):
        step()
    # a 4th step for member 0 of rank 0 only would desync step counters; instead member ids differ in init only
    rows = {m.cluster_id: m.state_view().detach().cpu().numpy().copy() for m in members}
    steps = {m.cluster_id: int(m.global_step) for m in members}
    allrows = comm.allgather(rows)
    allsteps = {}
    for s in comm.allgather(steps):
        allsteps.update(s)
    # winners 0 (rank 0) -> loser 3 (rank 1), winner 2 (rank 1) -> loser 1 (rank 0): both directions at once
    transfers = [(0, 0, 3, 1), (2, 1, 1, 0)]
    dp = DataPlane(comm)
    dp.execute(transfers, {m.cluster_id: m for m in members}, steps=allsteps)
    torch.cuda.synchronize()
    src_of = {3: 0, 1: 2}
    exact = {}
    for m in members:
        if m.cluster_id in src_of:
            src = src_of[m.cluster_id]
            want = allrows[src // 2][src]
            got = m.state_view().detach().cpu().numpy()
            exact[m.cluster_id] = bool((got == want).all())
    out["bitexact"] = exact
    out["bytes_moved"] = dp.bytes_moved
    # next captured step: the loser continues from the winner's weights and step counter
    losses = step()
    out["losses_after"] = dict(zip([m.cluster_id for m in members], losses))
    out["steps_after"] = {m.cluster_id: int(m.global_step) for m in members}
    out["state_steps_after"] = {m.cluster_id: float(m.state_view()[3 * eng.Pp + eng.R].item()) for m in members}
    allv = comm.allgather([out["losses_after"], out["steps_after"]])
    la = {}
    sa = {}
    for lv, sv in allv:
        la.update({int(k): v for k, v in lv.items()})
        sa.update({int(k): v for k, v in sv.items()})
    out["all_losses_after"] = la
    out["all_steps_after"] = sa
    from distributedtf_amd.engine.hip_resnet import graph_state
    out["graph_state"] = graph_state(eng.backend)


def run_dp(comm, out):
    import torch
    from distributedtf_amd.pbt.cluster import SPMDPopulation
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    from distributedtf_amd.engine.hip_resnet import graph_state
    hps = _hps(2, 5)
    pop = SPMDPopulation(2, comm, Cifar10Model, epochs_per_round=1, seed=5, verbose=False, hparams=hps, dp_size=2,
                         model_kwargs=dict(resnet_size=20, max_train_steps=4, use_synthetic_data=True,
                                           eval_every_round=False, checkpoint_every_round=False))
    pop.train(2)
    torch.cuda.synchronize()
    states = {g.cluster_id: g.export_state().detach().cpu().numpy().copy() for g in pop.worker.worker_graphs}
    gathered = comm.allgather(states)
    out["replicas_identical"] = {int(mid): bool((gathered[0][mid] == gathered[1][mid]).all()) for mid in gathered[0]}
    out["finite"] = all(bool(torch.isfinite(torch.from_numpy(v)).all()) for v in states.values())
    eng = pop.worker.worker_graphs[0].engine
    out["graph_state"] = graph_state(eng.backend)
    out["steps"] = {g.cluster_id: int(g.global_step) for g in pop.worker.worker_graphs}
    dst = os.environ.get("DTF_RCCL_OUT")
    if dst and comm.Get_rank() == 0:
        import numpy as np
        np.savez(os.path.join(dst, "dp_states.npz"), **{"m%d" % k: v for k, v in states.items()})


def main():
    from distributedtf_amd.parallel.comm import init_distributed, shutdown_distributed
    import faulthandler
    mode = sys.argv[1]
    # a hang leaves every thread's stack in the log before the test's subprocess timeout
    faulthandler.dump_traceback_later(int(os.environ.get("DTF_RCCL_DUMP_S", "100")), exit=True)
    comm = init_distributed()
    out = {"rank": comm.Get_rank(), "world": comm.Get_size(), "mode": mode}
    try:
        {"exploit": run_exploit, "dp": run_dp}[mode](comm, out)
    except Exception:
        import traceback
        out["error"] = traceback.format_exc()
    dst = os.environ.get("DTF_RCCL_OUT", ".")
    with open(os.path.join(dst, "rank%d.json" % comm.Get_rank()), "w") as f:
        json.dump(out, f)
    print(json.dumps({k: v for k, v in out.items() if k != "error"}), flush=True)
    comm.barrier()
    shutdown_distributed()
    faulthandler.cancel_dump_traceback_later()
    sys.exit(1 if "error" in out else 0)


if __name__ == "__main__":
    main()
