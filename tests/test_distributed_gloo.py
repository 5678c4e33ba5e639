"""Multi-process PBT over torch.distributed (gloo, CPU): the fake-cluster test the
reference never had (it relied on `mpirun --oversubscribe`)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp, q, pop=4):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    os.chdir(tmp)
    torch.set_num_threads(1)
    try:
        from distributedtf_amd.parallel.comm import init_distributed, shutdown_distributed
        from distributedtf_amd.pbt.cluster import SPMDPopulation
        from distributedtf_amd.models.cifar10_model import Cifar10Model
        from distributedtf_amd.pbt.hparams import generate_random_hparam
        import random
        comm = init_distributed(backend="gloo")
        rng = random.Random(3)
        hps = []
        for _ in range(pop):
            h = generate_random_hparam(rng)
            h["batch_size"] = 4
            hps.append(h)
        pop = SPMDPopulation(len(hps), comm, Cifar10Model, epochs_per_round=1, seed=5, verbose=False, hparams=hps,
                             model_kwargs=dict(resnet_size=8, max_train_steps=1, use_synthetic_data=True,
                                               device="cpu", eval_every_round=True))
        pop.train(1)
        plan = [(p.src_id, p.dst_id) for p in pop.last_plan]
        # bit-exact check: loser state == winner state right after the exploit copy
        states = {g.cluster_id: g.export_state().clone() for g in pop.worker.worker_graphs}
        gathered = comm.allgather({k: v for k, v in states.items()})
        allst = {}
        for d in gathered:
            allst.update(d)
        ok = all(torch.equal(allst[s], allst[d]) for s, d in plan)
        # the loser's HOST step counter (LR schedule) equals the winner's: learnt from the score all-gather,
        # never by reading the imported device row back
        hsteps = {}
        for d in comm.allgather({g.cluster_id: g.global_step for g in pop.worker.worker_graphs}):
            hsteps.update(d)
        e0 = pop.worker.worker_graphs[0].engine
        col = 3 * e0.Pp + e0.R  # step column of a state row
        ok = ok and all(hsteps[s] == hsteps[d] == int(allst[d][col].item()) for s, d in plan)
        q.put((rank, plan, ok, sorted(allst)))
        shutdown_distributed()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None))


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world,pop", [(2, 4), (8, 8)])
def test_spmd_gloo_exploit_bit_exact(tmp_path, world, pop):
    """Every rank computes the same plan; cross-rank copies (batch_isend_irecv) leave loser == winner bit-exact.
    world 8 / pop 8 is the headline layout (one member per rank, every exploit copy crosses ranks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q, pop)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=380) for _ in procs]
    for p in procs:
        p.join(30)
    for r in res:
        assert r[1] != "ERR", r[2]
    plans = {r[0]: r[1] for r in res}
    assert all(plans[k] == plans[0] for k in plans) and len(plans[0]) == -(-pop // 4)
    assert all(r[2] for r in res)
    assert res[0][3] == list(range(pop))


def _gather_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from distributedtf_amd.parallel.comm import init_distributed, shutdown_distributed
        comm = init_distributed(backend="gloo")
        small = comm.allgather([[rank, -0.5 * rank, {"lr": 0.1 * rank, "name": "m%d" % rank}]])
        # one rank over the slot: every rank must take the fallback together
        mixed = comm.allgather(b"x" * (comm.GATHER_SLOT + 10) if rank == 1 else rank)
        empty = comm.allgather(None)
        q.put((rank, small, [len(m) if isinstance(m, bytes) else m for m in mixed], empty))
        shutdown_distributed()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None))


@pytest.mark.timeout(120)
def test_allgather_fixed_slot_and_fallback():
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(world)], key=lambda t: t[0])
    for p in ps:
        p.join(30)
    for rank, small, mixed, empty in res:
        assert small != "ERR", mixed
        assert small == [[[r, -0.5 * r, {"lr": 0.1 * r, "name": "m%d" % r}]] for r in range(world)]
        assert mixed == [0, 8192 + 10, 2]
        assert empty == [None] * world
