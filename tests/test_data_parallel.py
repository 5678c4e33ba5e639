"""Intra-member data parallelism (parallel/dataparallel.py) over gloo on CPU: a world of
4 ranks with --dp_size 2 trains a population of 4 in 2 member groups.  Replicas stay bit-identical (gradients
are all-reduced before every optimizer step, BN running statistics at the end of each round), only group
leaders report values / write files, and exploit copies go replica-to-replica."""
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


def _worker(rank, world, port, tmp, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    os.chdir(tmp)
    torch.set_num_threads(1)
    try:
        from distributedtf_amd.parallel.comm import init_distributed, shutdown_distributed
        from distributedtf_amd.pbt.cluster import SPMDPopulation
        from distributedtf_amd.models.cifar10_model import Cifar10Model
        from distributedtf_amd.models.model_base import flush_checkpoints
        from distributedtf_amd.pbt.hparams import generate_random_hparam
        import random
        comm = init_distributed(backend="gloo")
        rng = random.Random(4)
        hps = []
        for _ in range(4):
            h = generate_random_hparam(rng)
            h["batch_size"] = 8
            h["opt_case"] = {"optimizer": "Momentum", "lr": 0.05, "momentum": 0.9}
            hps.append(h)
        pop = SPMDPopulation(4, comm, Cifar10Model, epochs_per_round=1, seed=5, verbose=False, hparams=hps,
                             dp_size=2, model_kwargs=dict(resnet_size=8, max_train_steps=2, use_synthetic_data=True,
                                                          device="cpu", eval_every_round=True))
        pop.train(2)
        flush_checkpoints()
        # numpy copies: torch CPU tensors would travel through the queue as shared-memory file descriptors, which
        # the parent cannot open once this process has exited
        states = {g.cluster_id: g.export_state().detach().cpu().numpy().copy() for g in pop.worker.worker_graphs}
        batches = {g.cluster_id: g.dp.local_batch(g.hparams["batch_size"]) for g in pop.worker.worker_graphs}
        gathered = comm.allgather(states)
        vals = pop.get_all_values()
        q.put((rank, gathered, sorted(v[0] for v in vals), [(p.src_id, p.dst_id) for p in pop.last_plan], batches))
        shutdown_distributed()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None, None))


@pytest.mark.timeout(300)
def test_dp_groups_world4_dp2(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 4, port, str(tmp_path), q)) for r in range(4)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=280) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(30)
    for r in res:
        assert r[1] != "ERR", r[2]
    gathered = res[0][1]  # per rank: {member id: state}
    # group 0 = ranks {0, 1} holds members {0, 1}; group 1 = ranks {2, 3} holds {2, 3}
    assert sorted(gathered[0]) == [0, 1] and sorted(gathered[1]) == [0, 1]
    assert sorted(gathered[2]) == [2, 3] and sorted(gathered[3]) == [2, 3]
    for a, b in ((0, 1), (2, 3)):
        for mid in gathered[a]:
            assert (gathered[a][mid] == gathered[b][mid]).all(), "replicas diverged (member %d)" % mid
    # the population table has every member once; the exploit plan agrees everywhere
    assert all(r[2] == [0, 1, 2, 3] for r in res)
    assert len({tuple(r[3]) for r in res}) == 1 and len(res[0][3]) == 1
    for mid in (0, 1):  # each member's batch is split over its 2 replicas (remainder to replica 0)
        assert res[0][4][mid] - res[1][4][mid] in (0, 1) and res[1][4][mid] > 0
    # files: one learning curve per member, written once per round (leader only)
    for mid in range(4):
        rows = open(os.path.join(tmp_path, "savedata", "model_%d" % mid, "learning_curve.csv")).read().splitlines()
        assert len(rows) == 1 + 2, rows


def _weighted_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from distributedtf_amd.parallel.comm import init_distributed, shutdown_distributed
        from distributedtf_amd.parallel.dataparallel import make_dp_context
        from distributedtf_amd.engine.population import PopulationEngine
        from distributedtf_amd.models.mnist import MnistArch
        comm = init_distributed(backend="gloo")
        dp = make_dp_context(comm, world)
        eng = PopulationEngine(MnistArch(), 2, "cpu")
        eng.set_data_parallel(dp)
        # member 0: batch 9 split 5 / 4; member 1: batch 8 split 4 / 4
        shard = [torch.zeros(dp.local_batch(9)), torch.zeros(dp.local_batch(8))]
        eng._set_dp_weights([0, 1], [(x, x) for x in shard], [{"batch_size": 9}, {"batch_size": 8}])
        eng.grads[0, :4] = torch.tensor([1.0, 2.0, 3.0, 4.0]) * (rank + 1)
        eng.grads[1, :4] = torch.tensor([1.0, 1.0, 1.0, 1.0]) * (rank + 1)
        eng.dp_sync_grads([0, 1])
        q.put((rank, eng.grads[:, :4].clone().numpy(), eng.dp_weight.clone().numpy()))
        shutdown_distributed()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


@pytest.mark.timeout(120)
def test_dp_gradient_weighted_by_shard():
    """An uneven split of a member batch (9 = 5 + 4) weights each replica's shard-mean gradient by its share:
    sum_r (n_r / N) * g_r is the gradient of the mean loss over the whole member batch (reference
    distribution_utils.py:24-78: MirroredStrategy averages equal per-replica batches)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_weighted_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(30)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    g = torch.tensor([1.0, 2.0, 3.0, 4.0])
    want0 = g * (5 / 9.0) * 1 + g * (4 / 9.0) * 2      # rank 0 holds 5 images, rank 1 holds 4
    want1 = torch.ones(4) * 0.5 * 1 + torch.ones(4) * 0.5 * 2
    for _, grads, w in res:
        torch.testing.assert_close(torch.from_numpy(grads[0]), want0)
        torch.testing.assert_close(torch.from_numpy(grads[1]), want1)
    assert abs(res[0][2][0] - 5 / 9.0) < 1e-6 and abs(res[1][2][0] - 4 / 9.0) < 1e-6


def test_dp_rejects_batch_smaller_than_group():
    """A member batch smaller than --dp_size would give some replica an empty shard: rejected."""
    from distributedtf_amd.parallel.dataparallel import DPContext
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    from distributedtf_amd.pbt.hparams import generate_random_hparam
    import random
    h = generate_random_hparam(random.Random(0))
    h["batch_size"] = 3
    m = Cifar10Model(0, h, "/tmp/dtf_dp_small/model_", seed=0, resnet_size=8, device="cpu", use_synthetic_data=True,
                     checkpoint_every_round=False)
    m.dp = DPContext(group=None, size=4, rank=0, group_index=0, n_groups=1)
    with pytest.raises(ValueError, match="dp_size"):
        m._batch(m.dataset(), None)
    m.hparams["batch_size"] = 9
    x, y = m._batch(m.dataset(), None)
    assert x.shape[0] == 3  # 9 = 3 + 2 + 2 + 2
