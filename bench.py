"""Headline benchmark: images/sec (whole node), ResNet-56 CIFAR-10, PBT population 8.

    python bench.py                                  # 1 GPU: all 8 members on one device
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One timed "step" = one training step of EVERY population member (forward,
backward, fused optimizer update), i.e. ``pop * batch`` images across the node.
Members are split over the ranks (8/N per GPU; on one GPU all 8 run
population-batched).  Every ``--exploit_every`` steps the full PBT exploit/explore
cycle runs inside the timed region: score all-gather, truncation selection,
winner->loser state copy (RCCL send/recv over xGMI across GPUs, D2D on one GPU),
hyper-parameter perturbation.  Data: a fixed synthetic device batch per member
(random-normal 32x32x3 images, uniform labels), random-init weights.
Hyper-parameters are sampled from the reference search space with a fixed seed;
``batch_size`` is pinned to 128 for every member so per-step work is identical
across runs (the search space samples 65..255).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_METRIC = "images/sec (whole node) ResNet-56 CIFAR-10 PBT pop=8 at 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--pop", type=int, default=8)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--model", default="resnet", choices=["resnet", "mnist", "imagenet"],
                   help="resnet = headline CIFAR-10 ResNet (BASELINE configs 3/4); mnist = config 2; "
                        "imagenet = ResNet-50 on synthetic 224x224x3 (config 5)")
    p.add_argument("--resnet_size", type=int, default=None, help="default 56 (CIFAR) / 50 (imagenet)")
    p.add_argument("--resnet_version", type=int, default=2, choices=[1, 2])
    p.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp16"],
                   help="compute dtype; fp32 = the reference's default (CIFAR ResNets, MNIST: the fp32 HIP steps); fp16 = the "
                        "reference's fp16 mode (ResNet v2: the half build of the HIP kernels, static loss scale 128)")
    p.add_argument("--exploit_every", type=int, default=None,
                   help="steps between PBT exploit/explore cycles inside the timed region; default "
                        "min(25, max(1, steps // 2)) so every timed run holds at least one cycle; 0 = none")
    p.add_argument("--exploit_lag", type=int, default=5,
                   help="steps queued behind an exploit's loss readback before the host runs the cycle (metric "
                        "all-gather, plan, weight copies, explore): the GPU keeps that many steps of work while the "
                        "host gathers and plans, so the cycle does not drain the queue")
    p.add_argument("--exploit_offset", type=int, default=None,
                   help="exploit at steps k with (k + 1 + offset) %% exploit_every == 0; default exploit_every // 2 "
                        "(mid-interval), 0 = on the interval's last step")
    p.add_argument("--seed", type=int, default=2024)
    p.add_argument("--graph", type=int, default=1, help="capture the population step in a HIP graph")
    p.add_argument("--profile_json", default=None)
    p.add_argument("--ragged", action="store_true",
                   help="keep the sampled per-member batch sizes (65..255) and let explore perturb them (real PBT: "
                        "a new batch composition after every exploit); default pins every member to --batch")
    p.add_argument("--batch_sizes", default=None,
                   help="with --ragged: comma-separated per-member batch sizes (e.g. a PBT round's mix from "
                        "metrics.jsonl 'batch_sizes') instead of the sampled ones")
    a = p.parse_args()
    if a.resnet_size is None:
        a.resnet_size = 50 if a.model == "imagenet" else 56
    if a.exploit_every is None:
        a.exploit_every = min(25, max(1, a.steps // 2))
    if a.exploit_offset is None:
        a.exploit_offset = (a.exploit_every or 0) // 2
    return a


def main():
    args = parse()
    import torch
    from distributedtf_amd.parallel.comm import init_distributed
    from distributedtf_amd.parallel.dataplane import DataPlane
    from distributedtf_amd.pbt.cluster import partition, sample_population
    from distributedtf_amd.pbt.exploit import plan_exploit, apply_plan_to_values
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    from distributedtf_amd.models.mnist_model import MNISTModel
    from distributedtf_amd.models.imagenet_model import ImageNetModel

    if args.dtype == "fp16":
        os.environ["DTF_HALF"] = "1"  # the fp16 build of the kernels (ops.lib(), loaded at first use)
    from distributedtf_amd.utils.flags import get_loss_scale
    loss_scale = get_loss_scale(args.dtype, None)
    comm = init_distributed()
    rank, world = comm.Get_rank(), comm.Get_size()
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    hps = sample_population(args.pop, args.seed)
    if not args.ragged:
        for h in hps:
            h["batch_size"] = args.batch
    elif args.batch_sizes:
        bs = [int(v) for v in args.batch_sizes.split(",")]
        assert len(bs) == args.pop, "--batch_sizes needs one size per member (--pop %d)" % args.pop
        for h, b in zip(hps, bs):
            h["batch_size"] = b
    begin, cnt = partition(args.pop, world)[rank]
    if args.model == "mnist":
        make = lambda i: MNISTModel(begin + i, hps[begin + i], "/tmp/bench_savedata_%d/model_" % rank,  # noqa: E731
                                    seed=args.seed, device=dev, backend=args.backend, capacity=max(1, cnt),
                                    dtype=args.dtype, use_synthetic_data=True, checkpoint_every_round=False)
    elif args.model == "imagenet":
        make = lambda i: ImageNetModel(begin + i, hps[begin + i], "/tmp/bench_savedata_%d/model_" % rank,  # noqa: E731
                                       seed=args.seed, resnet_size=args.resnet_size,
                                       resnet_version=args.resnet_version, device=dev, backend=args.backend,
                                       dtype=args.dtype, loss_scale=loss_scale,
                                       capacity=max(1, cnt), use_synthetic_data=True, checkpoint_every_round=False)
    else:
        make = lambda i: Cifar10Model(begin + i, hps[begin + i], "/tmp/bench_savedata_%d/model_" % rank,  # noqa: E731
                                      seed=args.seed, resnet_size=args.resnet_size, resnet_version=args.resnet_version,
                                      device=dev, backend=args.backend, dtype=args.dtype, loss_scale=loss_scale,
                                      capacity=max(1, cnt), use_synthetic_data=True, checkpoint_every_round=False)
    members = [make(i) for i in range(cnt)]
    eng = members[0].engine
    ds = members[0].dataset()
    dataplane = DataPlane(comm)
    owner = {}
    for r, (b, c) in enumerate(partition(args.pop, world)):
        for i in range(b, b + c):
            owner[i] = r

    slots = [m.slot for m in members]
    batches = [ds.batch_slice(args.batch) for _ in members]
    images_done = [0]

    def step():
        hp = [m.hparams for m in members]
        lrs = [m.learning_rate(eng.host_step[m.slot]) for m in members]
        bt = batches if not args.ragged else [ds.batch_slice(int(m.hparams["batch_size"])) for m in members]
        images_done[0] += sum(int(b[1].shape[0]) for b in bt)
        return eng.train_step(slots, bt, hp, lrs)

    exploits = [0]
    exploit_s = []  # host wall time of each timed exploit/explore cycle (gather + plan + copy + perturb)
    exploit_wait_s = []  # time each cycle waited for its loss readback (steps queued ahead still executing)

    def exploit_start(losses):
        """Queue the population's loss readback (pinned, non-blocking) behind the step that produced it."""
        host = torch.empty(losses.numel(), dtype=torch.float32, pin_memory=dev.type == "cuda")
        host.copy_(losses.float(), non_blocking=True)
        evt = torch.cuda.Event() if dev.type == "cuda" else None
        if evt is not None:
            evt.record()
        return host, evt

    def exploit_cycle(pending):
        # score = -loss (no eval inside the timed region); full gather/plan/copy/perturb cycle.  Called after
        # the NEXT step has been queued, so the readback wait, the metric all-gather and the planning run on
        # the host while the GPU executes that step; the winners' weights copied are the ones after it.
        host, evt = pending
        tw = time.perf_counter()
        if evt is not None:
            evt.synchronize()  # only the readback, not the step queued behind it
        tc = time.perf_counter()
        exploit_wait_s.append(tc - tw)  # GPU still running the steps queued before the readback
        ls = host.tolist()
        vals = [[m.cluster_id, -ls[i], m.hparams, m.global_step] for i, m in enumerate(members)]
        parts = comm.allgather(vals)
        allv = [v[:3] for p in parts for v in p]
        steps = {v[0]: v[3] for p in parts for v in p}  # winners' host steps travel with the scores
        plan = plan_exploit(allv)
        transfers = [(p.src_id, owner[p.src_id], p.dst_id, owner[p.dst_id]) for p in plan]
        dataplane.execute(transfers, {m.cluster_id: m for m in members}, steps=steps)
        upd = apply_plan_to_values(allv, plan)
        for m in members:
            if m.cluster_id in upd:
                m.set_values(upd[m.cluster_id])
                if not args.ragged:
                    m.hparams["batch_size"] = args.batch
                m.perturb_hparams()
                if not args.ragged:
                    m.hparams["batch_size"] = args.batch
        exploits[0] += 1
        exploit_s.append(time.perf_counter() - tc)

    def barrier_sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        losses = step()
    # RCCL P2P connections of every GPU pair are opened by init_distributed (DTF_RCCL_PRECONNECT=1, the default):
    # no timed exploit pays a lazy setup.  Without that pre-connect (env off, or gloo), one untimed exploit cycle
    # opens the connections of this plan's pairs instead, so the timed cycles do not include the setup.
    from distributedtf_amd.parallel.comm import preconnected
    from distributedtf_amd.engine.hip_resnet import graph_state
    warm_exploit = world > 1 and args.exploit_every and not preconnected()
    if warm_exploit:
        exploit_cycle(exploit_start(losses))
        exploit_s.clear()
        exploit_wait_s.clear()
        exploits[0] = 0
    barrier_sync()
    images_done[0] = 0
    t0 = time.perf_counter()
    pending = []  # (due step, readback) of started exploit cycles
    lag = max(1, args.exploit_lag)
    for k in range(args.steps):
        losses = step()
        while pending and pending[0][0] <= k:
            exploit_cycle(pending.pop(0)[1])  # overlaps the steps queued since its readback
        # exploit points sit mid-interval (steps every/2, every/2 + every, ..) rather than on the last step, so
        # each cycle's host work (all-gather, plan, copies) overlaps steps still queued behind it -- as it does in
        # a long run -- instead of being appended, fully exposed, after the final step
        if args.exploit_every and (k + 1 + args.exploit_offset) % args.exploit_every == 0:
            pending.append((k + lag, exploit_start(losses)))
    for _, pend in pending:
        exploit_cycle(pend)  # an exploit due after the last step still runs inside the timed region
    barrier_sync()
    dt = time.perf_counter() - t0
    dts = comm.allgather(dt)
    dt_max = max(dts)
    # images trained in the timed steps, summed over ranks (ragged: each member's own, changing batch size)
    images = sum(comm.allgather(images_done[0]))
    value = images / dt_max
    if rank == 0:
        flops = members[0].arch.flops_per_image() * 3.0 * images / dt_max
        metric = BASELINE_METRIC if args.model == "resnet" and args.resnet_size == 56 and args.resnet_version == 2 else \
            "images/sec (whole node) %s PBT pop=%d" % (members[0].arch.name, args.pop)
        out = {
            "metric": metric,
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt_max / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (device-resident random-normal %s, uniform labels), random-init weights"
                    % "x".join(str(d) for d in members[0].arch.input_shape),
            "config": {"model": members[0].arch.name,
                       "global_batch": args.pop * args.batch if not args.ragged else round(images / args.steps, 1),
                       "per_member_batch": args.batch if not args.ragged else "sampled 65..255 (ragged)",
                       "population": args.pop, "seq_len": None,
                       "parallelism": "pbt_pop%d_%dmembers_per_gpu" % (args.pop, cnt),
                       "backend": eng.backend.name, "exploit_every": args.exploit_every,
                       "exploits_timed": exploits[0],
                       "p2p_preconnected": preconnected() if world > 1 else None,
                       "untimed_warmup_exploit": bool(warm_exploit),
                       "step_graph": graph_state(eng.backend),
                       # persistent forward segments whose grid barrier timed out (must be 0; see hip_resnet)
                       "persist_barrier_failures": (eng.backend.persist_failures()
                                                    if hasattr(eng.backend, "persist_failures") else None)},
            "exploit_ms_mean": round(1000.0 * sum(exploit_s) / len(exploit_s), 3) if exploit_s else None,
            "exploit_readback_wait_ms_mean": (round(1000.0 * sum(exploit_wait_s) / len(exploit_wait_s), 3)
                                              if exploit_wait_s else None),
            "achieved_tflops": round(flops / 1e12, 2),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        from distributedtf_amd.parallel.comm import shutdown_distributed
        shutdown_distributed()


if __name__ == "__main__":
    main()
