"""Common entry point of all ranks (reference ``main_manager.py:1-73``).

    # reference-style: positional population size, module-level defaults
    python main_manager.py 20
    # one process per GPU (SPMD: every rank trains, RCCL exploit copies)
    torchrun --standalone --nproc-per-node 8 main_manager.py 8 --model cifar10 --resnet_size 56
    # reference-compatible master/worker protocol (rank 0 trains nothing)
    torchrun --nproc-per-node 2 main_manager.py 2 --model toy --mode master_worker --rounds 30 \
        --epochs_per_round 4

Outputs are the reference's: ``savedata/`` (wiped at start), ``initial_hp.json``,
per-member ``model_<id>/`` (checkpoint + learning curves), ``best_model.json``,
``{acc,lr,best3[,toy]}_<mode>.png`` and a line appended to ``test_results.txt``.
"""

from __future__ import annotations

import os
import shutil
import sys

##################
# configurations (reference main_manager.py:32-44)
##################
master_rank = 0
train_round = 20
population_size = 20
epochs_per_round = 1
do_exploit = True
do_explore = True
target_model = "mnist"   # 'toy' | 'mnist' | 'cifar10' | 'imagenet'


def main(argv=None):
    from distributedtf_amd.utils.flags import parse_main_args
    from distributedtf_amd.models import model_class
    from distributedtf_amd.parallel.comm import init_distributed, backend_name
    from distributedtf_amd.pbt.cluster import PBTCluster, SPMDPopulation
    from distributedtf_amd.pbt.worker import TrainingWorker
    from distributedtf_amd.pbt import reports

    args = parse_main_args(argv, defaults=dict(
        population_size=population_size, train_round=train_round, epochs_per_round=epochs_per_round,
        do_exploit=do_exploit, do_explore=do_explore, model=target_model))
    args.apply_runtime_modes()  # --debug_kernels / --deterministic, before the first GPU use
    cls = model_class(args.model)
    model_kwargs = args.model_kwargs()
    if args.model == "toy":
        backend = "gloo"
    else:
        backend = None
    comm = init_distributed(backend=backend)
    rank, world = comm.Get_rank(), comm.Get_size()
    savedata = args.savedata

    if rank == master_rank and not args.resume:
        shutil.rmtree(savedata, ignore_errors=True)
    if rank == master_rank:
        os.makedirs(savedata, exist_ok=True)
    comm.barrier()

    inject = args.inject_nan_schedule()
    from distributedtf_amd.utils import logger as bench_logger
    if args.mode == "master_worker":
        if world < 2:
            raise SystemExit("master_worker mode needs >= 2 ranks (1 master + workers)")
        from distributedtf_amd.parallel.dataplane import DataPlane
        if rank == master_rank:
            cluster = PBTCluster(args.population_size, comm, master_rank, epochs_per_round=args.epochs_per_round,
                                 do_exploit=args.do_exploit, do_explore=args.do_explore, seed=args.seed,
                                 exploit_transport=args.exploit_transport, savedata=savedata,
                                 reseed_dead=args.reseed_dead)
        else:
            worker = TrainingWorker(comm, master_rank, cls, save_base_dir=os.path.join(savedata, "model_"),
                                    seed=args.seed, model_kwargs=model_kwargs, dataplane=DataPlane(comm))
            # the worker process trains members: its eval results / hook metrics go to its own benchmark files
            with bench_logger.benchmark_context(args, rank=rank):
                worker.main_loop()
            if world > 1:
                from distributedtf_amd.parallel.comm import shutdown_distributed
                shutdown_distributed()
            return 0
    else:
        cluster = SPMDPopulation(args.population_size, comm, cls, epochs_per_round=args.epochs_per_round,
                                 do_exploit=args.do_exploit, do_explore=args.do_explore, seed=args.seed,
                                 savedata=savedata, model_kwargs=model_kwargs, inject_nan=inject,
                                 resume=args.resume, dp_size=args.dp_size, reseed_dead=args.reseed_dead)

    # benchmark logger (reference logger.benchmark_context / log_run_info, cifar10_main.py:314-318,
    # resnet_run_loop.py:408-421): configured in EVERY process (per-rank files, utils/logger.rank_log_dir), so the
    # eval records of the members each rank trains are kept; rank 0 also writes the run info
    with bench_logger.benchmark_context(args, rank=rank) as blog:
        if rank == master_rank:
            blog.log_run_info(args.model if args.model != "cifar10" else "resnet%s" % (args.resnet_size or 50),
                              {"toy": "toy", "mnist": "mnist", "cifar10": "cifar10", "imagenet": "imagenet"}.get(
                                  args.model, args.model),
                              {k: v for k, v in vars(args).items() if not k.startswith("_")})
        if not args.resume or getattr(cluster, "start_round", 0) == 0:
            cluster.dump_all_models_to_json(os.path.join(savedata, "initial_hp.json"))
        elapsed = cluster.train(args.train_round)
        if rank == master_rank:
            reports.append_test_result(world, args.population_size, elapsed, args.results_file)
        if rank == master_rank or args.mode != "master_worker":
            if rank == master_rank:
                if args.model == "toy":
                    cluster.report_plot_for_toy_model()
                cluster.report_accuracy_plot()
                cluster.report_lr_plot()
                cluster.report_best3_plot()
            cluster.report_best_model()
            if args.export_dir:
                cluster.export_best_model(args.export_dir)  # resnet_run_loop.py:510-514
            cluster.print_profiling_info()
            cluster.kill_all_workers()
    if world > 1:
        from distributedtf_amd.parallel.comm import shutdown_distributed
        shutdown_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
