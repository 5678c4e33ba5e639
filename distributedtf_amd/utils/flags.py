"""Typed configuration + CLI.

Replaces the reference's two config tiers: module constants in
``main_manager.py:32-44`` (+ positional ``argv[1]`` = population size) and the
vendored absl flag registry that ``cifar10_main.py:239-330`` deletes and
re-defines from every member's hparam dict on every train call
(``official/utils/flags/{core,_base,_performance,_benchmark,_misc}.py``).

Here a member's settings are an explicit ``MemberConfig`` derived from its
hparam dict (no global mutation), and the CLI keeps the reference flag names that
matter: ``batch_size``, ``train_epochs``, ``epochs_between_evals``,
``use_synthetic_data``, ``max_train_steps``, ``dtype``, ``loss_scale``,
``data_format``, ``resnet_size``, ``resnet_version``, ``hooks``,
``stop_threshold``, ``export_dir``, ``data_dir``, ``model_dir``.
Validators mirror the reference's: ``loss_scale > 0`` (``_performance.py:125``),
no fp16 with ResNet v1 (``resnet_run_loop.py:546-549``).
"""

from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch

DTYPE_MAP = {"fp32": (torch.float32, 1), "fp16": (torch.float16, 128), "bf16": (torch.bfloat16, 1)}


def get_dtype(name: str) -> torch.dtype:
    return DTYPE_MAP[name][0]


def get_loss_scale(dtype: str, loss_scale: Optional[float]) -> float:
    if loss_scale is not None:
        return float(loss_scale)
    return float(DTYPE_MAP[dtype][1])


def _positive(v):
    f = float(v)
    if f <= 0:
        raise argparse.ArgumentTypeError("loss_scale should be a positive number.")
    return f


def _str2bool(v):
    if isinstance(v, bool):
        return v
    return str(v).lower() in ("1", "true", "yes", "y", "t")


def _synthetic(v):
    """--use_synthetic_data: a boolean (reference flag), or ``learnable`` -- class-template CIFAR-shaped images
    through the real input path, so eval accuracy can climb without the dataset (datasets.learnable_cifar)."""
    if isinstance(v, str) and v.lower() == "learnable":
        return "learnable"
    return _str2bool(v)


@dataclass
class MemberConfig:
    """Per-member training settings derived from one hparam dict (no global flags)."""
    optimizer: str
    learning_rate: float
    momentum: float = 0.0
    grad_decay: float = 0.0
    decay_steps: int = 0
    decay_rate: float = 1.0
    weight_decay: float = 0.0
    regularizer: Optional[str] = None
    initializer: Optional[str] = None
    batch_size: int = 128
    model_id: int = 0

    @staticmethod
    def from_hparams(hp: Dict[str, Any], model_id: int = 0) -> "MemberConfig":
        opt = hp["opt_case"]
        return MemberConfig(optimizer=opt["optimizer"], learning_rate=float(opt["lr"]),
                            momentum=float(opt.get("momentum", 0.0)), grad_decay=float(opt.get("grad_decay", 0.0)),
                            decay_steps=int(hp.get("decay_steps", 0)), decay_rate=float(hp.get("decay_rate", 1.0)),
                            weight_decay=float(hp.get("weight_decay", 0.0)),
                            regularizer=None if hp.get("regularizer") in (None, "None") else hp.get("regularizer"),
                            initializer=None if hp.get("initializer") in (None, "None") else hp.get("initializer"),
                            batch_size=int(hp.get("batch_size", 128)), model_id=model_id)


def build_parser(defaults: Optional[Dict[str, Any]] = None) -> argparse.ArgumentParser:
    d = dict(population_size=20, train_round=20, epochs_per_round=1, do_exploit=True, do_explore=True,
             model="mnist")
    d.update(defaults or {})
    p = argparse.ArgumentParser(description="MI355X population-based training", conflict_handler="resolve")
    p.add_argument("pop_size", nargs="?", type=int, default=None, help="population size (reference argv[1])")
    p.add_argument("--population_size", type=int, default=d["population_size"])
    p.add_argument("--model", default=d["model"], help="toy | mnist | cifar10 | imagenet")
    p.add_argument("--mode", default="spmd", choices=["spmd", "master_worker"])
    p.add_argument("--rounds", "--train_round", dest="train_round", type=int, default=d["train_round"])
    p.add_argument("--epochs_per_round", "--train_epochs", dest="epochs_per_round", type=int,
                   default=d["epochs_per_round"],
                   help="epochs each member trains per PBT round (the reference passes train_epochs = "
                        "epochs_per_round to every member's main(), cifar10_main.py:321-327, mnist_model.py:128)")
    p.add_argument("--epochs_between_evals", type=int, default=1,
                   help="epochs per train -> eval cycle inside a round: a round of E epochs runs E // this cycles, "
                        "each appending one learning_curve.csv row (reference _base.py:74-79, "
                        "resnet_run_loop.py:446-447)")
    p.add_argument("--do_exploit", type=_str2bool, default=d["do_exploit"])
    p.add_argument("--do_explore", type=_str2bool, default=d["do_explore"])
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--savedata", "--model_dir", dest="savedata", default="savedata",
                   help="base directory of the member directories model_<id>/ (reference: save_base_dir, passed to "
                        "each member as model_dir = save_base_dir + id, cifar10_main.py:323)")
    p.add_argument("--results_file", default="test_results.txt")
    p.add_argument("--exploit_transport", default="dataplane", choices=["dataplane", "files"])
    p.add_argument("--inject_nan_member", action="append", default=[],
                   help="fault injection: '<member_id>@<round>' marks the member NaN after that round")
    # model / training flags (reference names)
    p.add_argument("--resnet_size", type=int, default=None)
    p.add_argument("--resnet_version", type=int, default=2, choices=[1, 2])
    p.add_argument("--data_dir", default=None)
    p.add_argument("--use_synthetic_data", type=_synthetic, default=None,
                   help="true / false (reference flag) or 'learnable' (CIFAR: class-template images, real input path)")
    p.add_argument("--max_train_steps", type=int, default=None)
    p.add_argument("--debug_steps", type=int, default=None, help="MNIST: steps per 'epoch' (reference used 10)")
    p.add_argument("--batch_size", type=int, default=None, help="override every member's batch_size")
    p.add_argument("--dtype", default="bf16", choices=list(DTYPE_MAP))
    p.add_argument("--loss_scale", type=_positive, default=None)
    p.add_argument("--data_format", default="channels_last", choices=["channels_last"])
    p.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("--hooks", default="",
                   help="comma list of training hooks: logging (lr / cross_entropy / train_accuracy of every member "
                        "every 100 steps), examples_per_second, profiler (torch.profiler chrome trace every 1000 "
                        "steps into savedata/), metric (the logging values into the benchmark logger)")
    p.add_argument("--log_every_n_steps", type=int, default=100,
                   help="period of the logging / metric / examples_per_second hooks (reference: 100 steps)")
    p.add_argument("--log_probabilities_every_n", type=int, default=50,
                   help="MNIST: print each member's training softmax every N steps (the reference's LoggingTensorHook "
                        "on softmax_tensor, mnist_model.py:149-151); 0 = off")
    p.add_argument("--stop_threshold", type=float, default=None,
                   help="a member's train call ends once its eval accuracy reaches this (resnet_run_loop.py:505)")
    p.add_argument("--export_dir", default=None, help="export the best member's inference weights here at the end")
    p.add_argument("--ready_steps", type=int, default=None,
                   help="PBT ready interval in optimizer steps: every member trains exactly this many steps per round "
                        "(instead of epochs_per_round epochs), so the population stays in lockstep")
    p.add_argument("--benchmark_logger_type", default="BaseBenchmarkLogger",
                   choices=["BaseBenchmarkLogger", "BenchmarkFileLogger"])
    p.add_argument("--benchmark_log_dir", default=None, help="BenchmarkFileLogger: metric.log / benchmark_run.log")
    p.add_argument("--no_checkpoint", action="store_true")
    p.add_argument("--tf_checkpoint", action="store_true",
                   help="also write each member's checkpoint as a TF 1.x tensor bundle (model.ckpt-<step>.*)")
    p.add_argument("--deterministic", action="store_true",
                   help="bitwise-replayable run: seeded RNGs; the CIFAR ResNet v2 HIP step runs the deterministic "
                        "kernel build (fixed-order BatchNorm-statistic and weight-gradient reductions, "
                        "libdtf_kernels_det.so); other families use deterministic torch algorithms")
    p.add_argument("--debug_kernels", action="store_true",
                   help="serialise and synchronise every kernel launch (AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING"
                        "=1), no HIP graphs: a faulting kernel is reported at its own launch")
    p.add_argument("--dp_size", type=int, default=1,
                   help="ranks per population member (intra-member data parallelism; must divide the world)")
    p.add_argument("--reseed_dead", action="store_true",
                   help="re-seed members with NaN accuracy from the best members instead of culling them")
    p.add_argument("--resume", action="store_true",
                   help="continue a run from savedata/population_state.json + member checkpoints (no wipe)")
    return p


class MainArgs(argparse.Namespace):
    def model_kwargs(self) -> Dict[str, Any]:
        kw: Dict[str, Any] = {}
        if self.model != "toy":
            kw["backend"] = self.backend
            kw["use_synthetic_data"] = self.use_synthetic_data
            kw["max_train_steps"] = self.max_train_steps
            kw["checkpoint_every_round"] = not self.no_checkpoint
            kw["tf_checkpoint"] = bool(getattr(self, "tf_checkpoint", False))
            if self.data_dir:
                kw["data_dir"] = self.data_dir
            kw["dtype"] = self.dtype
            kw["loss_scale"] = get_loss_scale(self.dtype, self.loss_scale)
            kw["hooks"] = self.hooks
            kw["hook_every_n"] = self.log_every_n_steps
            kw["model_dir"] = self.savedata
            kw["epochs_between_evals"] = getattr(self, "epochs_between_evals", 1)
            if self.stop_threshold is not None:
                kw["stop_threshold"] = self.stop_threshold
            if self.ready_steps:
                kw["ready_steps"] = self.ready_steps
            if self.batch_size:
                kw["batch_size"] = self.batch_size
        if self.model in ("cifar10", "imagenet"):
            if self.resnet_size:
                kw["resnet_size"] = self.resnet_size
            kw["resnet_version"] = self.resnet_version
        if self.model == "mnist" and self.debug_steps:
            kw["debug_steps"] = self.debug_steps
        if self.model == "mnist":
            kw["probabilities_every_n"] = getattr(self, "log_probabilities_every_n", 50)
        return kw

    def apply_runtime_modes(self) -> None:
        """Environment / library switches of --debug_kernels and --deterministic.  Call before
        the first GPU use: HIP reads its launch-serialisation variables when the runtime initialises."""
        import os
        import random
        if self.debug_kernels:
            os.environ["AMD_SERIALIZE_KERNEL"] = "3"
            os.environ["HIP_LAUNCH_BLOCKING"] = "1"
            os.environ["DTF_HIP_GRAPH"] = "0"
            os.environ["DTF_DEBUG"] = "1"  # debug kernel build + per-launch checks (ops._DebugLib)
        if self.deterministic:
            seed = 0 if self.seed is None else int(self.seed)
            if self.seed is None:
                self.seed = seed
            random.seed(seed)
            try:
                import numpy as np
                np.random.seed(seed)
            except ImportError:
                pass
            torch.manual_seed(seed)
            torch.use_deterministic_algorithms(True, warn_only=True)
            torch.backends.cudnn.benchmark = False
            torch.backends.cudnn.deterministic = True
            os.environ["DTF_DETERMINISTIC"] = "1"  # ops.lib() loads the deterministic build
            if self.backend == "auto" and not hip_deterministic(self):
                self.backend = "torch"  # this family's HIP path still has order-dependent reductions
        if (getattr(self, "dtype", "bf16") == "fp16" and self.backend != "torch"
                and self.model in ("cifar10", "imagenet") and self.resnet_version == 2):
            os.environ["DTF_HALF"] = "1"  # ops.lib() loads the fp16 build of the kernels (libdtf_kernels_f16.so)

    def inject_nan_schedule(self) -> Dict[int, List[int]]:
        out: Dict[int, List[int]] = {}
        for spec in self.inject_nan_member:
            mid, rnd = spec.split("@")
            out.setdefault(int(rnd), []).append(int(mid))
        return out


def hip_deterministic(args) -> bool:
    """Model families whose HIP step has a deterministic (bitwise-replayable) build: CIFAR ResNet v2 and v1 (64
    statistic replicas, capped workgroups; v1's BN-backward reductions as per-image rows added in image order),
    MNIST (one workgroup per member for every accumulation) and the ImageNet bottleneck nets (every cross-workgroup
    sum as int64 fixed point with integer atomics, common.h DTF_FIXED_ACC)."""
    dt = getattr(args, "dtype", "bf16")
    # fp32: the fp32 steps accumulate every cross-workgroup sum in int64 fixed point in the deterministic build too;
    # fp16 (ResNet v2): the deterministic half build (libdtf_kernels_f16_det.so)
    if dt == "fp16":
        return args.model in ("cifar10", "imagenet") and getattr(args, "resnet_version", 2) == 2
    return args.model in ("mnist", "cifar10", "imagenet") and dt in ("bf16", "fp32")


def parse_main_args(argv=None, defaults=None) -> MainArgs:
    p = build_parser(defaults)
    args = p.parse_args(argv, namespace=MainArgs())
    if args.pop_size is not None:
        args.population_size = args.pop_size
    if args.resnet_version == 1 and args.dtype == "fp16":
        p.error("ResNet version 1 is not currently supported with fp16. Please use version 2 instead.")
    if args.dtype == "fp32" and args.model in ("cifar10", "mnist", "imagenet"):
        # every family has an fp32 HIP step (engine/hip_f32.py, hip_mnist_f32.py, hip_imagenet_f32.py:
        # v_mfma_f32_16x16x4_f32, fp32 tensors); a static loss scale is a PyTorch-path feature
        if args.loss_scale is not None and args.loss_scale != 1:
            if args.backend == "hip":
                p.error("--loss_scale with --dtype fp32: the fp32 HIP step does not scale the loss; use --backend torch")
            args.backend = "torch"
    elif args.dtype == "fp16" and args.model in ("cifar10", "imagenet") and args.resnet_version == 2:
        # fp16 ResNet v2 runs the half build of the HIP kernels (ops/csrc/common.h DTF_HALF: fp16 storage,
        # v_mfma_f32_16x16x32_f16) with the reference's static loss scaling (default 128, _performance.py:30-33):
        # the head differentiates loss_scale * loss, the fused optimizer unscales (resnet_run_loop.py:284-294)
        # --deterministic loads the deterministic half build (libdtf_kernels_f16_det.so: DTF_HALF + the
        # deterministic build's fixed-order reductions)
        if args.debug_kernels and args.backend != "torch":
            p.error("--dtype fp16 with --debug_kernels: the fp16 kernel build has no debug variant; use "
                    "--backend torch")
        # (apply_runtime_modes sets DTF_HALF=1: ops.lib() then loads libdtf_kernels_f16.so)
    elif args.dtype != "bf16" and args.model != "toy":
        # fp16 of the families without a half-build step (MNIST; ResNet v1 is rejected above) runs on the PyTorch
        # backend with static loss scaling
        if args.backend == "hip":
            p.error("--dtype %s: the %s HIP kernels have no %s build; use --backend torch (or auto)"
                    % (args.dtype, args.model, args.dtype))
        args.backend = "torch"
    elif args.loss_scale is not None and args.loss_scale != 1 and args.backend != "torch" and args.model != "toy":
        p.error("--loss_scale applies to the fp16 / fp32 PyTorch path; bf16 needs no loss scaling "
                "(pass --backend torch to scale anyway)")
    if args.deterministic and args.backend == "hip" and args.model != "toy" and not hip_deterministic(args):
        p.error("--deterministic with --backend hip: the %s HIP step has no deterministic build yet; use --backend "
                "auto (deterministic PyTorch algorithms) or torch" % args.model)
    if args.epochs_between_evals < 1:
        p.error("--epochs_between_evals must be >= 1")
    if args.deterministic and args.debug_kernels:
        # the debug kernel build keeps the release reductions (8 replicas, atomics): not replayable
        p.error("--deterministic cannot be combined with --debug_kernels (the debug build is not the "
                "deterministic one)")
    if args.benchmark_logger_type == "BenchmarkFileLogger" and not args.benchmark_log_dir:
        p.error("--benchmark_logger_type BenchmarkFileLogger needs --benchmark_log_dir")
    return args
