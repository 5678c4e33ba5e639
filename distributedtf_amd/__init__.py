"""distributedtf_amd: MI355X-native population-based training (PBT).

Layers (see SURVEY.md §1 for the reference's):
  pbt/       search space, explore rule, exploit planner, PBTCluster / SPMD driver, worker, reports
  parallel/  control plane (TCPStore / gloo) and data plane (RCCL send/recv over xGMI), launcher
  models/    ModelBase API, Toy / MNIST / CIFAR-10 ResNet / ImageNet-shape ResNet families
  engine/    population engine (flat per-member state rows), optimizers, LR schedules, HIP ResNet executor
  ops/       hand-written CDNA4 HIP kernels (gfx950) + Python bindings
  data/      CIFAR / MNIST readers, synthetic device batches, on-device augmentation
  utils/     flags/config, metric logger, hooks, profiling, model helpers
"""

__version__ = "0.1.0"
