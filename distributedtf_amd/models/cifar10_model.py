"""CIFAR-10 ResNet population member.

Reference: ``cifar10_model.py:10-33`` (adapter) -> ``resnet/cifar10_main.py``
(model config, LR schedule, flags) -> ``resnet/resnet_run_loop.py`` (train /
eval loop, ``learning_curve.csv``).  Behaviour kept:
  * ResNet ``resnet_size`` (6n+2; reference default 50 -> n=8), version 2;
  * one "epoch" = ``int(50000 / batch_size)`` steps (``max_train_steps`` caps it);
  * LR: ``lr * B/128`` with the decay_steps/decay_rate piecewise schedule;
  * loss = softmax CE + conv-kernel regularizer (l1 / l2 / l1_l2, weight_decay);
  * eval accuracy on the 10k test set after each round; CSV columns
    ``epochs, eval_accuracy, optimizer, learning_rate, decay_rate, decay_steps,
    initializer, regularizer, weight_decay, batch_size, model_id[, momentum]
    [, grad_decay]`` (``resnet_run_loop.py:469-503``); ``learning_rate`` is the
    flag lr, not the decayed one (Appendix A13).

Differences: members are resident in the shared population engine (no graph
rebuild / checkpoint restore per call); default data is synthetic (no network
for the dataset); bf16 compute with fp32 master weights and BN statistics.
"""

from __future__ import annotations

import torch

from .engine_model import EngineModel
from .resnet import ResNetArch, cifar_config
from ..data import datasets
from ..engine import schedule

DEFAULT_CIFAR_DIR = "/home/K8S/dataset/cifar10"


class Cifar10Model(EngineModel):
    def __init__(self, cluster_id, hparams, save_base_dir, seed=None, resnet_size=50, resnet_version=2,
                 data_dir=DEFAULT_CIFAR_DIR, **kw):
        self.resnet_size = int(resnet_size)
        self.resnet_version = int(resnet_version)
        super().__init__(cluster_id, hparams, save_base_dir, seed=seed, data_dir=data_dir, **kw)

    def make_arch(self):
        return ResNetArch(cifar_config(self.resnet_size, self.resnet_version))

    def make_dataset(self, device):
        synthetic = self.use_synthetic_data
        if synthetic is None:
            synthetic = not datasets.cifar10_available(self.data_dir)
        if synthetic == "learnable":
            # class-template images through the real input path (augmentation, per-image standardisation): eval
            # accuracy can climb above chance without the real dataset (--use_synthetic_data learnable)
            on_gpu = torch.device(device).type == "cuda"
            trx, tr_y, tex, te_y = datasets.learnable_cifar(n_train=20000 if on_gpu else 2000,
                                                            n_test=datasets.CIFAR_NUM_TEST if on_gpu else 500)
            return datasets.DeviceDataset(trx, tr_y, tex, te_y, device, augment=datasets.augment_cifar,
                                          eval_transform=datasets.eval_cifar)
        if synthetic:
            # the reference evaluates on the full 10k-image test set every epoch (resnet_run_loop.py:463-466,
            # mnist_model.py:167-172): a synthetic eval set of the same size on the GPU (1k on CPU test runs)
            n_eval = datasets.CIFAR_NUM_TEST if torch.device(device).type == "cuda" else 1000
            return datasets.SyntheticDataset((32, 32, 3), 10, device, max_batch=256, n_eval=n_eval)
        trx, tr_y, tex, te_y = datasets.load_cifar10(self.data_dir)
        return datasets.DeviceDataset(trx, tr_y, tex, te_y, device, augment=datasets.augment_cifar,
                                      eval_transform=datasets.eval_cifar)

    def learning_rate(self, step):
        return schedule.cifar_lr(self.hparams, step)

    def steps_per_epoch(self):
        return int(datasets.CIFAR_NUM_TRAIN / int(self.hparams["batch_size"]))

    def csv_row(self, accuracy):
        hp = self.hparams
        opt = hp["opt_case"]
        fields = ["epochs", "eval_accuracy", "optimizer", "learning_rate", "decay_rate", "decay_steps",
                  "initializer", "regularizer", "weight_decay", "batch_size", "model_id"]
        row = {"epochs": self.epoches_trained, "eval_accuracy": accuracy, "optimizer": opt["optimizer"],
               "learning_rate": opt["lr"], "decay_rate": hp.get("decay_rate"), "decay_steps": hp.get("decay_steps"),
               "initializer": hp.get("initializer"), "regularizer": hp.get("regularizer"),
               "weight_decay": hp.get("weight_decay"), "batch_size": hp.get("batch_size"),
               "model_id": self.cluster_id}
        if opt["optimizer"] in ("Momentum", "RMSProp"):
            fields.append("momentum")
            row["momentum"] = opt.get("momentum")
        if opt["optimizer"] == "RMSProp":
            fields.append("grad_decay")
            row["grad_decay"] = opt.get("grad_decay")
        fields.append("effective_lr")
        row["effective_lr"] = self.learning_rate(self.global_step)
        return fields, row
