"""MNIST CNN population member (reference ``mnist_model.py:128-201``).

Kept: optimizer from the hparams (6 TF1 optimizers, constant lr), eval on the
10k test set per epoch, ``learning_curve.csv`` = ``global_step(=epoch index),
eval_accuracy, optimizer, lr``, ``epoches_trained += 1`` per call, un-normalised
pixels by default (Appendix A5).
Changed: the dataset is loaded once and kept on the device (the reference
re-reads the gz files on every call); an "epoch" is a full pass
(``60000 / batch`` steps) unless ``debug_steps`` (the reference's 10-step debug
epoch, Appendix A4) or ``max_train_steps`` is given; data is synthetic when
``./datasets/`` is absent.  The training softmax is logged every 50 steps, as the reference's
``LoggingTensorHook`` does (``--log_probabilities_every_n``; 0 = off).
"""

from __future__ import annotations

import torch

from .engine_model import EngineModel
from .mnist import MnistArch
from ..data import datasets
from ..engine import schedule


class MNISTModel(EngineModel):
    def __init__(self, cluster_id, hparams, save_base_dir, seed=None, data_dir="./datasets/", debug_steps=None,
                 normalize=False, probabilities_every_n=50, **kw):
        self.debug_steps = debug_steps
        # the reference logs the training softmax every 50 iterations (mnist_model.py:149-151): the
        # "probabilities" hook (utils/hooks.py ProbabilitiesHook) is on by default for MNIST; 0 turns it off
        self.probabilities_every_n = int(probabilities_every_n or 0)
        self.normalize = normalize
        super().__init__(cluster_id, hparams, save_base_dir, seed=seed, data_dir=data_dir, **kw)

    def make_arch(self):
        return MnistArch()

    def make_dataset(self, device):
        synthetic = self.use_synthetic_data
        if synthetic is None:
            synthetic = not datasets.mnist_available(self.data_dir)
        if synthetic:
            # the reference evaluates on the full 10k-image test set every epoch (resnet_run_loop.py:463-466,
            # mnist_model.py:167-172): a synthetic eval set of the same size on the GPU (1k on CPU test runs)
            n_eval = datasets.MNIST_NUM_TEST if torch.device(device).type == "cuda" else 1000
            return datasets.SyntheticDataset((28, 28, 1), 10, device, max_batch=256, n_eval=n_eval)
        trx, tr_y, tex, te_y = datasets.load_mnist(self.data_dir, self.normalize)
        return datasets.DeviceDataset(trx, tr_y, tex, te_y, device)

    def learning_rate(self, step):
        return schedule.constant_lr(self.hparams, step)

    def steps_per_epoch(self):
        if self.debug_steps:
            return int(self.debug_steps)
        return int(datasets.MNIST_NUM_TRAIN / int(self.hparams["batch_size"]))

    def finish_round(self, num_epoch):
        super().finish_round(1)  # reference adds 1 per call regardless of num_epoch

    def csv_row(self, accuracy):
        opt = self.hparams["opt_case"]
        return (["global_step", "eval_accuracy", "optimizer", "lr"],
                {"global_step": self.epoches_trained, "eval_accuracy": accuracy,
                 "optimizer": opt["optimizer"], "lr": opt["lr"]})
