"""ImageNet-shape ResNet population member (BASELINE config 5, SURVEY.md C12').

The reference's ResNet library supports bottleneck blocks and the first max-pool
(``resnet/resnet_model.py:215-320,487-529``) but ships no ImageNet entry point;
this family defines the upstream-standard config (7x7/2 stem, 3x3/2 max-pool,
[3,4,6,3] bottleneck stages, 2048 final) on synthetic 224x224x3 data.
LR: ``lr * B/256`` piecewise schedule with the same decay_steps/decay_rate rule
as the CIFAR family over 1.28M images.
"""

from __future__ import annotations

from .cifar10_model import Cifar10Model
from .resnet import ResNetArch, imagenet_config
from ..data import datasets
from ..engine import schedule

IMAGENET_NUM_TRAIN = 1281167


class ImageNetModel(Cifar10Model):
    def __init__(self, cluster_id, hparams, save_base_dir, seed=None, resnet_size=50, image_size=224,
                 num_classes=1001, **kw):
        self.image_size = int(image_size)
        self.num_classes = int(num_classes)
        super().__init__(cluster_id, hparams, save_base_dir, seed=seed, resnet_size=resnet_size, **kw)

    def make_arch(self):
        return ResNetArch(imagenet_config(self.resnet_size, self.resnet_version, self.num_classes, self.image_size))

    def make_dataset(self, device):
        shape = (self.image_size, self.image_size, 3)
        return datasets.SyntheticDataset(shape, self.num_classes, device, max_batch=256, n_eval=256)

    def learning_rate(self, step):
        b, v = schedule.cifar_boundaries(self.hparams, num_images=IMAGENET_NUM_TRAIN, batch_denom=256,
                                         total_epochs=90.0)
        return schedule.piecewise_constant(step, b, v)

    def steps_per_epoch(self):
        return int(IMAGENET_NUM_TRAIN / int(self.hparams["batch_size"]))
