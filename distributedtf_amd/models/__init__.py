from .model_base import ModelBase
from .toy_model import ToyModel


def __getattr__(name):
    # heavy model families import lazily
    if name == "MNISTModel":
        from .mnist_model import MNISTModel
        return MNISTModel
    if name == "Cifar10Model":
        from .cifar10_model import Cifar10Model
        return Cifar10Model
    if name == "ImageNetModel":
        from .imagenet_model import ImageNetModel
        return ImageNetModel
    raise AttributeError(name)


MODEL_FAMILIES = ("toy", "mnist", "cifar10", "imagenet")


def model_class(name: str):
    name = name.lower()
    if name in ("toy", "toymodel"):
        return ToyModel
    if name in ("mnist", "mnistmodel"):
        return __getattr__("MNISTModel")
    if name in ("cifar10", "cifar", "resnet", "cifar10model"):
        return __getattr__("Cifar10Model")
    if name in ("imagenet", "resnet50", "imagenetmodel"):
        return __getattr__("ImageNetModel")
    raise ValueError("unknown model family %r" % name)
