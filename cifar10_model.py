"""Reference-compatible module (reference ``cifar10_model.py``)."""
from distributedtf_amd.models.cifar10_model import Cifar10Model  # noqa: F401
