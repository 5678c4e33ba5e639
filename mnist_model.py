"""Reference-compatible module (reference ``mnist_model.py``)."""
from distributedtf_amd.models.mnist_model import MNISTModel  # noqa: F401
