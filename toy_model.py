"""Reference-compatible module (reference ``toy_model.py``)."""
from distributedtf_amd.models.toy_model import ToyModel, main  # noqa: F401
