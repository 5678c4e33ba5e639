"""Reference-compatible module (reference ``model_base.py``)."""
from distributedtf_amd.models.model_base import ModelBase  # noqa: F401
