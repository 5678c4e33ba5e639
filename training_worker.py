"""Reference-compatible module (reference ``training_worker.py``)."""
from distributedtf_amd.pbt.worker import TrainingWorker  # noqa: F401
