"""Reference-compatible module (reference ``constants.py``): search space + protocol enum."""
from distributedtf_amd.pbt.hparams import (WorkerInstruction, generate_random_hparam,  # noqa: F401
                                           get_hp_range_definition, load_hp_space)
