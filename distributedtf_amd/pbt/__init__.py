from .hparams import (WorkerInstruction, generate_random_hparam, get_hp_range_definition, load_hp_space,
                      perturb_hparams)
from .exploit import ExploitPair, plan_exploit, rank_population
