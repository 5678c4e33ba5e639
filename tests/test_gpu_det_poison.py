"""Deterministic ImageNet build (int64 fixed-point accumulation, ops/csrc/common.h dtf_fx): a diverged member must
still read as diverged.  A fixed-point word cannot hold NaN / Inf, so non-finite or out-of-range partials set the
member's flag word and cg_det_finish (convg_aux.hip) writes NaN into its loss and gradient row -- the engine's
non-finite check (models/engine_model.py) then culls it as in the float build.  The healthy member of the same
step must be unaffected.  Runs in a child process: the deterministic library is chosen at load time
(DTF_DETERMINISTIC=1, ops.lib())."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import math, torch
from distributedtf_amd import ops
from distributedtf_amd.engine.population import PopulationEngine
from distributedtf_amd.models.resnet import ResNetArch, imagenet_config
assert ops.build_deterministic(), "child must load the deterministic library"
arch = ResNetArch(imagenet_config(50, 2, num_classes=1001, image_size=64))
dev = torch.device("cuda")
eng = PopulationEngine(arch, 2, dev, backend="hip")
hp = lambda: {"opt_case": {"optimizer": "gd", "lr": 0.1}, "batch_size": 4, "regularizer": "None",
              "weight_decay": 0.0, "initializer": "he_init"}
slots = [eng.add_member(None, hp(), seed=3 + i) for i in range(2)]
g = torch.Generator().manual_seed(1)
batches = [(torch.randn(4, 64, 64, 3, generator=g).to(dev), torch.randint(0, 1001, (4,), generator=g).to(dev))
           for _ in slots]
res = []
for step in range(3):
    if step == 1:  # poison member 1: a huge stem weight overflows every downstream activation
        c = arch.prog.convs[arch.prog.stem]
        eng.state[slots[1], c.off:c.off + 8] = 3e38
    l = eng.train_step(slots, batches, [hp(), hp()], [0.1, 0.1])
    torch.cuda.synchronize()
    res.append([float(v) for v in l.cpu()])
print("LOSSES", res)
assert all(math.isfinite(v) for v in res[0]), res
assert math.isfinite(res[1][0]) and math.isfinite(res[2][0]), res      # the healthy member keeps training
assert math.isnan(res[1][1]) and math.isnan(res[2][1]), res            # the poisoned one reads NaN (and stays NaN)
print("POISON_OK")
"""


def test_det_fixed_point_poison_flags_member():
    env = dict(os.environ, DTF_DETERMINISTIC="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    print(out[-3000:])
    assert r.returncode == 0 and "POISON_OK" in r.stdout, out[-3000:]
