"""Side-stream state import + captured-step replay check (tests/test_gpu_state_import.py; run with
DTF_DETERMINISTIC=1 so that two members with the same state, batch and hyperparameters step bitwise identically).

ProcessGroupNCCL receives into the destination state row on its own stream; ``work.wait()`` makes the current stream
wait for it; parallel/dataplane.py then calls ``on_state_imported`` (host step counter, bf16 weight-shadow refresh)
before the next REPLAY of the captured step graph.  Here the copy runs on a side stream kept busy first (an unordered
replay would read the old row), the current stream waits on it, and the replayed step must leave the importing member
bitwise equal to the source member.  Prints IMPORT_OK."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributedtf_amd import ops  # noqa: E402
from distributedtf_amd.engine.population import PopulationEngine  # noqa: E402
from distributedtf_amd.models.resnet import ResNetArch, cifar_config  # noqa: E402

assert ops.deterministic_mode(), "run with DTF_DETERMINISTIC=1"


def run(opt):
    dev = torch.device("cuda")
    arch = ResNetArch(cifar_config(14))
    e = PopulationEngine(arch, 2, dev, backend="hip")
    hp = {"opt_case": {"optimizer": opt, "lr": 0.05, "momentum": 0.9}, "batch_size": 32,
          "regularizer": "l2_regularizer", "weight_decay": 2e-4, "initializer": "he_init", "decay_steps": 0,
          "decay_rate": 1.0}
    for i in range(2):
        e.add_member(None, hp, seed=21 + i)
    g = torch.Generator().manual_seed(4)
    xa, ya = torch.randn(32, 32, 32, 3, generator=g).to(dev), torch.randint(0, 10, (32,), generator=g).to(dev)
    xb, yb = torch.randn(32, 32, 32, 3, generator=g).to(dev), torch.randint(0, 10, (32,), generator=g).to(dev)
    for _ in range(3):  # member 1 runs ahead on its own plan
        e.train_step([1], [(xb, yb)], [hp], [0.05])
    for _ in range(3):  # both members, different batches: warm-up + capture of the pop-2 plan, then replays
        e.train_step([0, 1], [(xa, ya), (xb, yb)], [hp, hp], [0.05, 0.05])
    torch.cuda.synchronize()
    plan = next(p for k, p in e.backend._plans.items() if len(k[0]) == 2)
    assert plan.graph is not None, "the pop-2 step must be a captured graph"
    assert not torch.equal(e.state[0], e.state[1])
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    src = e.state[1].clone()
    with torch.cuda.stream(side):
        torch.cuda._sleep(50_000_000)  # the side stream is still busy when the replay is enqueued
        e.state[0].copy_(src, non_blocking=True)
    torch.cuda.current_stream().wait_stream(side)
    e.on_state_imported(0, e.host_step[1])
    e.train_step([0, 1], [(xb, yb), (xb, yb)], [hp, hp], [0.05, 0.05])
    torch.cuda.synchronize()
    same = torch.equal(e.state[0], e.state[1])
    sc = e.step_col()
    step_ok = float(sc[0]) == float(sc[1]) == float(e.host_step[1]) and e.host_step[0] == e.host_step[1]
    diff = float((e.state[0].double() - e.state[1].double()).abs().max())
    print("%s: rows bitwise equal after the replayed step %s (max |diff| %.3g), step counters %s %s" %
          (opt, same, diff, sc[:2].tolist(), e.host_step[:2]), flush=True)
    return same and step_ok


ok = all([run("Momentum"), run("Adam")])
print("IMPORT_OK" if ok else "IMPORT_FAIL")
sys.exit(0 if ok else 1)
