"""Multi-process runs of the real entry points on CPU (gloo), the rehearsal of the multi-GPU paths:

* ``bench.py`` at world 4 and 8 (owner map, cross-rank exploit with ``batch_isend_irecv``, metric all-gather,
  max-over-ranks timing, one JSON line from rank 0) -- the driver's N-GPU launch line with the torch backend;
* ``main_manager.py --model toy --mode master_worker`` at world 2 over the TorchComm TCPStore mailbox
  (reference config 1: ``mpirun -n 2 python main_manager.py``, README.md:20-23).
Reference: ``/root/reference/README.md:20-27``, ``test_runner.sh:5-24``.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(n, args, cwd, timeout):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""),
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port())] + args
    return subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [4, 8])
def test_bench_multiprocess_gloo(tmp_path, world):
    r = _torchrun(world, [os.path.join(REPO, "bench.py"), "--gpus", str(world), "--steps", "4", "--warmup", "1",
                          "--backend", "torch", "--resnet_size", "8", "--batch", "4"], str(tmp_path), 540)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["steps"] == 4 and out["value"] > 0
    assert out["config"]["exploits_timed"] >= 1  # the cross-rank exploit ran inside the timed region
    assert out["config"]["global_batch"] == 8 * 4
    assert out["config"]["parallelism"] == "pbt_pop8_%dmembers_per_gpu" % (8 // world)


@pytest.mark.timeout(300)
def test_main_manager_toy_master_worker_torchcomm(tmp_path):
    r = _torchrun(2, [os.path.join(REPO, "main_manager.py"), "4", "--model", "toy", "--mode", "master_worker",
                      "--rounds", "3", "--epochs_per_round", "2", "--seed", "1"], str(tmp_path), 280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    sd = tmp_path / "savedata"
    best = json.load(open(sd / "best_model.json"))
    assert set(best) == {"best_model_id", "best_acc", "best_hparams"}
    init = json.load(open(sd / "initial_hp.json"))
    assert sorted(d["model_id"] for d in init) == [0, 1, 2, 3]
    for f in ("toy_PBT.png", "acc_PBT.png", "lr_PBT.png", "best3_PBT.png"):
        assert (sd / f).is_file(), f
    for i in range(4):
        rows = open(sd / ("model_%d" % i) / "learning_curve.csv").read().strip().splitlines()
        assert len(rows) == 1 + 3 * 2  # one row per toy step (toy_model.py:52-61)
    assert open(tmp_path / "test_results.txt").read().startswith("n = 2, pop_size = 4")
    assert "Copied:" in r.stdout


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode,world", [("spmd", 2), ("master_worker", 3)])
def test_main_manager_per_rank_benchmark_logs(tmp_path, mode, world):
    """Every training process logs its own members' eval results (resnet_run_loop.py:466) to its own
    BenchmarkFileLogger directory: rank 0 -> <dir>, rank k -> <dir>/rank_k.  master_worker at world 3 also runs
    the exploit copy between two worker ranks with the winner's step sent on the control plane."""
    r = _torchrun(world, [os.path.join(REPO, "main_manager.py"), "4", "--model", "cifar10", "--resnet_size", "8",
                          "--use_synthetic_data", "true", "--backend", "torch", "--max_train_steps", "2",
                          "--rounds", "2", "--seed", "3", "--mode", mode, "--benchmark_logger_type",
                          "BenchmarkFileLogger", "--benchmark_log_dir", "blog"], str(tmp_path), 540)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    acc = []
    for k in range(world):
        d = tmp_path / "blog" / ("rank_%d" % k if k else "")
        p = d / "metric.log"
        if mode == "master_worker" and k == 0:
            assert not p.exists() or all(json.loads(l)["name"] != "accuracy" for l in open(p))  # master trains none
            continue
        assert p.is_file(), p
        acc += [json.loads(l) for l in open(p) if json.loads(l)["name"] == "accuracy"]
    assert len(acc) == 4 * 2  # every member's eval of both rounds, whichever rank trained it
    assert json.load(open(tmp_path / "blog" / "benchmark_run.log"))["status"] == "success"
    assert "Copied:" in r.stdout
