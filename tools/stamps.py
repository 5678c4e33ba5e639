"""In-kernel phase stamps of the conv_fwd_s1 / conv_bwd_fused launches of one population step (diagnostic).

    python tools/stamps.py build                 # CPU: tools/abl/libdtf_stamp.so (-DDTF_STAMP=1)
    python tools/stamps.py run --pop 1 [--batch 128]   # GPU: steps through the stamp build, prints per-launch phases

Stamps are s_memrealtime (100 MHz) reads by every wave, written by thread 0 of each workgroup (< 512) after the
kernel's last memory operation has drained.  Phases (µs, median over workgroups):
  fwd_s1: S0 entry -> S1 coefficients ready -> S2 first tile staged -> S3 loop done -> S4 stats flushed + drained
  fused:  S0 entry -> S1 coefficients -> S2 tiles staged -> S3 loop done -> S4 stats flushed -> S5 slab stored + drained
'skew' = spread of S0 over the grid (dispatch), 'span' = last drain - first entry.  Read shares, not lengths: the
drains and the stamps' own waits change the schedule.
"""
import argparse
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
LIBP = os.path.join(HERE, "abl", "libdtf_stamp.so")


def build(level=1):
    from distributedtf_amd.ops import build as kb
    os.makedirs(os.path.dirname(LIBP), exist_ok=True)
    kb.build(force=True, extra_flags=["-DDTF_STAMP=%d" % level], out=LIBP)


def run(args):
    os.environ["DTF_LIB"] = LIBP
    import numpy as np
    import torch
    from distributedtf_amd import ops
    from distributedtf_amd.models.cifar10_model import Cifar10Model
    from distributedtf_amd.pbt.cluster import sample_population
    hps = sample_population(args.pop, 2024)
    for h in hps:
        h["batch_size"] = args.batch
    ms = [Cifar10Model(i, hps[i], "/tmp/stamp_savedata/model_", seed=1, resnet_size=args.resnet_size,
                       device="cuda", capacity=args.pop, use_synthetic_data=True, checkpoint_every_round=False)
          for i in range(args.pop)]
    eng = ms[0].engine
    ds = ms[0].dataset()
    batches = [ds.batch_slice(args.batch) for _ in ms]
    for _ in range(args.steps):
        eng.train_step([m.slot for m in ms], batches, [m.hparams for m in ms], [0.1 for _ in ms])
    torch.cuda.synchronize()
    buf = np.zeros((256, 512, 16), dtype=np.uint64)
    L = ops.lib()
    L.dtf_stamp_read.argtypes = [ctypes.c_void_p, ctypes.c_long]
    assert L.dtf_stamp_read(buf.ctypes.data, buf.nbytes) == 0, "not a DTF_STAMP build"
    plan = next(iter(eng.backend._plans.values()))
    tot = {}
    print("%-34s %5s %6s %6s  %s" % ("launch", "nWG", "skew", "span", "median phase us (S1-S0, S2-S1, ...)"))
    for row, label in plan.stamp_rows:
        st = buf[row].astype(np.int64)
        live = st[:, 0] > 0
        if not live.any():
            continue
        st = st[live]
        nph = 5 if label.startswith("fused") else 4
        t0 = st[:, 0].min()
        span = (st[:, nph].max() - t0) / 100.0
        skew = (st[:, 0].max() - t0) / 100.0
        ph = [statistics.median((st[:, i + 1] - st[:, i]).tolist()) / 100.0 for i in range(nph)]
        key = label.split(" mdy")[0].split(" in=")[0]
        acc = tot.setdefault(key, [0, 0.0, [0.0] * nph])
        acc[0] += 1
        acc[1] += span
        acc[2] = [a + b for a, b in zip(acc[2], ph)]
        fine = ""
        if st[:, 8].min() > 0:  # DTF_STAMP=2 build: prologue split S0 -> work item -> weights -> tiles -> coef
            fp = [st[:, 0], st[:, 8], st[:, 9], st[:, 10], st[:, 12], st[:, 13], st[:, 11]]
            fine = " | fine wk/w/tile/cnt/dcoef/ecoef %s" % " ".join(
                "%5.2f" % (statistics.median((fp[i + 1] - fp[i]).tolist()) / 100.0) for i in range(len(fp) - 1))
        if args.verbose:
            print("%-34s %5d %6.2f %6.2f  %s  nit=%d" % (label, live.sum(), skew, span,
                                                       " ".join("%5.2f" % p for p in ph), int(st[0, 7])) + fine)
    print("per family (launches, mean span us, mean phases us):")
    for k, (n, sp, ph) in tot.items():
        print("  %-20s n=%3d span %6.2f  phases %s" % (k, n, sp / n, " ".join("%5.2f" % (p / n) for p in ph)))


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("cmd", choices=["build", "run"])
    p.add_argument("--pop", type=int, default=1)
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--resnet_size", type=int, default=56)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--verbose", type=int, default=1)
    p.add_argument("--level", type=int, default=1, help="build: 2 = also the fine prologue stamps")
    a = p.parse_args()
    build(a.level) if a.cmd == "build" else run(a)
