"""A/B of the step plans' work-split constants without editing the engine (diagnostic).

    python tools/ab_bench.py --set FWD_ITERS_PER_WG=1 --set DUAL_WG.64=32 --set DUAL_CS=32:64 -- --pop 8 --steps 60

Each ``--set`` overrides one module constant of ``engine/hip_resnet.py`` in this process only: ``NAME=int``,
``NAME.key=int`` for a dict constant, ``NAME=a:b:c`` for a tuple of ints, ``NAME=`` empties a dict constant;
``imagenet:NAME...`` addresses ``engine/hip_imagenet.py`` instead.  Everything after ``--`` goes to
``bench.py``.  Values are parsed as integers (no evaluation of the text).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def apply(sets):
    from distributedtf_amd.engine import hip_imagenet, hip_resnet
    for item in sets:
        name, val = item.split("=", 1)
        hr = hip_resnet
        if name.startswith("imagenet:"):  # a constant of engine/hip_imagenet.py
            hr, name = hip_imagenet, name[len("imagenet:"):]
        if isinstance(getattr(hr, name, None), dict) and val == "":
            getattr(hr, name).clear()  # NAME= empties a dict constant (e.g. switches a per-shape path off)
        elif "." in name:
            base, key = name.split(".", 1)
            d = getattr(hr, base)
            assert isinstance(d, dict), base
            d[int(key)] = int(val)
        else:
            cur = getattr(hr, name)
            if isinstance(cur, tuple):
                setattr(hr, name, tuple(int(v) for v in val.split(":") if v))
            else:
                setattr(hr, name, int(val))
        print("ab_bench: %s" % item, file=sys.stderr)


def main():
    argv = sys.argv[1:]
    if "--" in argv:
        i = argv.index("--")
        ours, bench_args = argv[:i], argv[i + 1:]
    else:
        ours, bench_args = argv, []
    sets = [ours[k + 1] for k in range(len(ours)) if ours[k] == "--set"]
    apply(sets)
    sys.argv = ["bench.py"] + bench_args
    import bench
    bench.main()


if __name__ == "__main__":
    main()
