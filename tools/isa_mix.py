"""Static instruction mix per kernel of a gfx950 .s file (hipcc --cuda-device-only -S)."""
import collections
import re
import sys


def main(path, pat):
    cur, cnt = None, None
    out = []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            if cur and pat in cur:
                out.append((cur, cnt))
            cur, cnt = m.group(1), collections.Counter()
            continue
        if cur is None:
            continue
        t = line.strip()
        if not t or t[0] in ".;_" or t.endswith(":"):
            if t.startswith(".Lfunc_end"):
                if pat in cur:
                    out.append((cur, cnt))
                cur = None
            continue
        op = t.split()[0]
        cnt[op] += 1
    for name, c in out:
        mf = sum(v for k, v in c.items() if k.startswith("v_mfma"))
        acc = sum(v for k, v in c.items() if k.startswith("v_accvgpr"))
        valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith(("v_mfma", "v_accvgpr")))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        vm = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_", "flat_")))
        sa = sum(v for k, v in c.items() if k.startswith("s_"))
        print("%s\n  mfma %d valu %d accvgpr %d lds %d vmem %d salu %d" % (name[:100], mf, valu, acc, lds, vm, sa))
        top = sorted(((v, k) for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma")),
                     reverse=True)[:30]
        print("  " + ", ".join("%s=%d" % (k, v) for v, k in top))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
