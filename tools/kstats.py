"""Summarise a rocprofv3 kernel_stats.csv: per-kernel-family time per step."""
import csv
import re
import sys


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = {}
    for r in rows:
        n = r["Name"]
        m = re.search(r"namespace\)::(\w+)", n)
        key = m.group(1) if m else n[:40]
        fam[key] = fam.get(key, 0.0) + float(r["TotalDurationNs"])
    print("total GPU time per step: %.3f ms" % (tot / 1e6 / steps))
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print("  %-40s %8.3f ms/step  %5.1f%%" % (k, v / 1e6 / steps, 100 * v / tot))
    print("top kernels:")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        print("  %8.3f ms/step avg %7.1f us x%-4s %s" % (float(r["TotalDurationNs"]) / 1e6 / steps,
                                                       float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:100]))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
