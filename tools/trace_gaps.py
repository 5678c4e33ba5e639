"""Per-step busy/gap analysis of a rocprofv3 kernel_trace.csv (single queue, graph-replayed steps).

usage: trace_gaps.py run_kernel_trace.csv [first_kernel_substring]
Splits the dispatch stream into steps at each occurrence of the marker kernel (default weight_prep_kernel),
then reports per step: wall span, summed kernel time, summed inter-kernel gaps, kernel count, and the
kernel families with the most time and the largest gaps before them (last complete step)."""
import csv
import re
import sys
from collections import defaultdict


def fam(n):
    m = re.search(r"namespace\)::(\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:50]


def main(path, marker="weight_prep_kernel"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        if marker in r["Kernel_Name"] and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
    steps.append(cur)
    print("steps found:", len(steps))
    for s in steps[-4:-1]:
        t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
        print("span %.1f us  busy %.1f us  gaps %.1f us  kernels %d" % ((t1 - t0) / 1e3, busy / 1e3,
                                                                       (t1 - t0 - busy) / 1e3, len(s)))
    s = steps[-2]
    by = defaultdict(lambda: [0, 0, 0.0])
    prev_end = None
    for r in s:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        f = fam(r["Kernel_Name"])
        by[f][0] += 1
        by[f][1] += en - st
        if prev_end is not None:
            by[f][2] += st - prev_end
        prev_end = en
    print("%-50s %5s %10s %10s" % ("family", "n", "busy_us", "gap_us"))
    for f, (n, b, g) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print("%-50s %5d %10.1f %10.1f" % (f[:50], n, b / 1e3, g / 1e3))


if __name__ == "__main__":
    main(*sys.argv[1:])
