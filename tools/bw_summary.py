"""Achieved memory traffic per kernel family: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (KB per dispatch, L2 <->
fabric: HBM or the MALL) joined with a kernel trace's durations (a separate, counter-free run of the same bench).

    python tools/bw_summary.py <fetch counters.csv> <write counters.csv> <kernel_stats.csv>

Per family: dispatches, mean duration, mean fetched / written MB per dispatch, and the achieved rate (fetch + write)
/ duration in TB/s -- compared with the ~6.3 TB/s a streaming copy reaches on MI355X HBM3E (MI355X_MICROARCH.md),
a family near it is bandwidth-bound and VALU / MFMA work inside it is hidden.  The traffic counters see L2 misses
only: re-reads that hit the XCD's 4 MB L2 are not counted (they cost no HBM bandwidth).
"""
from __future__ import annotations

import collections
import csv
import sys


def family(name: str) -> str:
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:58]


def counters(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[family(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) / 1024.0 for k, v in d.items()}  # MB per dispatch


def main(fpath, wpath, spath):
    fetch, write = counters(fpath, "FETCH_SIZE"), counters(wpath, "WRITE_SIZE")
    stats = {}
    for r in csv.DictReader(open(spath)):
        stats[family(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]))
    tot = sum(v[2] for v in stats.values())
    print("%-58s %6s %8s %8s %8s %7s %6s" % ("kernel family", "calls", "us", "rd MB", "wr MB", "TB/s", "time%"))
    for k, (n, us, t) in sorted(stats.items(), key=lambda kv: -kv[1][2]):
        if k not in fetch or k not in write:
            continue
        mb = fetch[k] + write[k]
        print("%-58s %6d %8.1f %8.1f %8.1f %7.2f %5.1f%%" % (k, n, us, fetch[k], write[k], mb / us if us > 0 else 0.0, 100 * t / tot))


if __name__ == "__main__":
    main(*sys.argv[1:4])
