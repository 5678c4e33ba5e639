"""Per-step GPU time distribution of a rocprofv3 kernel_trace.csv: steps split at the marker kernel (default
weight_prep_kernel, the first launch of every training step graph).  Reports the median / mean busy time per step,
the median in-step gaps and the median gap BETWEEN consecutive steps (GPU idle waiting for the host), for the
steps whose kernel count equals the most common one (training steps of one plan; eval chunks differ).

usage: step_spans.py run_kernel_trace.csv [marker]"""
import csv
import statistics
import sys
from collections import Counter


def main(path, marker="weight_prep_kernel"):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], []
    for r in rows:
        if marker in r["Kernel_Name"] and cur:
            steps.append(cur)
            cur = []
        cur.append(r)
    if cur:
        steps.append(cur)
    steps = steps[1:]  # before the first marker: init
    n_common = Counter(len(s) for s in steps).most_common(1)[0][0]
    busy, span, between = [], [], []
    for k, s in enumerate(steps):
        t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
        if len(s) == n_common:
            busy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e3)
            span.append((t1 - t0) / 1e3)
            if k + 1 < len(steps):
                between.append((int(steps[k + 1][0]["Start_Timestamp"]) - t1) / 1e3)
    print("%s: %d steps (%d with the common %d kernels)" % (path, len(steps), len(busy), n_common))
    q = lambda v: "median %.1f mean %.1f p90 %.1f" % (statistics.median(v), statistics.mean(v),
                                                      sorted(v)[int(0.9 * (len(v) - 1))])
    print("  busy us/step:  " + q(busy))
    print("  span us/step:  " + q(span))
    print("  gap to next step us: " + q(between))


if __name__ == "__main__":
    main(*sys.argv[1:])
