"""Per-kernel-family PMC summary of rocprofv3 --pmc counter_collection CSVs (tools/gpu_pmc_pop.sh output).

    python tools/pmc_summary.py gpurun_out/pmc/counters_*.csv

Counters are summed over every dispatch of a family (kernel name up to its template arguments' closing '>') and
reported per wave: MFMA, VALU, LDS and VMEM instructions, LDS bank-conflict cycles; plus the fraction of wave
cycles parked in s_waitcnt / barriers (SQ_WAIT_ANY / SQ_WAVE_CYCLES, both in quad-cycles) and the MFMA:VALU
instruction ratio.  Families missing a counter group show '-'.
"""

from __future__ import annotations

import collections
import csv
import sys


def family(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:60]


def main(paths):
    tot = collections.defaultdict(lambda: collections.Counter())
    for p in paths:
        for r in csv.DictReader(open(p)):
            tot[family(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    cols = ["waves", "MFMA/w", "VALU/w", "LDS/w", "VMEM/w", "bankcf/w", "WAIT_ANY%", "MFMA:VALU", "FETCH MB"]
    print("%-60s " % "kernel family" + " ".join("%9s" % c for c in cols))
    for fam, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        w = c.get("SQ_WAVES", 0)

        def per(k):
            return "%9.0f" % (c[k] / w) if w and k in c else "%9s" % "-"
        wait = "%9.1f" % (100 * c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]) if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in c \
            else "%9s" % "-"
        ratio = "%9.2f" % (c["SQ_INSTS_MFMA"] / c["SQ_INSTS_VALU"]) if c.get("SQ_INSTS_VALU") and "SQ_INSTS_MFMA" in c \
            else "%9s" % "-"
        fetch = "%9.1f" % (c["FETCH_SIZE"] / 1024) if "FETCH_SIZE" in c else "%9s" % "-"  # KB -> MB
        print("%-60s %9.0f %s %s %s %s %s %s %s %s" % (fam, w, per("SQ_INSTS_MFMA"), per("SQ_INSTS_VALU"),
                                                        per("SQ_INSTS_LDS"), per("SQ_INSTS_VMEM_RD"),
                                                        per("SQ_LDS_BANK_CONFLICT"), wait, ratio, fetch))


if __name__ == "__main__":
    main(sys.argv[1:])
