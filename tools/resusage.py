"""Per-kernel register / occupancy table of a .hip file (hipcc -Rpass-analysis=kernel-resource-usage)."""
import re
import subprocess
import sys


def main(src, filt=""):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-c",
           src, "-o", "/tmp/_resusage.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            m = re.search(r"remark: ([^:]+): (.*)$", line)
            if not m:
                continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    dm = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout
    for r, n in zip(rows, dm.splitlines()):
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = re.sub(r"\(ConvArgs\)", "", n)
        if filt and filt not in n:
            continue
        print("%-58s vgpr %4s agpr %4s occ %2s spill v%s s%s lds %s" % (
            n[:58], r.get("VGPRs", "?"), r.get("AGPRs", "?"), r.get("Occupancy [waves/SIMD]", "?"),
            r.get("VGPRs Spill", "?"), r.get("SGPRs Spill", "?"), r.get("LDS Size [bytes/block]", "?")))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
