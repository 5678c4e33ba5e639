"""CPU checks of the measurement tools whose outputs are committed under profiles/."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import imagenet_roofline  # noqa: E402
import pmc_summary  # noqa: E402


def test_imagenet_roofline_model_matches_resnet50():
    """The launch model covers ResNet-50 v2 at 224: 4.1 GMAC forward per image (8.2 GFLOP), backward = 2x forward
    (data + weight gradients), every conv launch once per pass."""
    ls = imagenet_roofline.launches(1)
    fwd = sum(fl for fam, lab, b, fl in ls if fam == "conv fwd")
    dgr = sum(fl for fam, lab, b, fl in ls if fam == "conv dgrad")
    wgr = sum(fl for fam, lab, b, fl in ls if fam == "conv wgrad")
    stem = [fl for fam, lab, b, fl in ls if lab.startswith("stem 7x7/2")][0]
    # the space-to-depth stem runs K = 4x4 taps x 16 block channels = 256, of which 7x7x3 = 147 are real
    assert 7.6e9 < fwd - stem + stem * 147 / 256 < 8.3e9, fwd
    assert abs(wgr - fwd) / fwd < 1e-9
    assert abs(dgr - (fwd - stem)) / fwd < 1e-9  # no data gradient of the stem
    n_conv = sum(1 for fam, *_ in ls if fam == "conv fwd")
    assert n_conv == 53  # stem + 16 blocks x 3 + 4 projections


def test_pmc_summary_per_wave(tmp_path):
    p = tmp_path / "counters_1.csv"
    cols = ["Kernel_Name", "Counter_Name", "Counter_Value"]
    rows = [("void (anonymous namespace)::k<1, 2>((anonymous namespace)::A)", n, v) for n, v in
            (("SQ_WAVES", 4), ("SQ_INSTS_MFMA", 40), ("SQ_INSTS_VALU", 200), ("SQ_WAVE_CYCLES", 1000),
             ("SQ_WAIT_ANY", 250))]
    with open(p, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(cols)
        w.writerows(rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(p)],
                         capture_output=True, text=True, check=True).stdout
    line = [l for l in out.splitlines() if l.startswith("k<1, 2>")][0].split()
    assert line[2] == "4" and line[3] == "10" and line[4] == "50"  # waves, MFMA/w, VALU/w
    assert "25.0" in line and "0.20" in line  # WAIT_ANY %, MFMA:VALU
    assert pmc_summary.family("void (anonymous namespace)::k<1, 2>(x)") == "k<1, 2>"
