"""XCD-aware work order of the ImageNet plan (engine/hip_imagenet.py _xcd_order): a permutation of the work items
that (mode 1) puts every run of operand-sharing items on one XCD (positions 8 apart: workgroup k runs on XCD k % 8)
and (mode 2, 8k members of equal work) every member's items on XCD m % 8."""
import pytest

from distributedtf_amd.engine import hip_imagenet as H


def _items(nmem, per_mem_runs, ng):
    return [[s, p, p + 1, c] for s in range(nmem) for p in range(per_mem_runs) for c in range(ng)]


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("nmem,runs,ng", [(8, 5, 3), (8, 16, 1), (2, 9, 4), (1, 13, 2), (16, 3, 2)])
def test_xcd_order_is_a_permutation_with_locality(monkeypatch, mode, nmem, runs, ng):
    monkeypatch.setattr(H, "_CG_XCD", mode)
    items = _items(nmem, runs, ng)
    out = H._ImageNetPlan._xcd_order(items, ng)
    assert sorted(map(tuple, out)) == sorted(map(tuple, items))
    xcd = {}
    for k, it in enumerate(out):
        xcd.setdefault((it[0], it[1]), set()).add(k % 8)
    if mode >= 2 and nmem % 8 == 0:
        for k, it in enumerate(out):
            assert it[0] % 8 == k % 8  # member m on XCD m % 8
    elif mode == 3 and 8 % nmem == 0:  # member m on XCDs m, m + nmem, ..; its complete blocks of 8 / nmem runs local
        q = 8 // nmem
        for k, it in enumerate(out):
            assert k % nmem == it[0] % nmem
        for (s, p), xs in xcd.items():
            if p < runs // q * q:
                assert len(xs) == 1, (s, p, xs)
    else:
        full = (len(items) // ng) // 8 * 8  # runs in complete blocks of 8
        for (s, p), xs in xcd.items():
            if s * runs + p < full:
                assert len(xs) == 1, (s, p, xs)  # a run's items share one XCD


def test_xcd_order_off(monkeypatch):
    monkeypatch.setattr(H, "_CG_XCD", 0)
    items = _items(8, 4, 2)
    assert H._ImageNetPlan._xcd_order(items, 2) == items
