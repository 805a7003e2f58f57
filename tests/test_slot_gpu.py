"""The pass chain's one-wave primitives (bre_slot.hip, bre_device_check kinds 6-8): the stable LSD radix
sort of (key, value) pairs and the exclusive scan that replace rocPRIM on the photon / build / camera /
segment-sort / film-compose chain (so that it runs beside a concurrent gather).  The sort must give
numpy's stable argsort of the keys' bit range -- the permutation rocPRIM's stable radix_sort_pairs
gives -- and the scan numpy's cumulative sum, at tile edges (1024 elements per workgroup), with few
and with many distinct keys, and for every bit range the library sorts (hash 32, tree 60 / 63, segment
keys 60, pixel keys ~21 bits)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ref_sort(keys, lo, hi):
    width = hi - lo
    mask = np.uint64((1 << width) - 1) if width < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    d = (keys.astype(np.uint64) >> np.uint64(lo)) & mask
    perm = np.argsort(d, kind="stable")
    return keys[perm], perm.astype(np.int32)


@pytest.mark.parametrize("n", [1, 63, 1023, 1024, 1025, 70_001, 2_700_000])
@pytest.mark.parametrize("bits", [(0, 64), (0, 60), (0, 32), (3, 24)])
def test_slot_sort_u64(bre, n, bits):
    rng = np.random.default_rng(n + bits[1])
    keys = rng.integers(0, 2 ** 63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n).astype(np.uint64)
    if n > 100:
        keys[::7] = keys[3]  # runs of equal keys: stability
    with bre.BeamGather(0) as g:
        sk, perm = g.slot_sort(keys, *bits)
    rk, rp = _ref_sort(keys, *bits)
    assert np.array_equal(perm, rp)
    assert np.array_equal(sk, rk)


@pytest.mark.parametrize("n", [5, 1024, 4097, 600_000])
@pytest.mark.parametrize("bits", [(0, 32), (0, 21), (0, 1)])
def test_slot_sort_u32(bre, n, bits):
    rng = np.random.default_rng(7 * n + bits[1])
    hi = 2 ** bits[1] if bits[1] < 32 else 2 ** 32
    keys = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
    with bre.BeamGather(0) as g:
        sk, perm = g.slot_sort(keys, *bits)
    rk, rp = _ref_sort(keys, *bits)
    assert np.array_equal(perm, rp) and np.array_equal(sk, rk)


@pytest.mark.parametrize("n", [1, 64, 1023, 1024, 1025, 99_999, 5_000_000])
def test_slot_scan(bre, n):
    rng = np.random.default_rng(n)
    v = rng.integers(0, 40, size=n).astype(np.int32)
    with bre.BeamGather(0) as g:
        y = g.slot_scan(v)
    ref = np.zeros(n + 1, np.int64)
    ref[1:] = np.cumsum(v.astype(np.int64))
    assert np.array_equal(y, ref)
