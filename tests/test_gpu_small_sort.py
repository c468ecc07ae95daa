"""The engine's post-scan key-value sort (engine.hip sort_pairs: hipcub, or the
two-launch k_tile_sort + k_tile_merge up to 64 K pairs that measured slower)
against hipcub::DeviceRadixSort::SortPairs' contract: order by key bits
[0, end_bit), stable (numpy's stable argsort of the masked keys is the
reference).  Sizes straddle
the tile (4096) and the small-sort limit (65536); keys with many duplicates,
all-ones keys (the padding's masked key), and bits above end_bit that must be
ignored but kept in the output."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = pytest.importorskip("trivy_amd._native")
S = pytest.importorskip("trivy_amd.secret")


def _sort(keys, vals, end_bit, small=1):
    eng = S.get_engine(None)
    n = len(keys)
    ok = np.empty(n, dtype=np.uint64)
    ov = np.empty(n, dtype=np.uint32)
    N.check(N.lib.tsg_diag_sort_pairs(eng, keys.ctypes.data, vals.ctypes.data, n, end_bit, ok.ctypes.data,
                                      ov.ctypes.data, small))
    return ok, ov


@pytest.mark.parametrize("n", [1, 2, 37, 4095, 4096, 4097, 30000, 34385, 65535, 65536, 65537, 200000])
@pytest.mark.parametrize("end_bit", [64, 47, 20])
@pytest.mark.parametrize("small", [1, 0])
def test_sort_pairs_equals_stable_radix_sort(n, end_bit, small):
    rng = np.random.default_rng(n * 131 + end_bit)
    keys = rng.integers(0, 1 << 63, size=n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, size=n, dtype=np.uint64)
    # duplicates in the sorted bits (and differing bits above end_bit)
    dup = rng.random(n) < 0.3
    keys[dup] = keys[rng.integers(0, n, size=int(dup.sum()))] ^ (np.uint64(1) << np.uint64(63))
    keys[rng.random(n) < 0.01] = np.uint64(0xFFFFFFFFFFFFFFFF)
    vals = np.arange(n, dtype=np.uint32) * np.uint32(7) + np.uint32(3)
    mask = np.uint64(0xFFFFFFFFFFFFFFFF) if end_bit == 64 else np.uint64((1 << end_bit) - 1)
    order = np.argsort(keys & mask, kind="stable")
    ok, ov = _sort(keys, vals, end_bit, small)
    assert np.array_equal(ov, vals[order])
    assert np.array_equal(ok, keys[order])


def test_sort_pairs_all_equal_keys_keep_input_order():
    n = 50000
    keys = np.full(n, 12345, dtype=np.uint64)
    vals = np.arange(n, dtype=np.uint32)[::-1].copy()
    ok, ov = _sort(keys, vals, 64)
    assert np.array_equal(ov, vals) and np.array_equal(ok, keys)
