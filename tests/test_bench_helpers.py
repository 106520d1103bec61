"""bench.py host-side helpers (CPU)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.parametrize("n", [1, 2, 7, 4096, 4097, (1 << 24) + 1, 1 << 28, 1 << 29, (1 << 31) + 5])
def test_sample_index_stays_in_bounds(n):
    """Sample indices of the N>1 correctness check: int64, first 0, last n-1, never n (a float32 linspace
    over 2^28 elements rounds its last index up to 2^28, one past the end of the bucket)."""
    import bench
    idx = bench.sample_index(n, "cpu")
    assert idx.dtype.is_floating_point is False
    assert int(idx[0]) == 0 and int(idx[-1]) == n - 1
    assert bool((idx[1:] >= idx[:-1]).all())


def test_factorizations():
    import bench
    assert bench._factorizations(8) == [[2, 2, 2], [2, 4], [4, 2], [8]]
    assert bench._factorizations(1) == []
