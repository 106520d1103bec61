"""Pins tests/sample_fold.py (the per-element fold the full-size GPU tests check against) to the oracle."""
import numpy as np
import pytest

import ftar_inputs as fi
import oracle_lib
import sample_fold


@pytest.mark.parametrize("P", [2, 3, 4, 5, 7, 8])
@pytest.mark.parametrize("form", ["ring", "tree"])
@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("n", [1, 17, 1003, 65541])
def test_sample_fold_matches_oracle(P, form, dt, n):
    ins = [fi.fill(dt, 77, r, n) for r in range(P)]
    topo = "1" if form == "ring" else str(P)
    ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt])
    bf16 = dt == "bf16"
    xs = np.stack([fi.bf16_bits_to_f32(x) if bf16 else x for x in ins])
    idx = np.arange(n)
    got = sample_fold.fold(xs, idx, n, form, bf16=bf16)
    exp = fi.bf16_bits_to_f32(ref[0]) if bf16 else ref[0]
    assert np.array_equal(got.view(np.uint32), np.ascontiguousarray(exp, np.float32).view(np.uint32))
    for r in range(1, P):   # every rank ends with the same bits
        assert np.array_equal(ref[r], ref[0])
