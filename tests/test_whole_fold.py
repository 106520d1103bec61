"""Pins tests/whole_fold.py (the whole-bucket fold the full-size GPU tests compare against) to the oracle."""
import numpy as np
import pytest

import ftar_inputs as fi
import oracle_lib
import whole_fold


def _torch_in(x, dt):
    import torch
    t = torch.from_numpy(x.view(np.int16) if dt == "bf16" else x)
    return t.view(torch.bfloat16) if dt == "bf16" else t


@pytest.mark.parametrize("P", [2, 3, 5, 8])
@pytest.mark.parametrize("form", ["ring", "tree"])
@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("n", [1, 7, 1003, 65541])
def test_whole_fold_matches_oracle(P, form, dt, n):
    ins = [fi.fill(dt, 91, r, n) for r in range(P)]
    topo = "1" if form == "ring" else str(P)
    ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt])
    # small slices, so the sliced path (a slice boundary inside a block) is exercised too
    got = whole_fold.fold([_torch_in(x, dt) for x in ins], n, form, block_elems=97)
    want = _torch_in(ref[0], dt)
    assert whole_fold.first_mismatch(got, want) is None


def test_first_mismatch_reports_the_first_differing_element():
    import torch
    a = torch.arange(10, dtype=torch.float32)
    b = a.clone()
    b[3] = -0.0 if a[3] == 0 else -a[3]
    b[7] = 100
    assert whole_fold.first_mismatch(a, a.clone()) is None
    assert whole_fold.first_mismatch(a, b) == (2, 3)
    z = torch.zeros(4)
    assert whole_fold.first_mismatch(z, -z) == (4, 0)   # bits, not values: -0.0 differs from 0.0
