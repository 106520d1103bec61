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


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("topo", ["ring", "tree"])
def test_explain_localises_and_classifies_each_kind_of_wrong_output(dt, topo):
    """whole_fold.explain on synthetic wrong outputs of every kind a broken hand-off produces: the bad
    (block, piece) cells, the runs, and what the values equal (poison, zero, this rank's input, another
    rank's input, a partial fold, data shifted by a piece)."""
    import torch
    P, n, piece, rank = 4, 4 * 1000, 256, 1
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
    gen = torch.Generator().manual_seed(5)
    xs = [(torch.rand(n, generator=gen) * 2 - 1).to(tdt) for _ in range(P)]
    exp = whole_fold.fold(xs, n, topo)
    split = n // P
    assert whole_fold.explain(exp.clone(), exp, xs, rank, topo, piece) is None
    iv = {torch.float32: torch.int32, torch.bfloat16: torch.int16}[tdt]
    poison = 0xFFFFFFFF if dt == "f32" else 0xFFFF

    def corrupt(b, k, a, z, fill):
        got = exp.clone()
        lo = b * split + k * piece
        got[lo + a:lo + z] = fill(lo + a, lo + z)
        return got, lo

    pf = whole_fold.partial_folds
    kinds = {
        "poison": lambda lo, hi: torch.full((hi - lo,), -1, dtype=iv).view(tdt),
        "zero": lambda lo, hi: torch.zeros(hi - lo, dtype=tdt),
        "own_input": lambda lo, hi: xs[rank][lo:hi],
        "input_of_3": lambda lo, hi: xs[3][lo:hi],
        "partial_1": lambda lo, hi: pf(xs, lo, hi, lo // split, topo, dt == "bf16")[0].to(tdt),
        f"shifted_{piece:+d}": lambda lo, hi: exp[lo + piece:hi + piece],
    }
    for name, fill in kinds.items():
        got, lo = corrupt(2, 1, 10, 200, fill)
        e = whole_fold.explain(got, exp, xs, rank, topo, piece, poison=poison)
        assert e is not None, name
        assert e["ncells"] == 1 and e["cells"][0][:2] == (2, 1), (name, e)
        fc = e["first_cell"]
        assert fc["block"] == 2 and fc["piece"] == 1
        # some elements of the fill may equal the right value, or an earlier class's, by chance (bf16's 8-bit
        # mantissa): nearly all the bad ones land in the named class
        assert max(fc["classes"], key=fc["classes"].get) == name, (name, fc["classes"])
        assert fc["classes"][name] >= 0.95 * e["count"], (name, fc["classes"])
        assert sum(fc["classes"].values()) == e["count"]
        assert fc["runs"][0][0] >= lo + 10 and sum(r[1] for r in fc["runs"]) <= 190 or fc["nruns"] > len(fc["runs"])
        assert "differ" in whole_fold.describe(e)


def test_explain_counts_every_bad_cell_and_run():
    import torch
    P, n, piece = 2, 2 * 1024, 128
    xs = [torch.arange(n, dtype=torch.float32) + 0.5 * r for r in range(P)]
    exp = whole_fold.fold(xs, n, "ring")
    got = exp.clone()
    got[5:9] = 0            # block 0 piece 0: two runs
    got[20:30] = 0
    got[1024 + 300] = 0     # block 1 piece 2
    got[1024 + 1000:1024 + 1024] = 7.25  # block 1 piece 7, "other"
    e = whole_fold.explain(got, exp, xs, 0, "ring", piece)
    assert e["count"] == 4 + 10 + 1 + 24
    assert [c[:3] for c in e["cells"]] == [(0, 0, 14), (1, 2, 1), (1, 7, 24)]
    assert e["first"] == 5 and e["ncells"] == 3
    assert e["first_cell"]["runs"] == [[5, 4], [20, 10]] and e["first_cell"]["nruns"] == 2
    assert e["first_cell"]["classes"] == {"zero": 14}
