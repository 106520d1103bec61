"""bf16 has no reference (mpi_mod.hpp:1365-1375 handles no 16-bit float), so ftar defines it: fp32 accumulate,
one round-to-nearest-even per reduce call -- per hop on the ring, per tree node, once for a flat fold.  These
CPU tests pin the oracle's restatement of that definition against an independent implementation, PyTorch's
own fp32 adds and float -> bfloat16 conversion, written out as the fold each schedule performs:

  * reduce (k sources):        round(x0 + x1 + ... + x_{k-1})                      (one rounding)
  * ring, block b:              acc = x_b; acc = round(acc + x_{b+j}) for j = 1..P-1 (mpi_mod.hpp:1689-1703)
  * tree(P), block b:           round(x_b + x_{p1} + ...), peers ascending          (mpi_mod.hpp:1316-1358)
  * tree(w0, w1), block b:      round over the w1 stage of rounded w0-group folds

The GPU kernels are pinned to the same definition by tests/test_gpu_reduce.py (flat fold against torch) and
by the oracle comparisons of tests/test_gpu_allreduce.py.  NaN: NaN exactly where torch has NaN (which NaN
is outside the contract)."""
import numpy as np
import pytest

import ftar_inputs as fi
import oracle_lib

torch = pytest.importorskip("torch")


def _t(x):
    return torch.from_numpy(np.ascontiguousarray(x).view(np.int16).copy()).view(torch.bfloat16)


def _bits(t):
    return t.view(torch.int16).numpy().view(np.uint16)


def _same(got, ref):
    ng, nr = (got & 0x7FFF) > 0x7F80, (ref & 0x7FFF) > 0x7F80
    return np.array_equal(ng, nr) and np.array_equal(got[~nr], ref[~nr])


def _inputs(P, n, seed):
    ins = [fi.fill("bf16", seed, r, n).copy() for r in range(P)]
    ins[0][::97] = 0x7FC1
    ins[-1][3::89] = 0x7F80
    ins[P // 2][5::83] = 0xFF80
    return ins


@pytest.mark.parametrize("k", [2, 3, 5, 8, 16, 20])
def test_oracle_bf16_reduce_is_torch(k):
    ins = _inputs(k, 30_011, 5)
    acc = _t(ins[0]).float()
    for x in ins[1:]:
        acc = acc + _t(x).float()
    assert _same(oracle_lib.reduce(9, 0, ins).view(np.uint16), _bits(acc.to(torch.bfloat16)))


@pytest.mark.parametrize("P", [2, 3, 5, 8])
def test_oracle_bf16_ring_rounds_every_hop_like_torch(P):
    n = 4 * P + 3   # ragged blocks
    ins = _inputs(P, n, 6)
    split = -(-n // P)
    outs = oracle_lib.allreduce(ins, "1", dtype=9)
    ref = np.empty(n, np.uint16)
    for b in range(P):
        lo, hi = b * split, min(n, (b + 1) * split)
        if lo >= hi:
            continue
        acc = _t(ins[b][lo:hi])
        for j in range(1, P):
            acc = (acc.float() + _t(ins[(b + j) % P][lo:hi]).float()).to(torch.bfloat16)
        ref[lo:hi] = _bits(acc)
    for r in range(P):
        assert _same(outs[r].view(np.uint16), ref), r


@pytest.mark.parametrize("topo", ["4", "8", "2,2", "2,4", "4,2", "2,2,2"])
def test_oracle_bf16_trees_round_per_node_like_torch(topo):
    widths = [int(w) for w in topo.split(",")]
    P = int(np.prod(widths))
    n = 3 * P + 1
    ins = _inputs(P, n, 7)
    split = -(-n // P)
    outs = oracle_lib.allreduce(ins, topo, dtype=9)
    ref = np.empty(n, np.uint16)
    for b in range(P):
        lo, hi = b * split, min(n, (b + 1) * split)
        if lo >= hi:
            continue
        # V_0(q) = x_q; at stage s rank q's partial of block b folds its own V_s first, then its stage
        # group's partials in ascending rank order (group = left + j*g, mpi_mod.hpp:274, :369), rounded
        vals = {q: _t(ins[q][lo:hi]) for q in range(P)}
        g = 1
        for w in widths:
            new = {}
            for q in range(P):
                left = q // (g * w) * g * w + q % g
                acc = vals[q].float()
                for j in range(w):
                    p = left + j * g
                    if p != q:
                        acc = acc + vals[p].float()
                new[q] = acc.to(torch.bfloat16)
            vals = new
            g *= w
        ref[lo:hi] = _bits(vals[b])
    for r in range(P):
        assert _same(outs[r].view(np.uint16), ref), (topo, r)
