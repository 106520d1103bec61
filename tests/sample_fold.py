"""Closed-form fold of single elements of the reference AllReduce -- TEST INFRASTRUCTURE.

At BASELINE's full sizes (C4: P=8 ring, 2^28 fp32 per rank; C5: P=8 width-8 tree, 2^29 bf16 per rank)
the oracle would need 8-16 GiB of host arrays, so the full-size GPU tests check a sample of elements
instead.  For an element i the reference's result depends only on the P inputs at i and on the block
b = i // split (split = ceil(n/P), mpi_mod.hpp:776-809):

  ring (mpi_mod.hpp:1673-1719): x_{b+P-1} + (... + (x_{b+1} + x_b)), indices mod P; bf16 rounds each hop
  one-stage tree(P) (mpi_mod.hpp:1510-1671, :274): x_b, then + x_p for p = 0..P-1, p != b, ascending;
      bf16 accumulates in fp32 and rounds once (the ftar extension)

tests/test_sample_fold.py pins both forms against the oracle (oracle/ftar_oracle.cpp) bit for bit.
"""
import numpy as np


def rne_bf16(f):
    """fp32 -> nearest-even bf16, returned as fp32 (finite inputs)."""
    u = np.ascontiguousarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32)


def fold(xs, idx, n, topo, bf16=False):
    """xs: (P, m) fp32 values of every rank at the sampled indices idx (bf16 inputs widened exactly).
    Returns the reference's fp32 (or bf16-valued fp32) result at idx."""
    xs = np.asarray(xs, dtype=np.float32)
    P, m = xs.shape
    split = -(-n // P)
    b = (np.asarray(idx, dtype=np.int64) // split).astype(np.int64)
    ar = np.arange(m)
    acc = xs[b, ar].copy()
    if topo == "ring":
        for j in range(1, P):
            acc = (xs[(b + j) % P, ar] + acc).astype(np.float32)
            if bf16:
                acc = rne_bf16(acc)
        return acc
    if topo != "tree":
        raise ValueError(topo)
    for p in range(P):
        acc = np.where(b != p, (acc + xs[p]).astype(np.float32), acc)
    return rne_bf16(acc) if bf16 else acc
