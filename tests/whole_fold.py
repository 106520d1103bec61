"""The reference AllReduce's fold order over a WHOLE bucket, in torch -- TEST INFRASTRUCTURE.

tests/sample_fold.py restates the per-element fold in numpy for a sample of indices; this module evaluates
the same fold for every element of a bucket with torch tensor arithmetic, on whatever device the inputs
live on (cuda:0 in the full-size GPU tests, so C4/C5's 8 x 1 GiB buckets check in seconds).  The result
depends only on the P inputs at an element and on its block b = i // split (split = ceil(n/P),
mpi_mod.hpp:776-809):

  ring (mpi_mod.hpp:1673-1719, block b folds hop by hop and ends on rank b-1):
      x_{b+P-1} + (... + (x_{b+1} + x_b)), indices mod P; bf16 rounds after every hop (one reduce per hop)
  one-stage tree(P) (mpi_mod.hpp:1510-1671; own block first, then the peers in ascending rank, :1316-1358):
      ((x_b + x_0) + x_1) + ... over p != b; bf16 accumulates in fp32 and rounds once

fp32 additions in torch are IEEE round-to-nearest-even on CPU and GPU alike (an add has nothing to
contract), so these are the reference's bits; tests/test_whole_fold.py pins this module to the oracle
(oracle/ftar_oracle.cpp, itself pinned to the unmodified reference) bit for bit.
"""


def fold_block(xs, lo, hi, b, topo, bf16=False):
    """The reference's value of elements [lo, hi) of block b, as fp32 (bf16-valued for bf16 inputs)."""
    import torch
    P = len(xs)
    acc = xs[b][lo:hi].float()
    if topo == "ring":
        for j in range(1, P):
            acc = xs[(b + j) % P][lo:hi].float() + acc
            if bf16:
                acc = acc.to(torch.bfloat16).float()
        return acc
    if topo != "tree":
        raise ValueError(topo)
    for p in range(P):
        if p != b:
            acc = acc + xs[p][lo:hi].float()
    return acc.to(torch.bfloat16).float() if bf16 else acc


def fold(xs, n, topo, out=None, block_elems=1 << 26):
    """xs: P tensors of n elements (fp32 or bf16), one per rank.  Returns (or writes into `out`) the
    reference's AllReduce result, in the inputs' dtype, computed block by block and in slices of at most
    `block_elems` elements so the fp32 temporaries stay small."""
    import torch
    P = len(xs)
    dt = xs[0].dtype
    bf16 = dt == torch.bfloat16
    if out is None:
        out = torch.empty(n, dtype=dt, device=xs[0].device)
    split = -(-n // P)
    for b in range(P):
        for lo in range(b * split, min(n, (b + 1) * split), block_elems):
            hi = min(lo + block_elems, (b + 1) * split, n)
            out[lo:hi] = fold_block(xs, lo, hi, b, topo, bf16).to(dt)
    return out


def first_mismatch(got, exp):
    """None if the two tensors are bit-identical, else (count, first index) of the differing elements."""
    import torch
    iv = {torch.float32: torch.int32, torch.bfloat16: torch.int16}[got.dtype]
    ne = got.view(iv) != exp.view(iv)
    cnt = int(ne.sum().item())
    if cnt == 0:
        return None
    return cnt, int(torch.nonzero(ne)[0].item())
