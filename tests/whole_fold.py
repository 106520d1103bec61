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


def partial_folds(xs, lo, hi, b, topo, bf16=False):
    """The fold of elements [lo, hi) of block b after each of its P - 1 additions, in order (the last is the
    final value): what a reader sees if it reads a fold that has not finished, or one owner's partial sum."""
    import torch
    P = len(xs)
    acc = xs[b][lo:hi].float()
    order = [(b + j) % P for j in range(1, P)] if topo == "ring" else [p for p in range(P) if p != b]
    out = []
    for i, p in enumerate(order):
        acc = xs[p][lo:hi].float() + acc if topo == "ring" else acc + xs[p][lo:hi].float()
        if bf16 and (topo == "ring" or i == len(order) - 1):
            acc = acc.to(torch.bfloat16).float()
        out.append(acc)
    return out


def explain(got, exp, xs, rank, topo, piece, split=None, poison=None, max_cells=8, max_runs=4):
    """Where the elements of `got` that differ from `exp` lie and what they hold -- the two-sided, localising
    check the reference's one-sided --check (benchmark.cpp:195-210) is not.  None if bit-identical, else:
      count, first           as first_mismatch
      cells                  [(block, piece, bad count, first bad index)] of the first max_cells cells that
                             hold bad elements (piece k of block b = elements b*split + [k*piece, (k+1)*piece),
                             the host pipeline's unit), ncells their number
      first_cell.runs        contiguous bad runs [start, length] in the first bad cell (max_runs of them),
                             nruns their number
      first_cell.classes     what that cell's bad elements equal, bit for bit, checked in this order: "poison"
                             (the fill the test wrote between cases), "zero" (+-0), "own_input" (this rank's
                             input at the same index), "input_of_<q>" (rank q's), "partial_<j>" (the block's
                             fold after j of its P - 1 additions), "shifted_<d>" (the right value of element
                             i + d, d = +-piece or +-split: data in the wrong place), else "other"
    xs: the P inputs (same device as got); rank: whose output `got` is; poison: the fill's bit pattern as an
    int (0xFFFFFFFF fp32 / 0xFFFF bf16 for a 0xFF byte fill) or None."""
    import torch
    iv = {torch.float32: torch.int32, torch.bfloat16: torch.int16}[got.dtype]
    gb, eb = got.view(iv), exp.view(iv)
    ne = gb != eb
    count = int(ne.sum().item())
    if count == 0:
        return None
    n, P = got.numel(), len(xs)
    split = split or -(-n // P)
    cells = []
    ncells = 0
    for b in range(P):
        lo, hi = b * split, min(n, (b + 1) * split)
        if lo >= hi:
            continue
        blk = ne[lo:hi]
        m = -(-(hi - lo) // piece)
        pad = torch.zeros(m * piece, dtype=torch.int32, device=got.device)
        pad[:hi - lo] = blk.to(torch.int32)
        per = pad.view(m, piece).sum(1).cpu().tolist()
        for k, c in enumerate(per):
            if c:
                ncells += 1
                if len(cells) < max_cells:
                    seg = blk[k * piece:(k + 1) * piece]
                    cells.append((b, k, int(c), lo + k * piece + int(torch.nonzero(seg)[0].item())))
    b0, k0 = cells[0][0], cells[0][1]
    clo = b0 * split + k0 * piece
    chi = min(n, b0 * split + min(split, (k0 + 1) * piece))
    cm = ne[clo:chi]
    # runs of the cell's mask
    d = torch.diff(torch.cat([torch.zeros(1, dtype=torch.int8, device=got.device), cm.to(torch.int8),
                              torch.zeros(1, dtype=torch.int8, device=got.device)]))
    starts = torch.nonzero(d == 1).flatten()
    ends = torch.nonzero(d == -1).flatten()
    runs = [[clo + int(s), int(e - s)] for s, e in zip(starts[:max_runs].tolist(), ends[:max_runs].tolist())]
    # classify the cell's bad elements
    idx = torch.nonzero(cm).flatten()
    g = gb[clo:chi][idx]
    left = torch.ones(idx.numel(), dtype=torch.bool, device=got.device)
    classes = {}

    def take(name, hit):
        nonlocal left
        h = hit & left
        c = int(h.sum().item())
        if c:
            classes[name] = classes.get(name, 0) + c
        left = left & ~h

    if poison is not None:
        pv = torch.tensor(poison, dtype=torch.int64).to(iv)  # wraps to the signed pattern
        take("poison", g == pv.to(got.device))
    take("zero", (got[clo:chi][idx] == 0))
    bf16 = got.dtype == torch.bfloat16
    take("own_input", g == xs[rank].view(iv)[clo:chi][idx])
    for q in range(P):
        if q != rank:
            take(f"input_of_{q}", g == xs[q].view(iv)[clo:chi][idx])
    for j, acc in enumerate(partial_folds(xs, clo, chi, b0, topo, bf16)[:-1], start=1):
        take(f"partial_{j}", g == acc.to(got.dtype).view(iv)[idx])
    for dd in (piece, -piece, split, -split):
        src = idx + clo + dd
        ok = (src >= 0) & (src < n)
        hit = torch.zeros_like(left)
        hit[ok] = g[ok] == eb[src[ok]]
        take(f"shifted_{dd:+d}", hit)
    rest = int(left.sum().item())
    if rest:
        classes["other"] = rest
    return {"count": count, "first": cells[0][3], "cells": cells, "ncells": ncells,
            "first_cell": {"block": b0, "piece": k0, "runs": runs, "nruns": int(starts.numel()),
                           "classes": classes}}


def describe(e):
    """One line for an assertion message from explain()'s result."""
    if e is None:
        return "bit-identical"
    fc = e["first_cell"]
    return (f"{e['count']} elements differ, first at {e['first']}, in {e['ncells']} (block, piece) cells "
            f"{[tuple(c) for c in e['cells']]}; first cell block {fc['block']} piece {fc['piece']}: "
            f"{fc['nruns']} runs {fc['runs']}, values {fc['classes']}")
