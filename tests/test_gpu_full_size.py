"""The AllReduce at BASELINE's full bucket sizes, through size-independent properties.

C3 = 2 ranks x 2^26 fp32 ring, C4 = 8 ranks x 2^28 fp32 ring (both data-movement forms), C5 = 8 ranks x
2^29 bf16 width-8 tree: every rank of an in-process group (ftar_comm_init_local) on cuda:0, the product's
plan executor, pipelining and reduce kernels, out of place.  The oracle would need 8-16 GiB of host arrays
here, so instead:
  * a sample of elements (every block boundary, the ends, 4096 seeded random indices) is bit-exact against
    the reference's fold of those elements (tests/sample_fold.py, itself pinned to the oracle by
    tests/test_sample_fold.py);
  * every rank ends with the same bits over the whole bucket;
  * the call on the negated inputs gives exactly the negated result everywhere (round-to-nearest-even is
    sign-symmetric), which also proves the call read all of this call's data.
"""
import numpy as np
import pytest

import sample_fold

pytestmark = pytest.mark.gpu


def _sample_index(n, P, seed=99):
    split = -(-n // P)
    pts = {0, n - 1}
    for b in range(1, P):
        for d in (-1, 0, 1):
            pts.add(b * split + d)
    rng = np.random.default_rng(seed)
    pts.update(int(v) for v in rng.integers(0, n, 4096))
    return np.array(sorted(p for p in pts if 0 <= p < n), dtype=np.int64)


@pytest.mark.parametrize("P,n,dt,topo,form", [
    (2, 1 << 26, "f32", "1", "direct"),     # C3
    (8, 1 << 28, "f32", "1", "direct"),     # C4, one-round forms (the default)
    (8, 1 << 28, "f32", "1", "stages"),     # C4, the reference's 2(P-1) ring steps
    (8, 1 << 29, "bf16", "8", "direct"),    # C5, the cost model's width-8 tree
])
def test_allreduce_full_size_properties(P, n, dt, topo, form):
    import torch

    import ftar
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
    dev = torch.device("cuda", 0)
    g = ftar.Comm.init_local(P)
    xs, ys = [], []
    try:
        g.set_allgather(form)
        g.set_reduce_scatter(form)
        for r in range(P):
            gen = torch.Generator(device=dev)
            gen.manual_seed(4242 + r)
            xs.append((torch.rand(n, generator=gen, device=dev) * 2 - 1).to(tdt))
            ys.append(torch.empty(n, dtype=tdt, device=dev))
        idx = _sample_index(n, P)
        it = torch.from_numpy(idx).to(dev)
        samp = np.stack([x[it].float().cpu().numpy() for x in xs])

        g.allreduce(xs, ys, n, dt, "sum", topo_=topo)
        torch.cuda.synchronize()
        exp = sample_fold.fold(samp, idx, n, "ring" if topo == "1" else "tree", bf16=dt == "bf16")
        got = ys[0][it].float().cpu().numpy()
        bad = np.nonzero(got.view(np.uint32) != exp.view(np.uint32))[0]
        assert bad.size == 0, f"{bad.size} sampled elements differ, first at {idx[bad[0]]}: {got[bad[0]]} vs {exp[bad[0]]}"
        for r in range(1, P):
            assert torch.equal(ys[r], ys[0]), f"rank {r} differs from rank 0"

        y0 = ys[0].clone()
        for x in xs:
            x.neg_()
        g.allreduce(xs, ys, n, dt, "sum", topo_=topo)
        torch.cuda.synchronize()
        assert torch.equal(ys[0], y0.neg_()), "negated inputs did not give the negated result"
        for r in range(1, P):
            assert torch.equal(ys[r], ys[0]), f"rank {r} differs from rank 0 (negated call)"
    finally:
        g.destroy()
        xs.clear()
        ys.clear()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("topo", ["1", "2"])
def test_allreduce_past_int32_elements(topo):
    """2^31 + 77 u8 elements per rank (the reference's `int count` stops below 2^31, mpi_mod.hpp:1724): block
    offsets and piece indices past 2^31 in the engine.  u8 sums wrap and are associative, so the sample check is
    exact in any order; then linearity over the whole bucket: inputs + 1 on every rank give result + P (mod 256)."""
    import torch

    import ftar
    P, n = 2, (1 << 31) + 77
    dev = torch.device("cuda", 0)
    g = ftar.Comm.init_local(P)
    xs, ys = [], []
    try:
        for r in range(P):
            gen = torch.Generator(device=dev)
            gen.manual_seed(777 + r)
            xs.append(torch.randint(0, 256, (n,), generator=gen, dtype=torch.uint8, device=dev))
            ys.append(torch.empty(n, dtype=torch.uint8, device=dev))
        idx = _sample_index(n, P)
        it = torch.from_numpy(idx).to(dev)
        g.allreduce(xs, ys, n, "u8", "sum", topo_=topo)
        torch.cuda.synchronize()
        exp = sum(x[it].to(torch.int64) for x in xs) % 256
        assert torch.equal(ys[0][it].to(torch.int64), exp)
        assert torch.equal(ys[1], ys[0])
        y0 = ys[0].clone()
        for x in xs:
            x.add_(1)
        g.allreduce(xs, ys, n, "u8", "sum", topo_=topo)
        torch.cuda.synchronize()
        assert torch.equal(ys[0], y0.add_(P)), "linearity: inputs + 1 must give result + P (mod 256)"
        assert torch.equal(ys[1], ys[0])
    finally:
        g.destroy()
        xs.clear()
        ys.clear()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("P,n,dt,topo", [
    (8, 1 << 28, "f32", "1"),     # C4 through the MPI_Allreduce_FT path (host buffers, in place)
    (8, 1 << 29, "bf16", "8"),    # C5, same
])
def test_host_allreduce_full_size_properties(P, n, dt, topo):
    """ftar_allreduce_host (H2D / exchange / D2H pipelined per piece) on pinned host buckets of BASELINE's full
    size, in place like benchmark.cpp:161: the sampled per-element fold, rank agreement, negation symmetry."""
    import torch

    import ftar
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
    dev = torch.device("cuda", 0)
    g = ftar.Comm.init_local(P)
    hs, orig = [], []
    try:
        for r in range(P):
            gen = torch.Generator(device=dev)
            gen.manual_seed(5151 + r)
            hs.append((torch.rand(n, generator=gen, device=dev) * 2 - 1).to(tdt).cpu().pin_memory())
        orig.extend(h.clone() for h in hs)
        idx = _sample_index(n, P)
        it = torch.from_numpy(idx)
        samp = np.stack([h[it].float().numpy() for h in hs])
        g.allreduce(None, hs, n, dt, "sum", topo_=topo, host=True)
        torch.cuda.synchronize()
        exp = sample_fold.fold(samp, idx, n, "ring" if topo == "1" else "tree", bf16=dt == "bf16")
        got = hs[0][it].float().numpy()
        bad = np.nonzero(got.view(np.uint32) != exp.view(np.uint32))[0]
        assert bad.size == 0, f"{bad.size} sampled elements differ, first at {idx[bad[0]]}"
        for r in range(1, P):
            assert torch.equal(hs[r], hs[0]), f"rank {r} differs from rank 0"
        y0 = hs[0].clone()
        for h, x in zip(hs, orig):
            torch.neg(x, out=h)
        g.allreduce(None, hs, n, dt, "sum", topo_=topo, host=True)
        torch.cuda.synchronize()
        assert torch.equal(hs[0], y0.neg_()), "negated inputs did not give the negated result"
        for r in range(1, P):
            assert torch.equal(hs[r], hs[0]), f"rank {r} differs from rank 0 (negated call)"
    finally:
        g.destroy()
        hs.clear()
        orig.clear()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("topo", ["1", "2"])
def test_allreduce_at_mpi_max_count_fp32(topo):
    """The largest bucket MPI_Allreduce_FT's `int count` can name (mpi_mod.hpp:1724): 2^31 - 1 fp32 elements
    (8 GiB) per rank, 2 ranks, ring and tree(2), out of place: block 1 starts 4 GiB into the bucket, so byte
    offsets pass 2^32.  With two ranks every element is one fp32 add, the same in either order, so the whole
    output is checked bit for bit against torch's x0 + x1."""
    import torch

    import ftar
    P, n = 2, (1 << 31) - 1
    dev = torch.device("cuda", 0)
    g = ftar.Comm.init_local(P)
    xs, ys = [], []
    try:
        for r in range(P):
            gen = torch.Generator(device=dev)
            gen.manual_seed(31 + r)
            xs.append(torch.rand(n, generator=gen, device=dev) * 2 - 1)
            ys.append(torch.empty(n, device=dev))
        g.allreduce(xs, ys, n, "f32", "sum", topo_=topo)
        torch.cuda.synchronize()
        exp = xs[0] + xs[1]
        for r in range(P):
            assert torch.equal(ys[r].view(torch.int32), exp.view(torch.int32)), r
    finally:
        g.destroy()
        xs.clear()
        ys.clear()
        torch.cuda.empty_cache()
