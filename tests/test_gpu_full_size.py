"""The AllReduce at BASELINE's full bucket sizes, every element checked.

C3 = 2 ranks x 2^26 fp32 ring, C4 = 8 ranks x 2^28 fp32 (the ring in both data-movement forms, and the
width-8 tree), C5 = 8 ranks x 2^29 bf16 width-8 tree: every rank of an in-process group (ftar_comm_init_local)
on cuda:0, the product's plan executor, pipelining and reduce kernels, out of place.  Random inputs differ per
rank, so the association order shows in the bits.  Every rank's WHOLE output is compared bit for bit with the
reference's fold of the P inputs, evaluated over the whole bucket on the GPU by tests/whole_fold.py (pinned to
the oracle by tests/test_whole_fold.py).  Some cases use pipeline pieces that do not divide a block
(FTAR_CHUNK_BYTES / the host piece size), so piece boundaries fall mid-block and every block ends on a short
piece; in host mode the (stage, piece) steps also run skewed (engine.cpp step_order).  Every data-movement form
runs at C4 (direct, stages, collective, peer-read, peer-write, auto), the peer forms at C5 too.
"""
import pytest

import whole_fold

pytestmark = pytest.mark.gpu

MiB = 1 << 20
# pieces that divide no block: 24 MiB + 4 KiB (C4: 128 MiB blocks -> 5 whole pieces + an 8 MiB tail; the
# element count is a multiple of 64, as the engine rounds it) and 20 MiB + 256 B for the host pipeline
ODD_CHUNK = 24 * MiB + 4096
ODD_HOST_CHUNK = 20 * MiB + 256


def _inputs(P, n, tdt, seed, dev):
    import torch
    xs = []
    for r in range(P):
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed + r)
        xs.append((torch.rand(n, generator=gen, device=dev) * 2 - 1).to(tdt))
    return xs


def _check_whole(ys, exp, what):
    for r, y in enumerate(ys):
        bad = whole_fold.first_mismatch(y, exp)
        assert bad is None, f"{what}: rank {r}: {bad[0]} elements differ from the reference's fold, first at {bad[1]}"


@pytest.mark.parametrize("P,n,dt,topo,form,chunk", [
    (2, 1 << 26, "f32", "1", "direct", 0),            # C3
    (8, 1 << 28, "f32", "1", "direct", 0),            # C4, one-round forms (the default)
    (8, 1 << 28, "f32", "1", "stages", 0),            # C4, the reference's 2(P-1) ring steps
    (8, 1 << 28, "f32", "8", "direct", 0),            # C4's bucket on the width-8 tree
    (8, 1 << 28, "f32", "1", "direct", ODD_CHUNK),    # C4, piece boundaries mid-block, short last pieces
    (8, 1 << 28, "f32", "1", "stages", ODD_CHUNK),
    (8, 1 << 29, "bf16", "8", "direct", 0),           # C5, the cost model's width-8 tree
    (8, 1 << 29, "bf16", "8", "direct", ODD_CHUNK),
    # the other data-movement forms at full size: IPC-mapped peer reads / writes (whole blocks per kernel),
    # the collective all-gather, and "auto" (whatever the execution model picks with its default constants)
    (8, 1 << 28, "f32", "1", "peer-read", 0),
    (8, 1 << 28, "f32", "1", "peer-write", 0),
    (8, 1 << 28, "f32", "8", "collective", 0),
    (8, 1 << 28, "f32", "1", "auto", 0),
    (8, 1 << 29, "bf16", "8", "peer-read", 0),
    (8, 1 << 29, "bf16", "8", "peer-write", 0),
])
def test_allreduce_full_size_whole_bucket(P, n, dt, topo, form, chunk):
    import torch

    import ftar
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
    dev = torch.device("cuda", 0)
    g = ftar.Comm.init_local(P)
    xs, ys = [], []
    try:
        if form in ("direct", "stages"):
            g.set_allgather(form)
            g.set_reduce_scatter(form)
        else:
            g.set_form(form)
        if chunk:
            g.set_chunk_bytes(chunk)
        xs = _inputs(P, n, tdt, 4242, dev)
        ys = [torch.empty(n, dtype=tdt, device=dev) for _ in range(P)]
        g.allreduce(xs, ys, n, dt, "sum", topo_=topo)
        torch.cuda.synchronize()
        ran = g.comms[0].last_exec()
        if form != "auto":
            assert ran["form"] == form, ran
        exp = whole_fold.fold(xs, n, "ring" if topo == "1" else "tree")
        _check_whole(ys, exp, f"P={P} n={n} {dt} topo={topo} {form} chunk={chunk} ran={ran}")
    finally:
        g.destroy()
        xs.clear()
        ys.clear()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("topo", ["1", "2"])
def test_allreduce_past_int32_elements(topo):
    """2^31 + 77 u8 elements per rank (the reference's `int count` stops below 2^31, mpi_mod.hpp:1724): block
    offsets and piece indices past 2^31 in the engine.  u8 sums wrap and are associative, so torch's x0 + x1
    (uint8, wrapping) is the reference's result in any order: every element of both ranks is compared; then
    linearity over the whole bucket: inputs + 1 on every rank give result + P (mod 256)."""
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
        g.allreduce(xs, ys, n, "u8", "sum", topo_=topo)
        torch.cuda.synchronize()
        exp = xs[0] + xs[1]
        assert torch.equal(ys[0], exp)
        assert torch.equal(ys[1], exp)
        del exp
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


@pytest.mark.parametrize("P,n,dt,topo,piece", [
    (8, 1 << 28, "f32", "1", 0),                 # C4 through the MPI_Allreduce_FT path (host buffers, in place)
    (8, 1 << 29, "bf16", "8", 0),                # C5, same
    (8, 1 << 28, "f32", "1", ODD_HOST_CHUNK),    # C4 with host pieces that divide no block (skewed steps)
])
def test_host_allreduce_full_size_whole_bucket(P, n, dt, topo, piece):
    """ftar_allreduce_host (H2D / exchange / D2H pipelined per piece, stage s+1 one piece behind stage s) on
    pinned host buckets of BASELINE's full size, in place like benchmark.cpp:161: every rank's whole bucket
    against the reference's fold of the P inputs."""
    import torch

    import ftar
    tdt = {"f32": torch.float32, "bf16": torch.bfloat16}[dt]
    dev = torch.device("cuda", 0)
    g = ftar.Comm.init_local(P)
    hs = []
    try:
        if piece:
            g.set_host_chunk_bytes(piece)
        xs = _inputs(P, n, tdt, 5151, dev)
        hs = [x.cpu().pin_memory() for x in xs]
        exp = whole_fold.fold(xs, n, "ring" if topo == "1" else "tree")
        del xs
        g.allreduce(None, hs, n, dt, "sum", topo_=topo, host=True)
        torch.cuda.synchronize()
        for r, h in enumerate(hs):
            bad = whole_fold.first_mismatch(h.to(dev), exp)
            assert bad is None, f"rank {r}: {bad[0]} elements differ from the reference's fold, first at {bad[1]}"
    finally:
        g.destroy()
        hs.clear()
        torch.cuda.empty_cache()


def test_host_comm_peer_forms_full_size_whole_bucket():
    """C4 and C5 on eight PROCESSES of a host-bootstrapped communicator (IPC-mapped exchange buffers across the
    process boundary, the machinery the peer forms use between the GPUs of a node): peer read and write on
    device buffers, and the host-buffer paths; every rank's whole bucket equals the reference's fold.  Each
    case starts on NaN-poisoned exchange buffers, every rank's view of every mapping is compared page by page
    after it, and every rank's failures are reported, localised and classified (tests/host_comm_cases.py)."""
    import host_comm_cases as hc
    cases = hc.CASES + hc.WIDE   # read and write forms at both sizes (keep both in the default suite)
    res = hc.run(cases)
    bad = hc.failures(res)
    assert not bad, "\n".join(bad)
    for r in range(8):
        assert [x["name"] for x in res[r]["results"]] == [c[0] for c in cases], r


def test_host_comm_gather_records():
    """The diagnostic gather of the host path (FTAR_DEBUG_HOST_GATHER_LOG=1) gives the same result
    and leaves one record per workgroup in host memory, and every workgroup id ran exactly once."""
    import host_comm_cases as hc
    res = hc.run([("c4_host_read", 1 << 24, "f32", "1", "read", True)], world=2,
                 env={"FTAR_DEBUG_HOST_GATHER_LOG": "1"})
    bad = hc.failures(res, world=2)
    assert not bad, "\n".join(bad)
    for r in range(2):
        g = res[r]["results"][0]["gather_log"]
        print(r, {k: v for k, v in g.items() if k != "bad"})
        # 64 MiB, 2 ranks: 32 MiB blocks in 4 MiB pieces, each piece one 4 MiB segment of 512 workgroups
        assert g["pieces"] == 8 and g["wgs"] == 8 * 512, g
        assert g["host_missing"] == 0 and g["dev_missing"] == 0 and g["bad"] == [], g
        assert g["runs"] == g["wgs"] and g["ids_run_twice"] == 0, g
        assert sum(g["queues"].values()) == g["wgs"], g


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
