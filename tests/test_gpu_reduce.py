"""Parity of the HIP k-way reduce kernel (ftar_reduce) with the reference.

Bit-exact for every dtype (integers wrap, floats add in their own precision,
left to right) against (a) the reference's own reduce_sum/reduce_band outputs
(tests/golden/reduce.npz) and (b) the pinned oracle on random sizes, k,
misalignments and in-place use, up to the C2 benchmark size (2^26 fp32).
"""
import numpy as np
import pytest

import ftar_inputs as fi
import golden_cases as gc
import oracle_lib
from gpu_util import filled_dev, from_dev, to_dev

pytestmark = pytest.mark.gpu


def run_reduce(ins, dtype, op, offsets=None, out_offset=0, inplace=False):
    import ftar
    n = ins[0].size
    offsets = offsets or [0] * len(ins)
    devs = [to_dev(x, offset_elems=o) for x, o in zip(ins, offsets)]
    esz = ins[0].dtype.itemsize
    if inplace:
        dst_t, dst = devs[0]
        out_offset = offsets[0]
    else:
        dst_t, dst = filled_dev((n + out_offset) * esz)
        dst += out_offset * esz
    ftar.reduce([p for _, p in devs], dst, n, dtype, op)
    return from_dev(dst_t, ins[0].dtype, n, out_offset)


@pytest.mark.parametrize("case", gc.reduce_cases(), ids=lambda c: c["id"])
def test_reduce_matches_reference_golden(case):
    ins = gc.reduce_inputs(case)
    got = run_reduce(ins, case["dtype"], case["op"])
    exp = gc.expected_reduce(case)
    if case["k"] == 1:
        # ftar_reduce follows vector_add/reduce_sum.h (k == 1 copies); mpi_mod.hpp's
        # k <= 1 no-op is honoured inside the AllReduce engine instead.
        exp = ins[0]
    np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))


DTS = ["f32", "bf16", "f64", "u8", "i8", "u16", "i16", "i32", "i64", "bool"]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("k", [2, 3, 5, 8, 9, 17, 33])
@pytest.mark.parametrize("n", [1, 5, 255, 4099, 100_003])
def test_reduce_sum_vs_oracle(dt, k, n):
    ins = [fi.fill(dt, 1000 + k, j, n) for j in range(k)]
    got = run_reduce(ins, dt, "sum")
    exp = oracle_lib.reduce(fi.BY_NAME[dt], 0, ins)
    np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))


@pytest.mark.parametrize("dt", ["u8", "i16", "i32", "i64"])
@pytest.mark.parametrize("k", [2, 4, 11])
def test_reduce_band_vs_oracle(dt, k):
    n = 70_001
    ins = [fi.fill(dt, 77, j, n) for j in range(k)]
    # make AND results non-trivial: OR a shared mask into every source
    mask = fi.fill(dt, 78, 0, n)
    ins = [np.bitwise_or(x, mask) for x in ins]
    got = run_reduce(ins, dt, "band")
    exp = oracle_lib.reduce(fi.BY_NAME[dt], 1, ins)
    np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))


@pytest.mark.parametrize("dt", ["f32", "bf16", "u8", "f64"])
@pytest.mark.parametrize("offs,out_off", [([1, 1], 1), ([3, 3, 3], 3), ([0, 1], 0), ([2, 0, 1], 3), ([0, 0], 1)])
def test_reduce_unaligned(dt, offs, out_off):
    """Block offsets in the AllReduce are arbitrary: heads/tails and non-co-aligned sources."""
    n = 33_333
    ins = [fi.fill(dt, 5, j, n) for j in range(len(offs))]
    got = run_reduce(ins, dt, "sum", offsets=offs, out_offset=out_off)
    exp = oracle_lib.reduce(fi.BY_NAME[dt], 0, ins)
    np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))


@pytest.mark.parametrize("dt", ["f32", "bf16", "i32"])
def test_reduce_in_place(dt):
    """dst == src0, the ring's in-place fold (mpi_mod.hpp:1699)."""
    n = 1 << 18
    ins = [fi.fill(dt, 9, j, n) for j in range(3)]
    got = run_reduce(ins, dt, "sum", inplace=True)
    exp = oracle_lib.reduce(fi.BY_NAME[dt], 0, ins)
    np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))


def test_reduce_zero_count_is_noop():
    import ftar
    t, p = filled_dev(64)
    ftar.reduce([p, p], p, 0, "f32")
    assert (t.cpu().numpy() == 0xA5).all()


@pytest.mark.parametrize("k", [2, 8])
def test_reduce_full_c2_size(k):
    """The benchmark workload itself: k sources x 2^26 fp32 (256 MiB each), bit-exact."""
    n = 1 << 26
    ins = [fi.fill("f32", 0x5EED, j, n) for j in range(k)]
    got = run_reduce(ins, "f32", "sum")
    exp = oracle_lib.reduce(6, 0, ins)
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_reduce_bf16_matches_fp32_reference_within_one_rounding():
    """bf16 (extension): fp32 accumulate, one RNE per reduce -> |err| <= 0.5 ulp(bf16) of the fp32 sum."""
    n, k = 1 << 16, 8
    ins = [fi.fill("bf16", 3, j, n) for j in range(k)]
    got = fi.bf16_bits_to_f32(run_reduce(ins, "bf16", "sum"))
    f32 = np.zeros(n, np.float32)
    for x in ins:
        f32 = (f32 + fi.bf16_bits_to_f32(x)).astype(np.float32)
    ulp = np.abs(f32) * 2.0 ** -8 + 1e-30
    assert np.all(np.abs(got - f32) <= ulp)


@pytest.mark.parametrize("k", [2, 3, 8, 16])
def test_reduce_bf16_is_torch_fp32_fold_rounded_once(k):
    """bf16 has no reference (mpi_mod.hpp handles no 16-bit float), so its semantics are pinned against an
    independent implementation instead of our own oracle: PyTorch, folding the sources left to right in fp32
    (torch's own adds) and converting once with torch's round-to-nearest-even float -> bfloat16.  The GPU
    kernel must give the same bits on every element, NaN and infinity inputs included."""
    import torch
    n = 50_001
    ins = [fi.fill("bf16", 11, j, n) for j in range(k)]
    ins[0][::97] = 0x7FC1       # NaN
    ins[1][5::89] = 0x7F80      # +inf
    ins[-1][7::83] = 0xFF80     # -inf
    ins[1][11::79] = 0x0001     # bf16 denormal
    got = run_reduce(ins, "bf16", "sum").view(np.uint16)
    t = [torch.from_numpy(x.view(np.int16).copy()).view(torch.bfloat16) for x in ins]
    acc = t[0].float()
    for x in t[1:]:
        acc = acc + x.float()
    ref = acc.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    nan_g = (got & 0x7FFF) > 0x7F80
    nan_r = (ref & 0x7FFF) > 0x7F80
    assert np.array_equal(nan_g, nan_r)                     # NaN exactly where torch has NaN
    assert np.array_equal(got[~nan_r], ref[~nan_r])


def test_reduce_beyond_int32_index():
    """2^31 + 77 elements (the reference kernel indexes with `int`, vector_add/reduce_sum_gpu.h:8):
    u8 sums wrap, checked on a head, a window across the 2^31 boundary and the tail."""
    import ftar
    import torch
    n = (1 << 31) + 77
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    b = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    out = torch.empty_like(a)
    ftar.reduce([a.data_ptr(), b.data_ptr()], out.data_ptr(), n, "u8", "sum")
    torch.cuda.synchronize()
    for lo, hi in ((0, 1 << 16), ((1 << 31) - (1 << 15), (1 << 31) + (1 << 15)), (n - (1 << 16), n)):
        exp = oracle_lib.reduce(0, 0, [a[lo:hi].cpu().numpy(), b[lo:hi].cpu().numpy()])
        np.testing.assert_array_equal(out[lo:hi].cpu().numpy(), exp)
    # full-size property: sum of all bytes is preserved mod 2^8 per element -> compare checksums
    assert int(((a.to(torch.int64) + b.to(torch.int64)) % 256).sum()) == int(out.to(torch.int64).sum())


def nested_oracle(dt, op, ins, shape):
    """Nested fold, every node one oracle reduce (what the staged tree computes)."""
    vals = ins
    for w in shape:
        vals = [oracle_lib.reduce(dt, op, vals[i:i + w]) if w > 1 else vals[i] for i in range(0, len(vals), w)]
    return vals[0]


@pytest.mark.parametrize("shape", [[2, 2], [2, 3], [3, 2], [2, 4], [4, 2], [2, 2, 2], [3, 3], [2, 3, 2], [4, 4],
                                   [2, 2, 2, 2], [3, 3, 3], [1, 4, 2], [8, 1]])
@pytest.mark.parametrize("dt", ["f32", "bf16", "f64", "i32", "u8"])
@pytest.mark.parametrize("n,off", [(100_003, 0), (4099, 1)])
def test_reduce_nested_vs_oracle(shape, dt, n, off):
    """ftar_reduce_nested (the one-round tree reduce-scatter's fold): bit-exact vs per-node oracle reduces,
    compile-time k (4, 6, 8, 16) and runtime k (9, 12, 27), co-aligned and element-wise (off=1, dst aligned)."""
    import ftar
    k = int(np.prod(shape))
    ins = [fi.fill(dt, 2000 + k, j, n) for j in range(k)]
    offs = [off if j % 2 else 0 for j in range(k)]
    devs = [to_dev(x, offset_elems=o) for x, o in zip(ins, offs)]
    dst_t, dst = filled_dev(n * ins[0].itemsize)
    ftar.reduce([p for _, p in devs], dst, n, dt, "sum", shape=shape)
    got = from_dev(dst_t, ins[0].dtype, n)
    exp = nested_oracle(fi.BY_NAME[dt], 0, ins, shape)
    np.testing.assert_array_equal(got.view(np.uint8), exp.view(np.uint8))


def test_reduce_nested_rejects_bad_shapes():
    import ftar
    t, p = filled_dev(64)
    for shape in ([2, 3], [0, 4], [2, 2, 2, 2, 1], [-1, -4]):
        with pytest.raises(ftar.FtarError):
            ftar.reduce([p] * 4, p, 4, "f32", "sum", shape=shape)
    ftar.reduce([p] * 4, p, 0, "f32", "sum", shape=[2, 2])   # zero count: no-op


@pytest.mark.parametrize("shape", [None, [2, 4]])
def test_reduce_captures_into_a_hip_graph(shape):
    """ftar_reduce / ftar_reduce_nested are stream-ordered launches with no host synchronisation, so a bucket's
    reduce chain can be captured once into a HIP graph and replayed (the launch-bound small-bucket regime):
    replays give the eager call's bits, and a replay after the sources change reads the new data."""
    import ftar
    import torch
    k, n = 8, (1 << 20) + 3
    srcs = [torch.from_numpy(fi.fill("f32", 61, j, n)).cuda() for j in range(k)]
    ptrs = [s.data_ptr() for s in srcs]
    eager = torch.empty(n, dtype=torch.float32, device="cuda")
    ftar.reduce(ptrs, eager.data_ptr(), n, "f32", "sum", stream=torch.cuda.current_stream(), shape=shape)
    out = torch.empty_like(eager)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for _ in range(3):   # a chain of launches in one graph
                ftar.reduce(ptrs, out.data_ptr(), n, "f32", "sum", stream=side, shape=shape)
    torch.cuda.current_stream().wait_stream(side)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), eager.view(torch.int32))
    srcs[0].neg_()
    srcs[1].neg_()
    g.replay()
    ftar.reduce(ptrs, eager.data_ptr(), n, "f32", "sum", stream=torch.cuda.current_stream(), shape=shape)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), eager.view(torch.int32))


@pytest.mark.parametrize("seed", range(3))
def test_random_soak_reduce(seed):
    """Seeded random ftar_reduce calls: k = 1..64, every dtype and op, sizes from 0 to 300k elements (block
    remainders of every kind), element offsets that are co-aligned with the destination (vector path with
    heads/tails) or not (element-wise path), and in place.  Bit-exact vs the oracle.  FTAR_SOAK scales the
    case count (default 60 per seed)."""
    import os
    import random
    rng = random.Random(3000 + seed)
    per = max(1, int(os.environ.get("FTAR_SOAK", "100")) * 3 // 5)
    for i in range(per):
        dt = rng.choice(["f32", "f32", "bf16", "f64", "u8", "i8", "u16", "i16", "i32", "i64", "bool"])
        op = "band" if dt in ("u8", "i8", "u16", "i16", "i32", "i64") and rng.random() < 0.3 else "sum"
        k = rng.choice([1, 2, 2, 3, 4, 5, 6, 7, 8, 8, 9, 12, 16, 17, 24, 33, 64])
        n = rng.choice([0, 1, 7, 15, 16, 17, 63, 64, 65, rng.randint(1, 5000), rng.randint(5000, 300_000)])
        vec = 16 // np.dtype(fi.np_dtype(dt)).itemsize
        mode = rng.choice(["aligned", "co-aligned", "mixed", "inplace"])
        if mode == "aligned":
            offs, out_off = [0] * k, 0
        elif mode == "co-aligned":   # same address mod 16 everywhere: vector path + head/tail
            o = rng.randint(0, max(0, vec - 1))
            offs, out_off = [o] * k, o
        elif mode == "mixed":        # at least one source off: element-wise path
            offs, out_off = [rng.randint(0, 7) for _ in range(k)], rng.randint(0, 7)
        else:
            offs, out_off = None, 0
        ins = [fi.fill(dt, 4000 + i, j, n) for j in range(k)]
        if op == "band":
            mask = fi.fill(dt, 4001 + i, 0, n)
            ins = [np.bitwise_or(x, mask) for x in ins]
        got = run_reduce(ins, dt, op, offsets=offs, out_offset=out_off, inplace=(mode == "inplace"))
        exp = oracle_lib.reduce(fi.BY_NAME[dt], 0 if op == "sum" else 1, ins, copy_k1=True)
        assert got.view(np.uint8).tobytes() == exp.view(np.uint8).tobytes(), (seed, i, dt, op, k, n, mode, offs, out_off)


@pytest.mark.parametrize("seed", range(2))
def test_random_soak_reduce_nested(seed):
    """Seeded random nested folds (ftar_reduce_nested): random mixed-radix shapes of 2-4 levels and k up to 64
    (compile-time shapes, runtime codes, runtime-k loops), float dtypes, sizes with every kind of remainder,
    co-aligned heads/tails or element-wise offsets, in place.  Bit-exact vs per-node oracle reduces.
    FTAR_SOAK scales the case count (default 40 per seed)."""
    import os
    import random
    import ftar
    rng = random.Random(5000 + seed)
    per = max(1, int(os.environ.get("FTAR_SOAK", "100")) * 2 // 5)
    for i in range(per):
        while True:
            shape = [rng.choice([1, 2, 2, 3, 4]) for _ in range(rng.randint(2, 4))]
            k = int(np.prod(shape))
            if 2 <= k <= 64:
                break
        dt = rng.choice(["f32", "bf16", "f64"])
        n = rng.choice([1, 15, 16, 17, 255, rng.randint(1, 9000), rng.randint(9000, 200_000)])
        vec = 16 // np.dtype(fi.np_dtype(dt)).itemsize
        mode = rng.choice(["aligned", "co-aligned", "mixed", "inplace"])
        o = rng.randint(0, vec - 1)
        offs = {"aligned": [0] * k, "co-aligned": [o] * k, "inplace": [o] * k,
                "mixed": [rng.randint(0, 7) for _ in range(k)]}[mode]
        ins = [fi.fill(dt, 6000 + i, j, n) for j in range(k)]
        devs = [to_dev(x, offset_elems=off) for x, off in zip(ins, offs)]
        if mode == "inplace":
            dst_t, dst = devs[0]
            out_off = offs[0]
        else:
            out_off = o if mode == "co-aligned" else 0
            dst_t, dst = filled_dev((n + out_off) * ins[0].itemsize)
            dst += out_off * ins[0].itemsize
        ftar.reduce([p for _, p in devs], dst, n, dt, "sum", shape=shape)
        got = from_dev(dst_t, ins[0].dtype, n, out_off)
        exp = nested_oracle(fi.BY_NAME[dt], 0, ins, shape)
        assert got.view(np.uint8).tobytes() == exp.view(np.uint8).tobytes(), (seed, i, shape, dt, n, mode, offs[:4])


def test_bf16_hardware_conversion_is_the_rne_for_every_float():
    """gfx950's v_cvt_pk_bf16_f32 against the bit-exact integer RNE (the oracle's f32_to_bf16_rne) on all
    2^32 float bit patterns, NaN payloads, infinities and denormals included: the kernels may use either."""
    import ctypes
    import ftar
    lib = ftar.bench_lib()
    lib.ftar_debug_bf16_cvt_check.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_uint)]
    bad, first = ctypes.c_ulonglong(0), ctypes.c_uint(0)
    assert lib.ftar_debug_bf16_cvt_check(ctypes.byref(bad), ctypes.byref(first)) == 0
    assert bad.value == 0, f"{bad.value} patterns differ, first 0x{first.value:08x}"


def assert_bits_equal_nan_as_nan(got, exp, dt):
    """Bit-exact wherever the expected value is a number (infinities and signed zeros included); NaN exactly
    where it is NaN.  Which NaN a sum returns when NaNs meet (its sign and payload, and the sign of the
    default NaN of inf - inf) is left open by IEEE 754 and by the LLVM IR the kernels compile from (fadd is
    commutative there, so operand order is the compiler's), and the reference's own NaN bits depend on its
    x86 compiler's operand order in the same way: that is outside the bit-exact contract."""
    if dt == "bf16":
        g, e = fi.bf16_bits_to_f32(got.view(np.uint16)), fi.bf16_bits_to_f32(exp.view(np.uint16))
        gb, eb = got.view(np.uint16), exp.view(np.uint16)
    else:
        g, e = got.view(np.float32), exp.view(np.float32)
        gb, eb = got.view(np.uint32), exp.view(np.uint32)
    nan = np.isnan(e)
    np.testing.assert_array_equal(np.isnan(g), nan)
    np.testing.assert_array_equal(gb[~nan], eb[~nan])
    assert nan.any()  # the inputs do exercise NaN


def _bf16_specials(seed, j, n):
    """bf16 inputs with NaNs (both signs, several payloads), infinities, bf16 denormals, values whose sum
    overflows and ties that round to even, mixed into random values"""
    x = fi.fill("bf16", seed, j, n).copy()
    specials = np.array([0x7FC0, 0xFFC0, 0x7F81, 0xFF81, 0x7FBF, 0x7F80, 0xFF80, 0x0001, 0x8001, 0x007F,
                         0x7F7F, 0xFF7F, 0x0000, 0x8000, 0x3F80, 0x3B80], dtype=np.uint16)
    rng = np.random.default_rng(seed * 31 + j)
    idx = rng.choice(n, size=n // 8, replace=False)
    x.view(np.uint16)[idx] = specials[rng.integers(0, specials.size, idx.size)]
    return x


def _f32_specials(seed, j, n):
    x = fi.fill("f32", seed, j, n).copy()
    specials = np.array([0x7FC00000, 0xFFC00000, 0x7F800001, 0xFF812345, 0x7FBFFFFF, 0x7F800000, 0xFF800000,
                         0x00000001, 0x80000001, 0x7F7FFFFF, 0xFF7FFFFF, 0x00000000, 0x80000000], dtype=np.uint32)
    rng = np.random.default_rng(seed * 37 + j)
    idx = rng.choice(n, size=n // 8, replace=False)
    x.view(np.uint32)[idx] = specials[rng.integers(0, specials.size, idx.size)]
    return x


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("k", [2, 3, 8, 16])
def test_reduce_special_values_vs_oracle(k, dt):
    n = 100_003
    ins = [(_bf16_specials if dt == "bf16" else _f32_specials)(7, j, n) for j in range(k)]
    got = run_reduce(ins, dt, "sum")
    exp = oracle_lib.reduce(fi.BY_NAME[dt], 0, ins)
    assert_bits_equal_nan_as_nan(got, exp, dt)


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("form", ["direct", "stages"])
@pytest.mark.parametrize("topo", ["1", "2,2", "4"])
def test_allreduce_special_values_vs_oracle(topo, form, dt):
    """NaNs (both signs, several payloads), infinities, denormals and overflow through the one-round and the
    staged forms, 4 in-process ranks: bit-exact except which NaN comes out where NaNs meet
    (assert_bits_equal_nan_as_nan)"""
    import ftar
    import torch
    P, n = 4, 50_001
    xs = [(_bf16_specials if dt == "bf16" else _f32_specials)(11, r, n) for r in range(P)]
    view = np.int16 if dt == "bf16" else np.int32
    group = ftar.Comm.init_local(P)
    try:
        group.set_reduce_scatter(form)
        group.set_allgather(form)
        bufs = [torch.from_numpy(x.view(view).copy()).cuda() for x in xs]
        group.allreduce(None, bufs, n, dt, "sum", topo_=topo)
        torch.cuda.synchronize()
        ref = oracle_lib.allreduce(xs, topo, dtype=fi.BY_NAME[dt])
        for r in range(P):
            assert_bits_equal_nan_as_nan(bufs[r].cpu().numpy().view(view), ref[r].view(view), dt)
    finally:
        group.destroy()


def test_reduce_reference_gpu_test_size_k1_to_16():
    """The reference's own GPU test (vector_add.cu:139-150, :182-187): k = 1..16 sources of n = 150e6 fp32
    uniform [0, 1) values (rand()/RAND_MAX there), GPU reduce against the CPU reduce_sum within 1e-5.  Here:
    ftar_reduce against torch's fp32 adds folded left to right (reduce_sum's order, mpi_mod.hpp:856-863;
    reduce_sum.h:36-222), every element bit for bit, at the reference's size; a 1-element offset copy of the
    sources (the unaligned head/tail path) at k = 3 and 16."""
    import torch

    import ftar
    n, kmax = 150_000_000, 16
    g = torch.Generator(device="cuda")
    g.manual_seed(150)
    srcs = [torch.rand(n + 1, device="cuda", generator=g) for _ in range(kmax)]
    dst = torch.empty(n + 1, device="cuda")
    acc = torch.empty(n, device="cuda")
    for k in range(1, kmax + 1):
        for off in ((0, 1) if k in (3, 16) else (0,)):
            acc.copy_(srcs[0][off:off + n])
            for j in range(1, k):
                acc.add_(srcs[j][off:off + n])
            dst.fill_(float("nan"))
            ftar.reduce([s[off:] for s in srcs[:k]], dst[off:], n, "f32", "sum")
            torch.cuda.synchronize()
            assert torch.equal(dst[off:off + n].view(torch.int32), acc.view(torch.int32)), (k, off)
