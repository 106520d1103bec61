"""numpy mirror of include/ftar_inputs.h (splitmix64 synthetic inputs).

Bit-identical to the C generator; tests/test_oracle_golden.py checks it
against the reference driver's own inputs (through the golden outputs).
"""
import numpy as np

DTYPES = {  # ftar dtype id -> (name, numpy dtype)
    0: ("u8", np.uint8),
    1: ("i8", np.int8),
    2: ("u16", np.uint16),
    3: ("i16", np.int16),
    4: ("i32", np.int32),
    5: ("i64", np.int64),
    6: ("f32", np.float32),
    7: ("f64", np.float64),
    8: ("bool", np.uint8),
    9: ("bf16", np.uint16),  # raw bf16 bits
}
BY_NAME = {v[0]: k for k, v in DTYPES.items()}

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_STREAM = np.uint64(0xD1B54A32D192ED03)


def _mix(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def raw(seed, stream, n):
    """The n uint64 draws of stream `stream` of `seed`."""
    with np.errstate(over="ignore"):
        st = _mix(np.uint64(seed) ^ (_STREAM * np.uint64(stream + 1)))
        idx = np.arange(1, n + 1, dtype=np.uint64)
        return _mix(st + idx * _GAMMA)


def f32_to_bf16_bits(x):
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & np.uint64(0x7FFFFFFF)) > np.uint64(0x7F800000)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) & np.uint64(0xFFFF)
    r = np.where(nan, (u >> np.uint64(16)) | np.uint64(0x40), r)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def fill(dtype, seed, stream, n):
    """numpy array of n elements of ftar dtype `dtype` (id or name)."""
    dt = BY_NAME[dtype] if isinstance(dtype, str) else dtype
    z = raw(seed, stream, n)
    if dt in (0, 1):
        return (z & np.uint64(0xFF)).astype(np.uint8).view(DTYPES[dt][1])
    if dt in (2, 3):
        return (z & np.uint64(0xFFFF)).astype(np.uint16).view(DTYPES[dt][1])
    if dt == 4:
        return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
    if dt == 5:
        return z.view(np.int64)
    if dt in (6, 9):
        f = ((z >> np.uint64(40)).astype(np.int64) - (1 << 23)).astype(np.float32) * np.float32(1.0 / 8388608.0)
        return f if dt == 6 else f32_to_bf16_bits(f)
    if dt == 7:
        return ((z >> np.uint64(11)).astype(np.int64) - (1 << 52)).astype(np.float64) * (1.0 / 4503599627370496.0)
    if dt == 8:
        return (z >> np.uint64(63)).astype(np.uint8)
    raise ValueError(dt)


def np_dtype(dtype):
    dt = BY_NAME[dtype] if isinstance(dtype, str) else dtype
    return DTYPES[dt][1]
