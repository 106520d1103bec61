"""ctypes front-end of the oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    src = os.path.join(ORACLE_DIR, "ftar_oracle.cpp")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)
    lib = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    lib.oracle_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.c_int, vp, ctypes.c_size_t, ctypes.c_int]
    lib.oracle_allreduce.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    lib.oracle_schedule_json.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    lib.oracle_schedule_json.restype = ctypes.c_long
    _lib = lib
    return lib


def parse_topo(topo):
    return [int(x) for x in str(topo).split(",") if x.strip()]


def reduce(dtype, op, srcs, out=None, copy_k1=False):
    lib = load()
    srcs = [np.ascontiguousarray(s) for s in srcs]
    n = srcs[0].size
    if out is None:
        out = np.empty_like(srcs[0])
    arr = (ctypes.c_void_p * max(1, len(srcs)))(*[s.ctypes.data for s in srcs])
    rc = lib.oracle_reduce(dtype, op, arr, len(srcs), out.ctypes.data, n, int(copy_k1))
    if rc:
        raise RuntimeError(f"oracle_reduce rc={rc}")
    return out


def allreduce(inputs, topo, lonely=0, dtype=6, op=0, outofplace=False):
    """Simulated reference AllReduce over len(inputs) ranks; returns per-rank outputs."""
    lib = load()
    P = len(inputs)
    st = parse_topo(topo)
    sarr = (ctypes.c_int * max(1, len(st)))(*st)
    n = inputs[0].size
    ins = [np.ascontiguousarray(x).copy() for x in inputs]
    if outofplace:
        # recvbuf starts as 0xA5 bytes, as in oracle/ref_golden.cpp
        outs = [np.frombuffer(b"\xa5" * x.nbytes, dtype=x.dtype).copy() for x in ins]
        send = (ctypes.c_void_p * P)(*[x.ctypes.data for x in ins])
    else:
        outs = ins
        send = None
    recv = (ctypes.c_void_p * P)(*[x.ctypes.data for x in outs])
    rc = lib.oracle_allreduce(P, sarr, len(st), lonely, dtype, op, n, send, recv)
    if rc:
        raise RuntimeError(f"oracle_allreduce rc={rc}")
    return outs


def schedule(P, topo, lonely, rank, n):
    lib = load()
    st = parse_topo(topo)
    sarr = (ctypes.c_int * len(st))(*st)
    need = lib.oracle_schedule_json(P, sarr, len(st), lonely, rank, n, None, 0)
    if need < 0:
        raise RuntimeError(f"oracle_schedule_json rc={need}")
    buf = ctypes.create_string_buffer(need + 1)
    lib.oracle_schedule_json(P, sarr, len(st), lonely, rank, n, buf, need + 1)
    return json.loads(buf.value.decode())
