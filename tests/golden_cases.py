"""Access to the committed reference fixtures in tests/golden/ (see oracle/gen_golden.py)."""
import hashlib
import json
import os

import numpy as np

import ftar_inputs as fi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_manifest = None
_npz = {}


def manifest():
    global _manifest
    if _manifest is None:
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            _manifest = json.load(f)
    return _manifest


def _arrays(name):
    if name not in _npz:
        _npz[name] = np.load(os.path.join(GOLDEN, name))  # allow_pickle=False (default)
    return _npz[name]


def allreduce_cases(max_n=None, filt=None):
    out = [c for c in manifest()["cases"] if c.get("kind") != "reduce"]
    if max_n is not None:
        out = [c for c in out if c["n"] <= max_n]
    if filt:
        out = [c for c in out if filt(c)]
    return out


def reduce_cases():
    return [c for c in manifest()["cases"] if c.get("kind") == "reduce"]


def case_inputs(c):
    """Per-rank inputs of an allreduce case, exactly as ref_golden generated them."""
    if c.get("init") == "linear":
        # benchmark.cpp:125-129: data[i] = i * 0.1f (i converts exactly to float below 2^24)
        x = np.arange(c["n"], dtype=np.float32) * np.float32(0.1)
        return [x.copy() for _ in range(c["P"])]
    return [fi.fill(c["dtype"], c["seed"], r, c["n"]) for r in range(c["P"])]


def reduce_inputs(c):
    return [fi.fill(c["dtype"], c["seed"], j, c["n"]) for j in range(c["k"])]


def expected(c, rank=0):
    """Full expected output for stored cases, else None."""
    arr = _arrays("allreduce.npz")
    if not c.get("stored"):
        return None
    key = c["id"] if c["all_equal"] else f'{c["id"]}__r{rank}'
    return arr[key]


def expected_reduce(c):
    return _arrays("reduce.npz")[c["id"]]


def sha256(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def check_output(c, rank, out):
    """Assert `out` equals the reference output of case c at `rank`, bit for bit."""
    assert out.dtype == fi.np_dtype(c["dtype"]), (out.dtype, c["dtype"])
    exp = expected(c, rank)
    if exp is not None:
        np.testing.assert_array_equal(out.view(np.uint8), exp.view(np.uint8), err_msg=c["id"])
    assert sha256(out) == c["sha256"][rank], f'{c["id"]} rank {rank}: sha256 differs from the reference'
