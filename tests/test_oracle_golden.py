"""Pin the oracle (oracle/ftar_oracle.cpp) to the reference's own outputs.

Every committed fixture in tests/golden/ was produced by the unmodified
reference (mpi_mod.hpp under MPICH, oracle/gen_golden.py). The oracle must
reproduce each one bit for bit before anything is checked against it.
"""
import json
import os

import numpy as np
import pytest

import ftar_inputs as fi
import golden_cases as gc
import oracle_lib


def test_input_generator_pinned():
    with open(os.path.join(gc.GOLDEN, "inputs.json")) as f:
        pins = json.load(f)
    assert [int(x) for x in fi.raw(1, 0, 4)] == pins["raw_seed1_stream0"]
    for p in pins["fills"]:
        got = fi.fill(p["dtype"], p["seed"], p["stream"], 8).tolist()
        assert got == p["values"], p


@pytest.mark.parametrize("case", gc.allreduce_cases(), ids=lambda c: c["id"])
def test_oracle_allreduce_matches_reference(oracle, case):
    ins = gc.case_inputs(case)
    outs = None
    for _ in range(case["repeat"]):
        outs = oracle_lib.allreduce(ins, case["topo"], case["lonely"], case["dtype"], case["op"],
                                    outofplace=case["outofplace"])
        ins = outs
    for r in range(case["P"]):
        gc.check_output(case, r, outs[r])


@pytest.mark.parametrize("case", gc.reduce_cases(), ids=lambda c: c["id"])
def test_oracle_reduce_matches_reference(oracle, case):
    ins = gc.reduce_inputs(case)
    n = case["n"]
    out = np.frombuffer(b"\xa5" * (n * np.dtype(fi.np_dtype(case["dtype"])).itemsize),
                        dtype=fi.np_dtype(case["dtype"])).copy()
    oracle_lib.reduce(case["dtype"], case["op"], ins, out=out, copy_k1=False)
    np.testing.assert_array_equal(out.view(np.uint8), gc.expected_reduce(case).view(np.uint8))


def _schedules():
    with open(os.path.join(gc.GOLDEN, "schedules.jsonl")) as f:
        return [json.loads(l) for l in f]


@pytest.mark.parametrize("sched", _schedules(), ids=lambda d: f'P{d["P"]}_t{d["topo"]}_l{d["lonely"]}_n{d["n"]}_r{d["rank"]}')
def test_oracle_schedule_matches_reference(oracle, sched):
    got = oracle_lib.schedule(sched["P"], sched["topo"], sched["lonely"], sched["rank"], sched["n"])
    for key in ("send", "send_lonely", "recv", "recv_lonely"):
        assert got[key] == sched[key], key


def test_invalid_topology_rejected(oracle):
    ins = [fi.fill(6, 1, r, 8) for r in range(4)]
    with pytest.raises(RuntimeError):
        oracle_lib.allreduce(ins, "3", 0)        # 3 != 4 (mpi_mod.hpp:1471)
    with pytest.raises(RuntimeError):
        oracle_lib.allreduce(ins, "3", 1)        # lonely needs >= 2 stages


def test_sum_order_closed_forms(oracle):
    """ring block b = x_{b+P-1} + (... + (x_{b+1} + x_b)); tree(P) = ((x_b + x_0) + x_1) ..."""
    P, n = 4, 16
    ins = [fi.fill(6, 99, r, n) for r in range(P)]
    split = (n + P - 1) // P
    ring = oracle_lib.allreduce(ins, "1")[0]
    tree = oracle_lib.allreduce(ins, str(P))[0]
    for b in range(P):
        sl = slice(b * split, (b + 1) * split)
        acc = ins[b][sl].copy()
        for j in range(1, P):
            acc = (ins[(b + j) % P][sl] + acc).astype(np.float32)
        np.testing.assert_array_equal(ring[sl], acc)
        acc = ins[b][sl].copy()
        for p in range(P):
            if p != b:
                acc = (acc + ins[p][sl]).astype(np.float32)
        np.testing.assert_array_equal(tree[sl], acc)
