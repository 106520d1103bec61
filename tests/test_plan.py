"""The product's plan compiler (libftar schedule.cpp), checked on the CPU.

1. Its FMA-level schedule equals the reference's, dumped from the reference
   itself (tests/golden/schedules.jsonl).
2. Its executable per-rank plans, executed by a numpy model of the engine
   (transfers matched per peer pair in posting order, reduces in the plan's
   source order, arithmetic by the pinned oracle), reproduce the reference's
   golden outputs bit for bit.  The GPU tests then run the same plans through
   the HIP engine.
"""
import collections
import json
import os

import numpy as np
import pytest

import ftar_inputs as fi
import golden_cases as gc
import oracle_lib
import plan_fold


def _schedules():
    with open(os.path.join(gc.GOLDEN, "schedules.jsonl")) as f:
        return [json.loads(l) for l in f]


@pytest.mark.parametrize("sched", _schedules(), ids=lambda d: f'P{d["P"]}_t{d["topo"]}_l{d["lonely"]}_n{d["n"]}_r{d["rank"]}')
def test_product_schedule_matches_reference(sched):
    import ftar
    got = ftar.schedule_json(ftar.topo(sched["topo"], sched["lonely"]), sched["P"], sched["rank"], sched["n"])
    for key in ("send", "send_lonely", "recv", "recv_lonely"):
        assert got[key] == sched[key], key


def simulate(plans, inputs, dtype, op, outofplace):
    """numpy model of engine.cpp executing per-rank plans (stage-synchronous)."""
    P = len(plans)
    src = [x.copy() for x in inputs]
    dst = [np.frombuffer(b"\xa5" * x.nbytes, dtype=x.dtype).copy() for x in inputs] if outofplace else src
    scratch = [np.zeros(max(1, 2 * p["scratch_half"]), dtype=inputs[0].dtype) for p in plans]
    bufs = [{"src": src[r], "dst": dst[r], "scratch": scratch[r]} for r in range(P)]
    nst = len(plans[0]["stages"])
    assert all(len(p["stages"]) == nst for p in plans)
    for s in range(nst):
        wire = collections.defaultdict(collections.deque)
        for r in range(P):
            for peer, buf, off, ln in plans[r]["stages"][s]["sends"]:
                wire[(r, peer)].append(bufs[r][buf][off:off + ln].copy())
        for r in range(P):
            for peer, buf, off, ln in plans[r]["stages"][s]["recvs"]:
                msg = wire[(peer, r)].popleft()
                assert msg.size == ln
                bufs[r][buf][off:off + ln] = msg
        assert all(not q for q in wire.values()), "unmatched send"
        for r in range(P):
            for it in plans[r]["stages"][s]["reduces"]:
                off, ln = it["off"], it["len"]
                srcs = [np.ascontiguousarray(bufs[r][b][o:o + ln]) for b, o in it["srcs"]]
                out = plan_fold.fold(it, srcs, dtype, op)
                bufs[r]["dst"][off:off + ln] = out
    if plans[0]["allgather"] == "collective":  # one all-gather: rank p contributes dst[p*split : (p+1)*split]
        split = plans[0]["split"]
        segs = [dst[p][p * split:(p + 1) * split].copy() for p in range(P)]
        for r in range(P):
            for p in range(P):
                dst[r][p * split:(p + 1) * split] = segs[p]
    return dst


CASES = gc.allreduce_cases(max_n=70000)


@pytest.mark.parametrize("form", ["stages", "direct"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: c["id"])
def test_product_plans_reproduce_reference(case, form):
    import ftar
    P = case["P"]
    t = ftar.topo(case["topo"], case["lonely"])
    plans = [ftar.plan_json(t, P, r, case["n"], allgather=form, reduce_scatter=form) for r in range(P)]
    ins = gc.case_inputs(case)
    outs = None
    for _ in range(case["repeat"]):
        outs = simulate(plans, ins, case["dtype"], case["op"], case["outofplace"])
        ins = outs
    for r in range(P):
        gc.check_output(case, r, outs[r])


def test_scratch_is_compact():
    """The plan's scratch is one received range per slot (the reference keeps 2*P*split)."""
    import ftar
    n = 1 << 20
    ring = ftar.plan_json("1", 8, 0, n, reduce_scatter="stages")
    assert ring["scratch_half"] == n // 8
    assert ftar.plan_json("1", 8, 0, n)["scratch_half"] == 7 * (n // 8)   # direct: P-1 slots, one round
    tree = ftar.plan_json("8", 8, 3, n)
    assert tree["scratch_half"] == 7 * (n // 8)
    assert tree["max_k"] == 8


@pytest.mark.parametrize("P,topo", [(2, "2"), (4, "4"), (4, "2,2"), (6, "2,3"), (8, "8"), (8, "2,4"), (8, "4,2"),
                                    (8, "2,2,2"), (9, "3,3")])
def test_collective_allgather_plans_match_oracle(P, topo):
    """Every non-lonely FlexTree leaves rank r holding block r, so the all-gather phase may be one
    collective (ftar_comm_set_allgather(FTAR_AG_COLLECTIVE)): same result, bit for bit."""
    import ftar
    n = P * 1001
    ins = [fi.fill("f32", 404, r, n) for r in range(P)]
    ref = oracle_lib.allreduce(ins, topo)
    for rs in ("stages", "direct"):
        plans = [ftar.plan_json(topo, P, r, n, allgather="collective", reduce_scatter=rs) for r in range(P)]
        assert all(p["allgather"] == "collective" for p in plans)
        # reduce-scatter stages only: one per tree stage, or one round
        assert len(plans[0]["stages"]) == (len(topo.split(",")) if rs == "stages" else 1)
        outs = simulate(plans, ins, 6, 0, False)
        for r in range(P):
            np.testing.assert_array_equal(outs[r].view(np.uint32), ref[r].view(np.uint32))
    # not applicable: ragged counts, lonely ranks and the ring keep their stages
    # not applicable: ragged counts and the ring (its final blocks sit one rank off) fall back to direct
    assert ftar.plan_json(topo, P, 0, n + 1, allgather="collective")["allgather"] == "direct"
    assert ftar.plan_json("1", P, 0, n, allgather="collective")["allgather"] == "direct"


def test_random_plans_match_oracle():
    """200 seeded random cases: topologies incl. lonely, ragged sizes, every dtype, SUM/BAND, in/out of place."""
    import ftar
    import random_cases
    for c in random_cases.cases(seed=2024, count=200):
        P = c["P"]
        t = ftar.topo(c["topo"], c["lonely"])
        form = ("stages", "direct")[c["n"] % 2]
        plans = [ftar.plan_json(t, P, r, c["n"], allgather=form, reduce_scatter=form) for r in range(P)]
        outs = simulate(plans, c["ins"], fi.BY_NAME[c["dtype"]], 0 if c["op"] == "sum" else 1, c["oop"])
        for r in range(P):
            assert outs[r].tobytes() == c["ref"][r].tobytes(), (c["P"], c["topo"], c["lonely"], c["n"], c["dtype"], r)


def test_product_rejects_exactly_the_topologies_the_reference_cannot_run():
    """Lonely layouts where the reference asserts (followers > 1) or would block: the product refuses them
    (FTAR_ERR_INVALID_TOPO) instead of posting a schedule that hangs; every other layout builds."""
    import random
    import ftar
    import random_cases
    rng = random.Random(5)
    seen = set()
    for _ in range(400):
        P = rng.randint(2, 13)
        topo, lonely = random_cases.random_topology(rng, P)
        if (P, topo, lonely) in seen:
            continue
        seen.add((P, topo, lonely))
        ins = [fi.fill("f32", 1, r, 97) for r in range(P)]
        try:
            oracle_lib.allreduce(ins, topo, lonely)
            ref_ok = True
        except RuntimeError:
            ref_ok = False
        try:
            ftar.topo_parse(topo, str(lonely), P)
            prod_ok = True
        except ftar.FtarError:
            prod_ok = False
        assert ref_ok == prod_ok, (P, topo, lonely, ref_ok, prod_ok)


@pytest.mark.parametrize("P,topo,lonely", [(13, "2,2,3", 1), (17, "2,2,2,2", 1), (18, "2,2,2,2", 2), (33, "2,2,2,2,2", 1)])
def test_deep_lonely_plans_match_oracle(P, topo, lonely):
    import ftar
    n = 4099
    ins = [fi.fill("f32", 93, r, n) for r in range(P)]
    plans = [ftar.plan_json(ftar.topo(topo, lonely), P, r, n) for r in range(P)]
    outs = simulate(plans, ins, 6, 0, False)
    ref = oracle_lib.allreduce(ins, topo, lonely)
    for r in range(P):
        np.testing.assert_array_equal(outs[r].view(np.uint32), ref[r].view(np.uint32))


def test_direct_allgather_is_one_round():
    """Ring and trees: one all-gather stage with P-1 sends and P-1 receives per rank."""
    import ftar
    for P, topo, L in ((8, "1", 0), (8, "2,2,2", 0), (5, "2,2", 1)):
        for r in range(P):
            p = ftar.plan_json(ftar.topo(topo, L), P, r, 8000, allgather="direct")
            ag = p["stages"][-1]
            assert p["allgather"] == "direct" and not ag["reduces"]
            assert len(ag["sends"]) == P - 1 and len(ag["recvs"]) == P - 1


@pytest.mark.parametrize("dt", ["f32", "bf16", "i32", "f64"])
@pytest.mark.parametrize("P", [2, 3, 5, 8])
def test_direct_ring_is_the_ring_bit_for_bit(P, dt):
    """One-round ring reduce-scatter (fold x_b, x_b+1, ..., x_b+P-1 on rank b-1) == the reference's ring,
    including bf16's per-hop rounding; one stage each way."""
    import ftar
    n = 7 * P + 3
    ins = [fi.fill(dt, 66, r, n) for r in range(P)]
    plans = [ftar.plan_json("1", P, r, n, allgather="direct", reduce_scatter="direct") for r in range(P)]
    assert all(len(p["stages"]) == 2 and p["reduce_scatter"] == "direct" for p in plans)
    outs = simulate(plans, ins, fi.BY_NAME[dt], 0, False)
    staged = simulate([ftar.plan_json("1", P, r, n, "stages", "stages") for r in range(P)], ins, fi.BY_NAME[dt], 0,
                      False)
    ref = oracle_lib.allreduce(ins, "1", dtype=fi.BY_NAME[dt])   # the oracle's ring rounds bf16 once per hop
    for r in range(P):
        assert outs[r].tobytes() == staged[r].tobytes()
        assert outs[r].tobytes() == ref[r].tobytes()


def tree_leaves_py(w, n, s):
    """Depth-first leaf order of block n's fold tree (restated independently of schedule.cpp)."""
    if s == 0:
        return [n]
    g = int(np.prod(w[:s - 1], dtype=np.int64))
    G = g * w[s - 1]
    left = n // G * G + n % g
    out = tree_leaves_py(w, n, s - 1)
    for j in range(w[s - 1]):
        if left + j * g != n:
            out += tree_leaves_py(w, left + j * g, s - 1)
    return out


@pytest.mark.parametrize("dt", ["f32", "bf16", "f64", "i16", "u8", "bool"])
@pytest.mark.parametrize("P,topo", [(4, "2,2"), (6, "2,3"), (6, "3,2"), (8, "2,4"), (8, "4,2"), (8, "2,2,2"),
                                    (9, "3,3"), (12, "2,3,2"), (16, "2,2,2,2"), (16, "4,4"), (27, "3,3,3")])
def test_direct_tree_is_the_tree_bit_for_bit(P, topo, dt):
    """One-round reduce-scatter of a multi-stage tree: rank b gathers every copy of block b and folds them in
    depth-first order of b's fold tree (shape = stage widths, bf16 rounded per inner node) == the staged tree
    and the reference (oracle), one stage each way."""
    import ftar
    n = 7 * P + 3
    w = [int(x) for x in topo.split(",")]
    ins = [fi.fill(dt, 67, r, n) for r in range(P)]
    plans = [ftar.plan_json(topo, P, r, n, allgather="direct", reduce_scatter="direct") for r in range(P)]
    for r, p in enumerate(plans):
        assert len(p["stages"]) == 2 and p["reduce_scatter"] == "direct" and p["max_k"] == P
        if not p["stages"][0]["reduces"]:  # ragged tail: this rank's block is empty
            assert r * ((n + P - 1) // P) >= n
            continue
        (red,) = p["stages"][0]["reduces"]
        assert red["shape"] == w
        # leaf order: own copy where the tree has it, every peer's copy once
        order = [r if b == "src" else None for b, _ in red["srcs"]]
        leaves = tree_leaves_py(w, r, len(w))
        assert [q for q in order if q is not None] == [r] and order.index(r) == leaves.index(r)
        recv_peers = [peer for peer, _, _, _ in p["stages"][0]["recvs"]]
        assert recv_peers == [q for q in leaves if q != r]
    outs = simulate(plans, ins, fi.BY_NAME[dt], 0, False)
    staged = simulate([ftar.plan_json(topo, P, r, n, "stages", "stages") for r in range(P)], ins, fi.BY_NAME[dt], 0,
                      False)
    ref = oracle_lib.allreduce(ins, topo, dtype=fi.BY_NAME[dt])
    for r in range(P):
        assert outs[r].tobytes() == staged[r].tobytes()
        assert outs[r].tobytes() == ref[r].tobytes()


def test_direct_tree_eligibility():
    """Lonely ranks, single-stage trees and trees deeper than the fold kernel's 4 levels keep their stages."""
    import ftar
    assert ftar.plan_json(ftar.topo("2,2", 1), 5, 0, 500)["reduce_scatter"] == "stages"
    assert ftar.plan_json("8", 8, 0, 800)["reduce_scatter"] == "stages"       # already one round
    assert ftar.plan_json("2,2,2,2,2", 32, 0, 3200)["reduce_scatter"] == "stages"
    assert ftar.plan_json("2,2,2,2", 16, 0, 1600)["reduce_scatter"] == "direct"


def test_direct_forms_fall_back_beyond_max_k():
    """More ranks than one reduce takes (FTAR_MAX_K = 64): the ring keeps its neighbour steps."""
    import ftar
    p = ftar.plan_json("1", 65, 3, 65 * 10)
    assert p["reduce_scatter"] == "stages" and p["max_k"] == 2
    assert ftar.plan_json("1", 64, 3, 64 * 10)["reduce_scatter"] == "direct"
    assert ftar.topo_cost("ring", 65, 1 << 30) > ftar.topo_cost("65", 65, 1 << 30)
    # a 65-wide stage is more sources than one reduce takes: the choice never proposes it
    assert str(ftar.topo_choose(67, 1 << 30)) == "ring"     # prime > 64: no tree fits
    for P in (96, 128, 130):
        t = ftar.topo_choose(P, 1 << 30)
        assert t.ring or max(t.widths) <= 64, (P, str(t))
        assert ftar.plan_json(t, P, 1, P * 10)["max_k"] <= 64
