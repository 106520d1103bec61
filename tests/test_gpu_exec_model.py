"""The engine runs what the execution model chooses (csrc/cost_model.cpp, engine.cpp decide_exec), and the
result keeps the reference's bits whatever it chose.

In-process groups on cuda:0 (ftar_comm_init_local), form "auto" and piece 0 -- the defaults: the model's
constants are steered so that it picks whole blocks, many small pieces, or the peer-read / peer-write form;
ftar_comm_last_exec must report exactly ftar_exec_choose's answer, and every rank's output must equal the
pinned oracle's.  Explicit settings are kept over the model."""
import numpy as np
import pytest

import ftar_inputs as fi
import oracle_lib
from gpu_util import from_dev, to_dev

pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.fixture
def model(monkeypatch):
    import ftar
    for k in ("ALPHA_US", "LINK_GBPS", "HBM_GBPS", "ISSUE_US", "BARRIER_US", "PEER_READ_GBPS", "PEER_WRITE_GBPS",
              "COPY_GBPS", "COLL_GBPS"):
        monkeypatch.delenv("FTAR_COST_" + k, raising=False)
    for k in ("FTAR_FORM", "FTAR_CHUNK_BYTES", "FTAR_PEER_DIRECT", "FTAR_ALLGATHER", "FTAR_REDUCE_SCATTER",
              "FT_TOPO", "FT_LONELY"):
        monkeypatch.delenv(k, raising=False)
    ftar.cost_set()
    yield ftar
    ftar.cost_set()


def _run(ftar, g, ins, topo):
    n = ins[0].size
    bufs = [to_dev(x) for x in ins]
    g.allreduce(None, [p for _, p in bufs], n, "f32", "sum", topo_=topo)
    return [from_dev(t, ins[0].dtype, n) for t, _ in bufs]


@pytest.mark.parametrize("P,topo", [(4, "4"), (4, "1"), (6, "2,3"), (8, None)])
@pytest.mark.parametrize("steer,want_form", [
    ({"alpha_us": 5000.0}, "direct"),                                    # per-piece cost dominates: whole blocks
    # per-piece costs tiny, transfer and fold of a block comparable: the pipeline hides one under the other,
    # so the model cuts blocks into pieces
    ({"alpha_us": 0.05, "issue_us": 0.05, "link_gbps": 700.0}, "direct"),
    ({"peer_read_gbps": 5000.0, "barrier_us": 1.0}, "peer-read"),
    ({"peer_write_gbps": 5000.0, "barrier_us": 1.0}, "peer-write"),
])
def test_engine_runs_the_models_choice_with_the_reference_bits(model, P, topo, steer, want_form):
    ftar = model
    n = (1 << 22) + 37   # 16 MiB per rank, ragged blocks
    ins = [fi.fill("f32", 55, r, n) for r in range(P)]
    ftar.cost_set(**steer)
    g = ftar.Comm.init_local(P)
    try:
        assert all(c.form == "auto" and c.chunk_bytes == 0 for c in g.comms)
        outs = _run(ftar, g, ins, topo)
        want = ftar.exec_choose(P, n * 4, topo_=topo).as_dict()
        for c in g.comms:
            ran = c.last_exec()
            assert ran == want, (ran, want)
        assert want["form"] == want_form, want
        if "alpha_us" in steer and steer["alpha_us"] > 1000:
            assert want["chunk_bytes"] == 0   # whole blocks
        elif want_form == "direct":
            assert 0 < want["chunk_bytes"] < 4 * MiB   # several pieces per 4 MiB block
        ref = oracle_lib.allreduce(ins, topo or want["topology"].replace("ring", "1"))
        for r in range(P):
            assert outs[r].tobytes() == ref[r].tobytes(), f"rank {r}"
    finally:
        g.destroy()


def test_explicit_settings_are_kept_over_the_model(model):
    ftar = model
    P, n = 4, (1 << 20) + 5
    ins = [fi.fill("f32", 56, r, n) for r in range(P)]
    ftar.cost_set(peer_read_gbps=5000.0, barrier_us=1.0)   # the model alone would take peer-read
    g = ftar.Comm.init_local(P)
    try:
        g.set_form("stages")
        g.set_chunk_bytes(64 << 10)
        outs = _run(ftar, g, ins, "4")
        ran = g.comms[0].last_exec()
        assert ran["form"] == "stages" and ran["chunk_bytes"] == 64 << 10, ran
        ref = oracle_lib.allreduce(ins, "4")
        assert all(outs[r].tobytes() == ref[r].tobytes() for r in range(P))
        g.set_form("auto")
        g.set_chunk_bytes(0)
        _run(ftar, g, ins, "4")
        assert g.comms[0].last_exec()["form"] == "peer-read"
        # a setter for one knob fixes the form the knobs then describe
        g.set_reduce_scatter("direct")
        g.set_allgather("collective")
        assert g.comms[0].form == "collective"
        g.set_reduce_scatter("stages")
        assert g.comms[0].form == -2   # stages reduce-scatter + collective all-gather: no single form names it
        outs = _run(ftar, g, ins, "4")
        assert all(outs[r].tobytes() == ref[r].tobytes() for r in range(P))
    finally:
        g.destroy()


def test_model_choice_follows_new_constants_between_calls(model):
    """Choices are cached per communicator; a change of constants (ftar_cost_set) is seen at the next call."""
    ftar = model
    P, n = 4, 1 << 22
    ins = [fi.fill("f32", 57, r, n) for r in range(P)]
    g = ftar.Comm.init_local(P)
    try:
        _run(ftar, g, ins, "4")
        first = g.comms[0].last_exec()
        ftar.cost_set(peer_write_gbps=5000.0, barrier_us=1.0)
        outs = _run(ftar, g, ins, "4")
        second = g.comms[0].last_exec()
        assert first["form"] == "direct" and second["form"] == "peer-write", (first, second)
        ref = oracle_lib.allreduce(ins, "4")
        assert all(np.array_equal(outs[r].view(np.uint32), ref[r].view(np.uint32)) for r in range(P))
    finally:
        g.destroy()
