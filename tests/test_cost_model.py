"""The xGMI execution model (csrc/cost_model.cpp): what it prices and that its choice moves with the node's
constants.  The reference's model (cost_model/CostModel.h:82-120) chooses a width list for a chunk size; on
one MI355X node the one-round forms make every topology move tree(P)'s bytes, so the decisions that vary are
the data-movement form and the pipeline piece -- these tests drive them with synthetic constants, as a fit
from ftar_xgmi_probe and the sweep would (bench.py)."""
import pytest

import ftar

GiB, MiB = 1 << 30, 1 << 20


@pytest.fixture(autouse=True)
def _defaults(monkeypatch):
    monkeypatch.delenv("FTAR_COST_FILE", raising=False)
    for k in ("ALPHA_US", "LINK_GBPS", "HBM_GBPS", "ISSUE_US", "BARRIER_US", "PEER_READ_GBPS", "PEER_WRITE_GBPS",
              "COPY_GBPS", "COLL_GBPS"):
        monkeypatch.delenv("FTAR_COST_" + k, raising=False)
    monkeypatch.delenv("FTAR_COST_MODEL", raising=False)
    ftar.cost_set()
    ftar.cost_load(None)
    yield
    ftar.cost_set()
    ftar.cost_load(None)


def _piece(e):
    return e.chunk_bytes or float("inf")   # 0 = whole blocks


def test_defaults_choose_one_round_width_p_with_pipelined_pieces():
    e = ftar.exec_choose(8, GiB)
    assert str(e.topo) == "8" and ftar.FORM_NAME[e.form] == "direct"
    assert 16 * MiB <= e.chunk_bytes < 128 * MiB   # a few pieces per 128 MiB block: the last fold hides
    assert e.seconds == pytest.approx(ftar.cost_predict("8", "direct", e.chunk_bytes, 8, GiB))
    # unmeasured rates: the peer forms and the collective are never chosen, nor priced
    assert ftar.cost_predict("8", "peer-read", 0, 8, GiB) is None
    assert ftar.cost_predict("8", "collective", 0, 8, GiB) is None


def test_the_direct_form_topology_tie_is_reported():
    """In the direct form every one-round topology (tree(8), 2,4, 4,2, 2,2,2, the ring) moves tree(P)'s
    bytes over the same links and prices identically: the choice of tree(8) is a tie broken by the fewest
    stages, and the result says so."""
    e = ftar.exec_choose(8, GiB)
    assert e.tied >= 5 and ftar.TIE_NAME[e.tie_broken_by] == "stages"
    assert e.as_dict()["tie_broken_by"] == "stages" and e.as_dict()["tied"] == e.tied
    # the topology fixed, the piece free: a strict argmin, no tie
    f = ftar.exec_choose(8, GiB, topo_="8", form="direct")
    assert f.tied == 1 and f.tie_broken_by == 0 and "tie_broken_by" not in f.as_dict()


def test_default_link_is_the_spec_times_the_stated_efficiency():
    """The default link rate is the xGMI spec (76.8 GB/s per direction) times the stated RCCL p2p
    efficiency (0.7, csrc/cost_model.cpp), not an unexplained constant."""
    assert ftar.cost_get()["link_gbps"] == pytest.approx(76.8 * 0.7)


def test_small_buckets_take_whole_blocks():
    for nbytes in (4096, 1 << 20):
        assert ftar.exec_choose(8, nbytes).chunk_bytes == 0


def test_piece_grows_with_per_piece_overhead():
    """alpha (one p2p group) and issue (the host's enqueue of a piece) charge every piece: the more they
    cost, the fewer and larger the pieces."""
    pieces = []
    for alpha in (0.5, 20.0, 400.0, 4000.0):
        ftar.cost_set(alpha_us=alpha, issue_us=0.5)
        pieces.append(_piece(ftar.exec_choose(8, GiB)))
    assert pieces == sorted(pieces) and pieces[0] < pieces[-1], pieces
    ftar.cost_set(alpha_us=0.5, issue_us=2000.0)
    assert _piece(ftar.exec_choose(8, GiB)) > pieces[0]


def test_piece_shrinks_when_the_fold_is_exposed():
    """A fast link leaves the fold (on the reduce stream) as the long pole: smaller pieces hide all but the
    last one, so the choice moves toward more pieces as the link rate rises."""
    pieces = []
    for link in (10.0, 48.0, 1000.0, 20000.0):
        ftar.cost_set(link_gbps=link, alpha_us=2.0, issue_us=1.0)
        pieces.append(_piece(ftar.exec_choose(8, GiB)))
    assert pieces == sorted(pieces, reverse=True) and pieces[-1] < pieces[0], pieces


def test_form_moves_with_the_peer_rates():
    ftar.cost_set(peer_read_gbps=300.0, barrier_us=30.0)
    assert ftar.FORM_NAME[ftar.exec_choose(8, GiB).form] == "peer-read"
    ftar.cost_set(peer_read_gbps=20.0, barrier_us=30.0)           # slower than RCCL's 48 GB/s per link
    assert ftar.FORM_NAME[ftar.exec_choose(8, GiB).form] == "direct"
    ftar.cost_set(peer_write_gbps=300.0, peer_read_gbps=100.0)
    assert ftar.FORM_NAME[ftar.exec_choose(8, GiB).form] == "peer-write"
    # the peer forms are a choice only where the caller allows them (device buffers, no capture)
    assert ftar.FORM_NAME[ftar.exec_choose(8, GiB, peer=False).form] == "direct"
    # registered buffers skip the local pass
    assert ftar.cost_predict("8", "peer-write", 0, 8, GiB, registered=True) < \
        ftar.cost_predict("8", "peer-write", 0, 8, GiB)


def test_barriers_price_the_peer_forms_out_of_small_buckets():
    ftar.cost_set(peer_read_gbps=300.0, barrier_us=200.0)
    assert ftar.FORM_NAME[ftar.exec_choose(8, 1 << 20).form] == "direct"
    assert ftar.FORM_NAME[ftar.exec_choose(8, GiB).form] == "peer-read"


def test_collective_all_gather_when_its_rate_is_known():
    ftar.cost_set(coll_gbps=400.0)
    e = ftar.exec_choose(8, GiB)
    assert ftar.FORM_NAME[e.form] == "collective" and not e.topo.ring
    assert ftar.cost_predict("ring", "collective", 0, 8, GiB) is None   # the ring's blocks sit one rank off
    ftar.cost_set(coll_gbps=10.0)
    assert ftar.FORM_NAME[ftar.exec_choose(8, GiB).form] == "direct"


def test_staged_rounds_cost_more_than_one_round():
    for P in (2, 4, 8):
        for c in (4 * MiB, 64 * MiB, 0):
            d = ftar.cost_predict("1", "direct", c, P, GiB)
            s = ftar.cost_predict("1", "stages", c, P, GiB)
            assert d <= s, (P, c)
            if P > 2:
                assert d < s
    # with stages fixed the topology matters again: tree(8) moves each byte once per direction
    e = ftar.exec_choose(8, GiB, form="stages")
    assert str(e.topo) == "8"
    assert ftar.cost_predict("2,2,2", "stages", 64 * MiB, 8, GiB) > ftar.cost_predict("8", "stages", 64 * MiB, 8, GiB)


def test_fixed_choices_are_kept():
    e = ftar.exec_choose(8, GiB, topo_="2,4", form="stages", chunk_bytes=4 * MiB)
    assert str(e.topo) == "2,4" and ftar.FORM_NAME[e.form] == "stages" and e.chunk_bytes == 4 * MiB
    e = ftar.exec_choose(8, GiB, topo_="1", form="direct")
    assert e.topo.ring and e.chunk_bytes > 0


def test_environment_overrides_the_set_constants(monkeypatch):
    ftar.cost_set(alpha_us=7.0, issue_us=3.0)
    assert ftar.cost_get()["alpha_us"] == pytest.approx(7.0)
    monkeypatch.setenv("FTAR_COST_ALPHA_US", "123")
    monkeypatch.setenv("FTAR_COST_PEER_WRITE_GBPS", "55")
    p = ftar.cost_get()
    assert p["alpha_us"] == pytest.approx(123.0) and p["peer_write_gbps"] == pytest.approx(55.0)
    assert p["issue_us"] == pytest.approx(3.0)


def test_round2_three_constant_api_still_sets_the_model():
    ftar.cost_params(alpha_us=50.0, link_gbps=60.0, hbm_gbps=6000.0)
    p = ftar.cost_get()
    assert (p["alpha_us"], p["link_gbps"], p["hbm_gbps"]) == pytest.approx((50.0, 60.0, 6000.0))
    assert ftar.cost_params() == pytest.approx({"alpha_us": 50.0, "link_GBps": 60.0, "hbm_GBps": 6000.0})


def test_topology_choice_is_the_reference_question_at_the_default_form():
    # the ring and multi-stage trees move tree(P)'s bytes in the direct forms: tree(P) on the tie
    for P in (2, 4, 6, 8):
        assert str(ftar.topo_choose(P, GiB)) == str(P)
    assert ftar.topo_cost("ring", 8, GiB) == pytest.approx(ftar.topo_cost("8", 8, GiB))


def test_choice_is_a_pure_function_of_the_constants():
    """Every rank computes the same choice from the same constants (they are compared across ranks at a
    communicator's first call): repeated calls agree, and a change of constants changes the cached result."""
    a = ftar.exec_choose(8, GiB).as_dict()
    assert ftar.exec_choose(8, GiB).as_dict() == a
    ftar.cost_set(alpha_us=4000.0)
    assert ftar.exec_choose(8, GiB).as_dict() != a


def test_calibration_file_round_trip_and_precedence(tmp_path, monkeypatch):
    """A run on the node saves its fitted constants (ftar_cost_save, bench.py --save-cost); a later process
    loads them (ftar_cost_load or FTAR_COST_FILE) and the model prices with them.  Precedence:
    FTAR_COST_<FIELD> > ftar_cost_set > the file > the defaults."""
    path = str(tmp_path / "node.cost")
    ftar.cost_set(alpha_us=33.0, link_gbps=61.5, peer_read_gbps=90.0, issue_us=12.0)
    fitted = ftar.cost_get()
    ftar.cost_save(path)
    ftar.cost_set()
    assert ftar.cost_get()["peer_read_gbps"] == 0.0
    assert ftar.cost_load(path) == pytest.approx(fitted)
    with open(path) as f:
        assert "alpha_us 33\n" in f.read()
    # the loaded peer rate makes the peer form a candidate: the choice moves with the file
    e = ftar.exec_choose(8, GiB)
    assert ftar.cost_predict("8", "peer-read", 0, 8, GiB) is not None
    ftar.cost_set(link_gbps=10.0)   # set beats the file
    assert ftar.cost_get()["link_gbps"] == pytest.approx(10.0) and ftar.cost_get()["alpha_us"] == pytest.approx(33.0)
    monkeypatch.setenv("FTAR_COST_LINK_GBPS", "7")   # the environment beats both
    assert ftar.cost_get()["link_gbps"] == pytest.approx(7.0)
    assert e.seconds > 0


def test_cost_file_from_the_environment(tmp_path, monkeypatch):
    a, b = tmp_path / "a.cost", tmp_path / "b.cost"
    a.write_text("# node A\nalpha_us = 40\nlink_gbps 70   # per peer\n\n")
    b.write_text("coll_gbps 300\n")
    monkeypatch.setenv("FTAR_COST_FILE", str(a))
    k = ftar.cost_get()
    assert k["alpha_us"] == pytest.approx(40.0) and k["link_gbps"] == pytest.approx(70.0) and k["coll_gbps"] == 0.0
    monkeypatch.setenv("FTAR_COST_FILE", str(b))   # re-read when the variable changes
    k = ftar.cost_get()
    assert k["alpha_us"] == pytest.approx(20.0) and k["coll_gbps"] == pytest.approx(300.0)
    monkeypatch.delenv("FTAR_COST_FILE")
    assert ftar.cost_get()["coll_gbps"] == 0.0


def test_cost_file_variable_and_explicit_load_are_kept_apart(tmp_path, monkeypatch):
    """a malformed FTAR_COST_FILE leaves the previous file's constants in effect (and fails bring-up,
    cost_file_status); unsetting the variable drops its file's constants but not ftar_cost_load's; the
    variable's file beats the explicit load field by field."""
    a, bad, loaded = tmp_path / "a.cost", tmp_path / "bad.cost", tmp_path / "l.cost"
    a.write_text("alpha_us 40\n")
    bad.write_text("alpha_us fast\n")
    loaded.write_text("alpha_us 11\nissue_us 13\n")
    ftar.cost_load(str(loaded))
    assert ftar.cost_get()["alpha_us"] == pytest.approx(11.0)
    monkeypatch.setenv("FTAR_COST_FILE", str(a))
    k = ftar.cost_get()
    assert k["alpha_us"] == pytest.approx(40.0) and k["issue_us"] == pytest.approx(13.0)
    monkeypatch.setenv("FTAR_COST_FILE", str(bad))
    assert ftar.cost_get()["alpha_us"] == pytest.approx(40.0)   # a's constants stay
    monkeypatch.delenv("FTAR_COST_FILE")
    k = ftar.cost_get()
    assert k["alpha_us"] == pytest.approx(11.0) and k["issue_us"] == pytest.approx(13.0)   # the load stays
    ftar.cost_load(None)
    assert ftar.cost_get()["alpha_us"] == pytest.approx(20.0)


@pytest.mark.parametrize("text", ["alpha_us 0\n", "alpha_us -3\n", "not_a_field 5\n", "link_gbps 5 6\n",
                                  "link_gbps fast\n", "link_gbps nan\n"])
def test_malformed_cost_files_are_refused(tmp_path, text):
    p = tmp_path / "bad.cost"
    p.write_text("issue_us 10\n" + text)
    before = ftar.cost_get()
    with pytest.raises(ftar.FtarError) as e:
        ftar.cost_load(str(p))
    assert e.value.status == 1 and "line 2" in str(e.value)
    assert ftar.cost_get() == before   # nothing of the file applied
    with pytest.raises(ftar.FtarError):
        ftar.cost_load(str(tmp_path / "missing.cost"))
