"""bench.py host-side helpers (CPU)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.parametrize("n", [1, 2, 7, 4096, 4097, (1 << 24) + 1, 1 << 28, 1 << 29, (1 << 31) + 5])
def test_sample_index_stays_in_bounds(n):
    """Sample indices of the N>1 correctness check: int64, first 0, last n-1, never n (a float32 linspace
    over 2^28 elements rounds its last index up to 2^28, one past the end of the bucket)."""
    import bench
    idx = bench.sample_index(n, "cpu")
    assert idx.dtype.is_floating_point is False
    assert int(idx[0]) == 0 and int(idx[-1]) == n - 1
    assert bool((idx[1:] >= idx[:-1]).all())


def test_factorizations():
    import bench
    assert bench._factorizations(8) == [[2, 2, 2], [2, 4], [4, 2], [8]]
    assert bench._factorizations(1) == []


def test_roofline_world_size_one_is_hbm():
    """P = 1 crosses no link: the line's roofline is the local pass over the bucket (read + write) against
    HBM, never an xGMI fraction (the round-1 world-size-1 rehearsal printed xgmi frac 38.29)."""
    import bench
    r = bench.allreduce_roofline(1, 1, 1 << 30, 0.35, 7)
    assert r["bound"] == "hbm" and r["peak"] == bench.HBM_PEAK_GBPS
    assert r["achieved"] == pytest.approx(2 * (1 << 30) / 0.35e-3 / 1e9, rel=1e-4)
    assert 0 < r["frac"] <= 1


def test_roofline_rehearsal_has_none():
    import bench
    assert bench.allreduce_roofline(4, 1, 1 << 28, 10.0, 3) is None


@pytest.mark.parametrize("world,links", [(2, 1), (4, 3), (8, 7)])
def test_roofline_xgmi_frac_in_range(world, links):
    import bench
    bucket = 1 << 30
    for ms in (3.0, 10.0, 50.0, 100.0):
        r = bench.allreduce_roofline(world, 8, bucket, ms, links)
        alg = bucket / (ms * 1e-3) / 1e9
        assert r["achieved"] == pytest.approx(alg * 2 * (world - 1) / world, rel=1e-3)
        if r["frac"] is not None:
            assert 0 < r["frac"] <= 1
            assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-4)
    # a run faster than the links allow: no fraction at all
    r = bench.allreduce_roofline(world, 8, bucket, 0.01, links)
    assert r["frac"] is None and "no fraction" in r["note"]


def test_roofline_frac_is_against_the_spec_and_the_probe_only_adds_a_ratio():
    """frac is always busBW / (links x 76.8 GB/s spec, one direction); the probe's measured per-link
    rate gives only `frac_of_probe`, so a slow or under-driven probe cannot raise frac."""
    import bench
    probe = {"read_one_peer": [60.0, 62.0], "read_all_peers": [400.0, 410.0], "write_one_peer": [50.0, 51.0],
             "write_all_peers": [350.0, 360.0], "note": "x"}
    rate = bench.link_rate_from_probe(probe, 8)
    assert rate == pytest.approx(60.0)   # the slowest rank's best per-link mode: one peer beats 400/7
    bucket = 1 << 30
    ms = bucket * 2 * 7 / 8 / (7 * 50.0 * 1e9) * 1e3   # busBW 50 GB/s per link
    r = bench.allreduce_roofline(8, 8, bucket, ms, 7, rate)
    assert r["peak"] == pytest.approx(7 * 76.8) and r["frac"] == pytest.approx(50.0 / 76.8, abs=1e-4)
    assert r["probe_peak"] == pytest.approx(420.0) and r["frac_of_probe"] == pytest.approx(50.0 / 60.0, abs=1e-4)
    assert "ONE-direction" in r["direction_convention"]
    slow = bench.allreduce_roofline(8, 8, bucket, ms, 7, 10.0)   # a bad probe: frac unchanged
    assert slow["frac"] == r["frac"] and slow["frac_of_probe"] > 1
    assert "frac_of_probe" not in bench.allreduce_roofline(8, 8, bucket, ms, 7)
    assert bench.link_rate_from_probe(None, 8) is None
    assert bench.link_rate_from_probe({"error": "x"}, 8) is None
    assert bench.link_rate_from_probe(probe, 1) is None


def test_links_driven():
    import bench
    assert bench.links_driven(8, "8", "direct") == 7
    assert bench.links_driven(8, "ring", "peer-read-reg:dma") == 7
    assert bench.links_driven(8, "ring", "stages") == 1
    assert bench.links_driven(8, "2,4", "stages") == 3
    assert bench.links_driven(5, "2,2+1", "stages") == 1
    assert bench.links_driven(2, "2", "direct:ncclreg") == 1


def test_rccl_p2p_best_is_reported_when_a_peer_form_wins():
    """the headline may be an IPC peer form; the fastest validated RCCL ncclSend/ncclRecv
    configuration is reported next to it with its own roofline.  Invalid entries, errors and the collective
    form (ncclAllGather) do not count."""
    import bench
    bucket = 1 << 30
    sweep = [
        {"topology": "8", "chunk_bytes": 16 << 20, "form": "direct", "ms": 6.0, "check": "ok"},
        {"topology": "8", "chunk_bytes": 1 << 20, "form": "direct", "ms": 5.5, "check": "MISMATCH (sample)"},
        {"topology": "8", "chunk_bytes": 4 << 20, "form": "direct:ncclreg", "ms": 5.8, "check": "ok"},
        {"topology": "8", "chunk_bytes": 16 << 20, "form": "collective", "ms": 5.0, "check": "ok"},
        {"topology": "ring", "chunk_bytes": 16 << 20, "form": "stages", "ms": 40.0, "check": "ok"},
        {"topology": "8", "chunk_bytes": 16 << 20, "form": "peer-write-reg", "ms": 4.0, "check": "ok"},
        {"topology": "2,4", "chunk_bytes": 16 << 20, "form": "direct", "error": "ncclSend failed"},
        {"skipped": "sweep budget"},
    ]
    best = bench.rccl_p2p_best(sweep, 8, 8, bucket, lambda r: bench.links_driven(8, r["topology"], r["form"]))
    assert best["form"] == "direct:ncclreg" and best["chunk_bytes"] == 4 << 20 and best["ms"] == 5.8
    assert best["roofline"]["bound"] == "xgmi" and best["roofline"]["peak"] == pytest.approx(7 * 76.8)
    alg = bucket / 5.8e-3 / 1e9
    assert best["busbw_GBps_per_rank"] == pytest.approx(alg * 14 / 8, rel=1e-3)
    only_peer = [e for e in sweep if e.get("form", "").startswith("peer")]
    assert bench.rccl_p2p_best(only_peer, 8, 8, bucket, lambda r: 7) is None


def test_pmc_traffic_only_for_the_kernel_it_measured(tmp_path):
    """roofline.traffic comes from profiles/pmc_summary.json only when that entry measured
    the kernel this run launched (same template id) built from the same kernel sources; otherwise None and a
    note saying which kernel the summary holds."""
    import json
    import bench
    dig = bench.kernel_source_digest()
    k = "reduce_lds_kernel<F32Sum, 2, 1, 2, 2, true>"
    entry = {"kernel": k, "commit": "abc", "kernel_sources_sha": dig, "hbm_bytes_per_launch": 805339648.0,
             "source": "profiles/r03/final"}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"reduce_k2_f32_n67108864": entry}))
    t, prov = bench.pmc_traffic("reduce_k2_f32_n67108864", k, str(p))
    assert t == 805339648.0 and prov["traffic_source"]["commit"] == "abc"
    t, prov = bench.pmc_traffic("reduce_k2_f32_n67108864", "reduce_lds_kernel<F32Sum, 2, 4, 4, 2, true>", str(p))
    assert t is None and k in prov["traffic_note"]
    p.write_text(json.dumps({"reduce_k2_f32_n67108864": dict(entry, kernel_sources_sha="0" * 16)}))
    t, prov = bench.pmc_traffic("reduce_k2_f32_n67108864", k, str(p))
    assert t is None and "kernel sources" in prov["traffic_note"]
    t, prov = bench.pmc_traffic("reduce_k8_f32_n67108864", k, str(p))
    assert t is None and "no PMC measurement" in prov["traffic_note"]


def test_committed_pmc_summary_names_kernel_commit_and_sources():
    """Every entry of the committed summary says which kernel, commit and kernel sources it measured."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", "pmc_summary.json")) as f:
        d = json.load(f)
    for key, e in d.items():
        assert e["kernel"].startswith("reduce_"), key
        assert e.get("commit") and e.get("kernel_sources_sha"), key
        assert 0.99 < e["traffic_over_algorithmic"] < 1.05, key


def test_pmc_summary_keeps_only_the_bench_lines_own_launches(tmp_path):
    """tools/pmc_summary.py: the same k-way kernel also runs on smaller pieces in later line items (engine_local,
    host_local); only launches with the grid of the first one enter the median, and the two passes must name
    one kernel."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    name = ("void ftar::(anonymous namespace)::reduce_lds_kernel<ftar::(anonymous namespace)::F32Sum, 2, 1, 2, 2, "
            "true>(ftar::(anonymous namespace)::Srcs<2>, void*, unsigned long, int, int)")
    n = 1 << 26
    write_kb = n * 4 / 1024

    def csv_of(counter, big, small):
        lines = ["Kernel_Name,Grid_Size,Counter_Name,Counter_Value"]
        lines += [f'"{name}",16384,{counter},{big}'] * 5 + [f'"{name}",4096,{counter},{small}'] * 9
        return "\n".join(lines) + "\n"
    (tmp_path / "f.csv").write_text(csv_of("FETCH_SIZE", 2 * n * 4 / 2 / 1024, 100.0))  # 2 x FETCH x 1 KiB = 2 inputs
    (tmp_path / "w.csv").write_text(csv_of("WRITE_SIZE", write_kb, 10.0))
    (tmp_path / "meta.json").write_text(json.dumps({"commit": "c0ffee", "kernel_sources_sha": "s" * 16}))
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(root, "tools", "pmc_summary.py"), str(tmp_path / "f.csv"),
                    str(tmp_path / "w.csv"), "--k", "2", "--out", str(out), "--meta", str(tmp_path / "meta.json")],
                   check=True, capture_output=True)
    e = json.loads(out.read_text())[f"reduce_k2_f32_n{n}"]
    assert e["launches"] == 5 and e["kernel"] == "reduce_lds_kernel<F32Sum, 2, 1, 2, 2, true>"
    assert e["traffic_over_algorithmic"] == pytest.approx(1.0) and e["commit"] == "c0ffee"
    (tmp_path / "w.csv").write_text(csv_of("WRITE_SIZE", write_kb, 10.0).replace("2, 1, 2, 2", "2, 4, 2, 2"))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "pmc_summary.py"), str(tmp_path / "f.csv"),
                        str(tmp_path / "w.csv"), "--k", "2", "--out", str(out)], capture_output=True, text=True)
    assert r.returncode != 0 and "different kernels" in r.stderr


def test_kernel_symbol_normalises_rocprof_names():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "allreduce-over-mpi_amd", "ftar"))
    from names import kernel_symbol
    raw = ("void ftar::(anonymous namespace)::reduce_lds_kernel<ftar::(anonymous namespace)::F32Sum, 8, 4, 2, 2, "
           "true>(ftar::(anonymous namespace)::Srcs<8>, void*, unsigned long, int, int)")
    assert kernel_symbol(raw) == "reduce_lds_kernel<F32Sum, 8, 4, 2, 2, true>"
    assert kernel_symbol("void ftar::(anonymous namespace)::gather_kernel<true>(ftar::SegArgs, int)") == \
        "gather_kernel<true>"


def test_host_cores_reports_the_share_not_the_machine():
    """the CPU baseline states the cores this process may use (affinity, cgroup quota)."""
    import bench
    hc = bench.host_cores()
    assert hc["machine_cpus"] == os.cpu_count()
    assert hc["affinity_cpus"] == len(os.sched_getaffinity(0))
    assert 0 < hc["available_cpus"] <= hc["machine_cpus"]


def test_reference_mpi_path_runs_the_reference_on_the_host():
    """bench.py's N>1 line item `reference_cpu_mpi`: the reference's own MPI_Allreduce_FT (oracle/_ref/ref_golden
    arbench, built from the unmodified mpi_mod.hpp) with P MPI ranks on the host, timed like benchmark.cpp.
    Runs here on CPU (no GPU needed); P = 1 has nothing to time."""
    import bench
    ref = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "ref_golden")
    if not (os.path.exists(ref) and os.path.exists("/opt/conda/bin/mpiexec")):
        pytest.skip("reference driver or MPICH not built here")
    assert bench.reference_mpi_path(1) is None
    d = bench.reference_mpi_path(2, n=1 << 16, repeat=3, seconds=60)
    assert "error" not in d, d
    assert d["kind"] == "reference" and d["P"] == 2 and d["n"] == 1 << 16 and d["topo"] == "1"
    assert 0 < d["min_s"] <= d["first_s"] and d["algbw_GBps_min"] > 0


def test_probe_cap_entries_only_where_a_cap_wins():
    """The peer forms' copy cap is tried only where the xGMI probe saw a capped copy beat the uncapped one by
    more than 10 % (rates: min over ranks), per direction."""
    import bench
    probe = {"read_all_peers": [300.0, 310.0], "write_all_peers": [400.0, 405.0]}
    by_cap = {4: {"read_all_peers": 200.0, "write_all_peers": 300.0},
              16: {"read_all_peers": 350.0, "write_all_peers": 420.0},
              64: {"read_all_peers": 320.0, "write_all_peers": 410.0}}
    assert bench.probe_cap_entries(probe, by_cap) == ["peer-read-reg:wg16"]
    assert bench.probe_cap_entries(probe, {8: {"read_all_peers": 100.0, "write_all_peers": 100.0}}) == []
    assert bench.probe_cap_entries({"error": "x"}, by_cap) == []
    assert bench.probe_cap_entries(probe, {}) == []


@pytest.fixture
def model_defaults():
    import ftar
    saved = {k: os.environ.pop(k) for k in list(os.environ) if k.startswith("FTAR_COST_")}
    ftar.cost_set()
    yield ftar
    ftar.cost_set()
    os.environ.update(saved)


def _synthetic_sweep(ftar, bench, world, bucket, true):
    """sweep entries timed by the model itself under `true` constants: direct / stages over three topologies
    and the C4 piece sizes, the peer forms and the collective"""
    ftar.cost_set(**true)
    sweep = []
    for topo in ("8", "ring", "2,4"):
        for form in ("direct", "stages"):
            for c in (256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
                if form == "stages" and topo == "ring" and c != 16 << 20:
                    continue
                sweep.append({"topology": topo, "form": form, "chunk_bytes": c, "check": "ok",
                              "ms": bench.predict_ms(ftar, topo, form, c, world, bucket)})
    for topo in ("8", "2,4", "ring"):   # one-round plans: the peer forms run each
        for form in ("peer-read", "peer-write", "peer-read-reg") + (("peer-write-reg:plain",) if topo == "8" else ()):
            sweep.append({"topology": topo, "form": form, "chunk_bytes": 0, "check": "ok",
                          "ms": bench.predict_ms(ftar, topo, form, 0, world, bucket)})
    sweep.append({"topology": "8", "form": "collective", "chunk_bytes": 16 << 20, "check": "ok",
                  "ms": bench.predict_ms(ftar, "8", "collective", 16 << 20, world, bucket)})
    sweep.append({"topology": "8", "form": "direct", "chunk_bytes": 1 << 20, "check": "MISMATCH (sample)",
                  "ms": 0.001})   # never fitted: it did not validate
    ftar.cost_set()
    return sweep


def test_sweep_forms_are_priced_as_their_base_form(model_defaults):
    import bench
    ftar = model_defaults
    assert bench.sweep_form("peer-read-reg:wg16") == ("peer-read", True)
    assert bench.sweep_form("direct:ncclreg") == ("direct", False)
    assert bench.predict_ms(ftar, "8", "direct:ncclreg", 1 << 20, 8, 1 << 30) == \
        bench.predict_ms(ftar, "8", "direct", 1 << 20, 8, 1 << 30)
    assert bench.predict_ms(ftar, "8", "peer-read", 0, 8, 1 << 30) is None   # no peer rate yet
    assert bench.predict_ms(ftar, "8", "auto", 0, 8, 1 << 30) is None


def test_pieces_per_round_follow_the_engine():
    import bench
    # 1 GiB over 8 ranks: 128 MiB blocks
    assert bench.pieces_per_round(16 << 20, 8, 1 << 30, 4) == 8
    assert bench.pieces_per_round(24 * (1 << 20) + 4096, 8, 1 << 30, 4) == 6
    assert bench.pieces_per_round(0, 8, 1 << 30, 4) == 1
    assert bench.pieces_per_round(256 << 20, 8, 1 << 30, 4) == 1


def test_issue_cost_comes_from_the_enqueue_times():
    import bench
    sweep = [{"form": "direct", "chunk_bytes": 1 << 20, "enqueue_ms": 25.6, "ms": 60.0, "check": "ok"},  # 256 groups
             {"form": "direct", "chunk_bytes": 16 << 20, "enqueue_ms": 1.6, "ms": 9.0, "check": "ok"},   # 16 groups
             {"form": "stages", "chunk_bytes": 1 << 20, "enqueue_ms": 99.0, "ms": 300.0, "check": "ok"},
             {"form": "direct", "chunk_bytes": 4 << 20, "enqueue_ms": 6.4, "ms": 20.0, "check": "ok"},    # 64 groups
             # the enqueue waited for the device (RCCL's work queue full): not a host cost, left out
             {"form": "direct", "chunk_bytes": 256 << 10, "enqueue_ms": 900.0, "ms": 910.0, "check": "ok"}]
    assert bench.issue_from_enqueue(sweep, 8, 1 << 30, 4) == pytest.approx(100.0)
    assert bench.issue_from_enqueue([], 8, 1 << 30, 4) is None


@pytest.mark.parametrize("true", [dict(alpha_us=35.0, link_gbps=60.0, issue_us=12.0),
                                  dict(alpha_us=150.0, link_gbps=20.0, issue_us=5.0)])
def test_refit_recovers_the_constants_of_a_synthetic_node(model_defaults, true):
    """The sweep timed by the model under known constants: the refit finds them again (alpha and link;
    issue is held at its directly measured value) and predicts every entry within 1 %."""
    import bench
    ftar = model_defaults
    world, bucket = 8, 1 << 30
    sweep = _synthetic_sweep(ftar, bench, world, bucket, dict(true, peer_read_gbps=90.0, peer_write_gbps=70.0,
                                                             coll_gbps=300.0))
    fit = bench.refit_cost_model(ftar, sweep, world, bucket, fixed={"issue_us": true["issue_us"]})
    assert fit["entries"] == 26 and fit["rms_log_err"] < 0.01 and fit["unidentified"] == {}
    assert fit["params"]["alpha_us"] == pytest.approx(true["alpha_us"], rel=0.05)
    assert fit["params"]["link_gbps"] == pytest.approx(true["link_gbps"], rel=0.02)
    for field, forms, want in (("peer_read_gbps", ("peer-read", "peer-read-reg"), 90.0),
                               ("peer_write_gbps", ("peer-write", "peer-write-reg"), 70.0)):
        r = bench.refit_form_rate(ftar, sweep, world, bucket, field, forms)
        if field == "peer_write_gbps":   # the ":plain" entry is a tuning variant, not a fit point
            assert r["entries"] == 3
        assert r["unidentified"] is None and r["value"] == pytest.approx(want, rel=0.02), field
    # the collective ran once: too few entries to fit a rate -- flagged, the prior (unmeasured: 0) kept
    r = bench.refit_form_rate(ftar, sweep, world, bucket, "coll_gbps", ("collective",))
    assert r["entries"] == 1 and r["unidentified"].startswith("entries") and r["value"] == 0.0
    assert ftar.cost_get()["coll_gbps"] == 0.0
    assert ftar.cost_get()["peer_write_gbps"] == pytest.approx(70.0, rel=0.02)   # left on the fitted constants


def test_refit_with_too_few_points_keeps_the_priors(model_defaults):
    """Fewer entries than free constants + 2: nothing is fitted, every free constant is flagged and keeps
    its prior (the value set when the refit started)."""
    import bench
    ftar = model_defaults
    ftar.cost_set(alpha_us=33.0, link_gbps=44.0, issue_us=22.0)
    prior = ftar.cost_get()
    one = [{"form": "direct", "topology": "8", "chunk_bytes": 1 << 20, "ms": 5.0, "check": "ok"}] * 3
    fit = bench.refit_cost_model(ftar, one, 8, 1 << 30)
    assert set(fit["unidentified"]) == {"alpha_us", "link_gbps", "issue_us"}
    assert all(v.startswith("entries") for v in fit["unidentified"].values())
    assert fit["prior"] == {"alpha_us": 33.0, "link_gbps": 44.0, "issue_us": 22.0}
    assert ftar.cost_get() == pytest.approx(prior)
    assert bench.refit_cost_model(ftar, [], 8, 1 << 30) is None
    assert bench.refit_form_rate(ftar, [], 8, 1 << 30, "coll_gbps", ("collective",)) is None


def test_refit_flags_a_flat_direction_and_keeps_its_prior(model_defaults):
    """Issue held at its measured value (as bench.py does), and every piece so small that the link term is
    a rounding error next to alpha: the predictions do not depend on link, so it is flagged "flat" and keeps
    its prior; alpha is fitted."""
    import bench
    ftar = model_defaults
    world, bucket = 8, 1 << 30
    ftar.cost_set(alpha_us=5000.0, link_gbps=60.0, issue_us=25.0)
    sweep = [{"topology": t, "form": "direct", "chunk_bytes": c, "check": "ok",
              "ms": bench.predict_ms(ftar, t, "direct", c, world, bucket)}
             for t in ("8", "2,4", "ring") for c in (256 << 10, 1 << 20)]
    ftar.cost_set(alpha_us=20.0, link_gbps=54.0, issue_us=25.0)   # the priors
    fit = bench.refit_cost_model(ftar, sweep, world, bucket, fixed={"issue_us": 25.0})
    assert fit["unidentified"] == {"link_gbps": "flat"} and fit["prior"] == {"link_gbps": 54.0}
    assert fit["params"]["link_gbps"] == 54.0 and ftar.cost_get()["link_gbps"] == pytest.approx(54.0)
    assert fit["params"]["alpha_us"] == pytest.approx(5000.0, rel=0.02)


def test_refit_flags_confounded_constants(model_defaults):
    """Every piece host-issue bound and issue left free: "each piece costs 3 ms" is explained as well by
    alpha as by issue (and link then does not matter), so no constant is pinned -- all three keep their
    priors instead of a self-consistent but wrong alpha = 3 ms."""
    import bench
    ftar = model_defaults
    world, bucket = 8, 1 << 30
    ftar.cost_set(alpha_us=35.0, link_gbps=60.0, issue_us=3000.0)
    sweep = [{"topology": t, "form": "direct", "chunk_bytes": c, "check": "ok",
              "ms": bench.predict_ms(ftar, t, "direct", c, world, bucket)}
             for t in ("8", "2,4", "ring") for c in (256 << 10, 1 << 20)]
    ftar.cost_set(alpha_us=20.0, link_gbps=54.0, issue_us=25.0)
    fit = bench.refit_cost_model(ftar, sweep, world, bucket)
    assert set(fit["unidentified"]) == {"alpha_us", "link_gbps", "issue_us"}
    assert "confounded" in fit["unidentified"].values()
    assert (fit["params"]["alpha_us"], fit["params"]["link_gbps"], fit["params"]["issue_us"]) == (20.0, 54.0, 25.0)


def test_refit_flags_a_constant_on_its_search_bound(model_defaults):
    """Timings no link rate in the search box explains (here: far slower than the slowest link) drive link
    onto its lower bound: flagged "bound", the prior kept -- the loopback rehearsal's link = 0.5 GB/s of
    round 4 would now read that way."""
    import bench
    ftar = model_defaults
    world, bucket = 8, 1 << 30
    ftar.cost_set(alpha_us=20.0, link_gbps=0.01, issue_us=25.0)   # 10 MB/s per link
    sweep = [{"topology": t, "form": f, "chunk_bytes": c, "check": "ok",
              "ms": bench.predict_ms(ftar, t, f, c, world, bucket)}
             for t in ("8", "2,4") for f in ("direct", "stages") for c in (4 << 20, 64 << 20)]
    ftar.cost_set(alpha_us=20.0, link_gbps=54.0, issue_us=25.0)
    fit = bench.refit_cost_model(ftar, sweep, world, bucket, fixed={"issue_us": 25.0})
    assert fit["unidentified"].get("link_gbps") == "bound"
    assert fit["params"]["link_gbps"] == 54.0


def test_form_labels_say_what_moved():
    """Every N > 1 line names its form in words: the one-round ring is a gather plus a
    fold in the ring's order, the staged ring the reference's own steps."""
    import bench
    assert bench.form_label("ring", "direct") == "direct (gather + ring-order fold)"
    assert bench.form_label("1", "direct") == "direct (gather + ring-order fold)"
    assert bench.form_label("ring", "stages") == "stages (reference ring steps)"
    assert bench.form_label("8", "direct") == "direct (gather + tree-order fold)"
    assert bench.form_label("2,4", "stages") == "stages (reference tree stages)"
    assert bench.form_label("8", "collective").startswith("collective (gather + tree-order fold")
    assert bench.form_label("8", "peer-read-reg:plain") == \
        "peer-read (IPC loads over xGMI + tree-order fold) on registered buffers [plain]"
    assert bench.form_label("ring", "direct:ncclreg") == "direct (gather + ring-order fold) [ncclreg]"


def test_c4_ring_item_labels_each_rccl_form(model_defaults):
    import bench
    bucket = 1 << 30
    sweep = [{"topology": "ring", "form": "direct", "chunk_bytes": c, "ms": ms, "check": "ok"}
             for c, ms in ((4 << 20, 9.0), (64 << 20, 7.0))]
    sweep += [{"topology": "ring", "form": "stages", "chunk_bytes": 16 << 20, "ms": 40.0, "check": "ok"},
              {"topology": "8", "form": "direct", "chunk_bytes": 64 << 20, "ms": 6.0, "check": "ok"},
              {"topology": "ring", "form": "direct", "chunk_bytes": 1 << 20, "ms": 1.0, "check": "MISMATCH (x)"}]
    out = bench.c4_ring_by_form(sweep, 8, 8, bucket, lambda r: bench.links_driven(8, r["topology"], r["form"]))
    assert set(out) == {"direct", "stages"}
    assert out["direct"]["form_label"] == "direct (gather + ring-order fold)" and out["direct"]["judged"]
    assert out["direct"]["ms"] == 7.0 and out["direct"]["pieces_swept"] == [1 << 20, 4 << 20, 64 << 20]
    assert out["stages"]["form_label"] == "stages (reference ring steps)" and not out["stages"]["judged"]
    assert out["stages"]["roofline"]["peak"] == pytest.approx(76.8) and out["direct"]["roofline"]["peak"] == pytest.approx(7 * 76.8)
    best = bench.rccl_p2p_best(sweep, 8, 8, bucket, lambda r: bench.links_driven(8, r["topology"], r["form"]))
    assert best["form_label"] == "direct (gather + tree-order fold)"


def _round4_loopback_line():
    import json
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "profiles", "r04", "loopback", "dist8_loopback_1GiB.json")
    with open(path) as f:
        for line in f:
            if line.startswith("{"):
                return json.loads(line)
    raise AssertionError("no bench line in " + path)


def test_refit_of_the_round4_loopback_sweep_leaves_no_constant_on_a_bound(model_defaults):
    """Round 4's 8-rank RCCL loopback rehearsal (1 GiB per rank, sockets) re-fitted its constants onto
    link = 0.5 GB/s (the search floor) and peer_write = 4,981 GB/s from 2 entries.  The same sweep through
    today's refit: link is flagged "bound" and keeps the probe's value, the 2-entry peer rates and the
    collective rate on its floor keep theirs, and no returned constant sits on a search bound."""
    import bench
    ftar = model_defaults
    d = _round4_loopback_line()
    cm = d["cost_model"]
    ftar.cost_set(**cm["constants_probe"])
    p2p = bench.refit_cost_model(ftar, d["sweep"], 8, 1 << 30, fixed={"issue_us": cm["issue_us_from_enqueue"]})
    assert p2p["unidentified"] == {"link_gbps": "bound"}
    assert p2p["params"]["link_gbps"] == pytest.approx(cm["constants_probe"]["link_gbps"])
    assert p2p["rms_log_err"] < p2p["rms_log_err_prior"]
    for k, lo, hi in (("alpha_us", 0.1, 1e5), ("link_gbps", 0.5, 5e3)):
        assert lo * 1.01 < p2p["params"][k] < hi / 1.01, (k, p2p["params"][k])
    rates = {f: bench.refit_form_rate(ftar, d["sweep"], 8, 1 << 30, f, forms)
             for f, forms in (("peer_read_gbps", ("peer-read", "peer-read-reg")),
                              ("peer_write_gbps", ("peer-write", "peer-write-reg")),
                              ("coll_gbps", ("collective",)))}
    assert rates["peer_write_gbps"]["unidentified"].startswith("entries")
    assert rates["peer_write_gbps"]["value"] == pytest.approx(cm["constants_probe"]["peer_write_gbps"])
    assert rates["coll_gbps"]["unidentified"] == "bound" and rates["coll_gbps"]["value"] == 0.0
    for r in rates.values():
        assert r["value"] == 0.0 or 1.01 < r["value"] < 5000 / 1.01


def test_cpu_baseline_states_its_regime():
    """the CPU leg says which buffers it ran on and which statistic `value` is -- the warm leg
    (the same buffers every call, the reference harness's way) as the best call, the median beside it, and a
    cold leg over 2 rotated buffer sets (the GPU line's regime) -- whichever of the reference build
    (oracle/_ref/ref_golden) or the port ran."""
    import bench
    d = bench.cpu_baseline(2, 1 << 18, 1.0)
    assert d["unit"] == "GB/s" and d["value"] > 0 and d["kind"] in ("reference", "port")
    assert d["buffers"] == "same every call (warm)" and d["statistic"] == "best"
    assert 0 < d["median"] <= d["value"] * 1.0001
    if d["kind"] == "reference":
        r = d["rotated"]
        assert r["buffers"].startswith("2 disjoint sets") and 0 < r["median"] <= r["best"] * 1.0001 and r["samples"] > 0
        assert d["cores"] == 14   # PARALLEL_THREAD, mpi_mod.hpp:820


class _FakeTime:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def test_n_gt_1_stage_order_and_budget_with_synthetic_stage_times():
    """the N > 1 line's required stages (c4_ring's sweep entries, C5 per width, the host-memory
    rate, the model's refit, the re-timed headline) run first and inside FTAR_BENCH_BUDGET_S even when the
    optional ones are slow (the loopback rehearsal's probe took 40 s); bounded stages get only the time the
    later required stages leave; the extras are skipped, not the required stages."""
    import bench
    req = [n for n, r, _ in bench.DIST_STAGES if r]
    assert req == ["sweep core", "C5 bf16", "host e2e", "cost model", "headline"]
    names = [n for n, _, _ in bench.DIST_STAGES]
    assert names.index("sweep core") < names.index("xgmi probe") < names.index("C5 bf16") < names.index("sweep rest")
    for budget, times in ((300.0, {}), (300.0, {"xgmi probe": 40.0, "sweep rest": 1e9, "reference cpu/mpi": 60}),
                          (150.0, {"sweep core": 25.0, "C5 bf16": 35.0, "host e2e": 20.0})):
        clk = _FakeTime()
        clock = bench.StageClock(budget, 0.0, now=clk)
        used = {}

        def stage(name):
            def fn(limit):
                want = times.get(name, 3.0)
                took = min(want, max(0.0, limit)) if name in ("sweep core", "sweep rest", "xgmi probe") else want
                used[name] = (took, limit)
                clk.t += took
            return fn
        ran = bench.run_stage_plan(clock, {n: stage(n) for n in names})
        assert [n for n in ran if n in req] == req, (budget, ran)       # every required stage, in order
        assert clk.t <= budget - clock.margin + 1e-9, (budget, clk.t, used)
        if times.get("sweep rest") == 1e9:                              # an endless sweep is cut at its limit
            assert used["sweep rest"][0] == used["sweep rest"][1]
            assert "reference cpu/mpi" not in ran and "reference cpu/mpi" in clock.skipped
    # a run that reaches the probe with 60 s of its 300 left: the probe is skipped (C5, host e2e, the refit and
    # the headline need its time), the required stages all run, and what they leave goes to the sweep's rest
    clk = _FakeTime()
    clock = bench.StageClock(300.0, 0.0, now=clk)
    clk.t = 230.0
    ran = bench.run_stage_plan(clock, {n: (lambda lim: None) for n in names})
    assert "xgmi probe" not in ran and "xgmi probe" in clock.skipped and set(req) <= set(ran) and "sweep rest" in ran
    # a rehearsal's small budget scales the reserves down: at its start every stage still fits
    clock = bench.StageClock(100.0, 0.0, now=_FakeTime())
    assert bench.run_stage_plan(clock, {n: (lambda lim: None) for n in names}) == names
