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


def test_roofline_uses_probe_rate_and_falls_back_to_spec():
    import bench
    probe = {"read_one_peer": [60.0, 62.0], "read_all_peers": [400.0, 410.0], "write_one_peer": [50.0, 51.0],
             "write_all_peers": [350.0, 360.0], "note": "x"}
    rate = bench.link_rate_from_probe(probe, 8)
    assert rate == pytest.approx(60.0)   # the slowest rank's best per-link mode: one peer beats 400/7
    bucket = 1 << 30
    ms = bucket * 2 * 7 / 8 / (7 * 50.0 * 1e9) * 1e3   # busBW 50 GB/s per link
    r = bench.allreduce_roofline(8, 8, bucket, ms, 7, rate)
    assert "ftar_xgmi_probe" in r["note"] and r["peak"] == pytest.approx(420.0, rel=1e-3)
    assert r["frac"] == pytest.approx(50.0 / 60.0, abs=1e-4)
    ms2 = bucket * 2 * 7 / 8 / (7 * 70.0 * 1e9) * 1e3  # beats the probe's rate: spec denominator
    r2 = bench.allreduce_roofline(8, 8, bucket, ms2, 7, rate)
    assert "spec" in r2["note"] and 0 < r2["frac"] <= 1
    assert bench.link_rate_from_probe(None, 8) is None
    assert bench.link_rate_from_probe({"error": "x"}, 8) is None
    assert bench.link_rate_from_probe(probe, 1) is None


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
