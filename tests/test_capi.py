"""C-ABI boundary checks that need no GPU: the library loads, exports every
entry point include/ftar.h declares, and its host logic (topology parsing,
cost model, error reporting) behaves like the reference's get_stages."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "ftar.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ftar_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import ftar
    names = header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(ftar.lib(), n)]
    assert not missing, missing


def test_kernel_variants_live_in_the_bench_library_only():
    """The A/B kernel variants and kernel test hooks are in libftar_bench.so (tools/kbench*.py, the bf16
    conversion test), not in the product library, which keeps only what the engine dispatches and the
    ftar_debug_last_kernel hook bench.py ties its PMC traffic to."""
    import ftar
    moved = ("ftar_debug_reduce_variant", "ftar_debug_reduce_nested_lds", "ftar_debug_bf16_cvt_check")
    assert not [n for n in moved if hasattr(ftar.lib(), n)]
    assert all(hasattr(ftar.bench_lib(), n) for n in moved)
    assert hasattr(ftar.lib(), "ftar_debug_last_kernel")


def test_version_and_status_strings():
    import ftar
    assert "gfx950" in ftar.version()
    assert ftar.lib().ftar_status_string(3) == b"invalid FT_TOPO/FT_LONELY"


@pytest.mark.parametrize("dt,size", [("u8", 1), ("i8", 1), ("u16", 2), ("i16", 2), ("i32", 4), ("i64", 8),
                                     ("f32", 4), ("f64", 8), ("bool", 1), ("bf16", 2)])
def test_dtype_sizes(dt, size):
    import ftar
    assert ftar.dtype_size(dt) == size


@pytest.mark.parametrize("spec,lonely,P,expect", [
    ("1", "", 8, "ring"), ("2,1", "", 8, "ring"), ("8", "", 8, "8"), ("2,4", "", 8, "2,4"), ("2,2,2", "", 8, "2,2,2"),
    ("2,2", "1", 5, "2,2+1"), ("3,2", "2", 8, "3,2+2"), ("2,4,", "", 8, "2,4"),
])
def test_topo_parse_valid(spec, lonely, P, expect):
    import ftar
    assert str(ftar.topo_parse(spec, lonely, P)) == expect


@pytest.mark.parametrize("spec,lonely,P", [
    ("3", "", 4),        # product != P (mpi_mod.hpp:1471)
    ("4", "1", 5),       # lonely needs >= 2 stages
    (None, None, 4),     # unset FT_TOPO with P > 1 (reference: exit(1))
    ("", None, 4),
    ("2,x", None, 4),
    ("3", None, 1),      # checked before the P <= 1 copy (mpi_mod.hpp:1732-1746)
    (None, "1", 1),      # lonely ranks with FT_TOPO unset: product 1 + 1 != 1
    ("2", "1", 1),
])
def test_topo_parse_invalid(spec, lonely, P):
    import ftar
    with pytest.raises(ftar.FtarError):
        ftar.topo_parse(spec, lonely, P)


def test_topo_parse_single_rank_defaults():
    import ftar
    t = ftar.topo_parse(None, None, 1)
    assert t.nstages == 1


def test_cost_model_prefers_all_links_on_8_gpus():
    """One stage of width 8 drives all 7 xGMI links at once; a ring drives one."""
    import ftar
    big = 1 << 30
    t = ftar.topo_choose(8, big)
    assert str(t) == "8"
    # direct forms (default): the ring and multi-stage trees are one round each way, like tree(P)
    assert ftar.topo_cost("ring", 8, big) == ftar.topo_cost("8", 8, big)
    assert ftar.topo_cost("2,4", 8, big) == ftar.topo_cost("8", 8, big)
    assert ftar.topo_cost("2,2,2", 8, big) == ftar.topo_cost("8", 8, big)
    # lonely layouts and trees deeper than 4 stages keep the staged cost
    assert ftar.topo_cost("2,2,2,2,2", 32, big) > ftar.topo_cost("32", 32, big)
    assert ftar.topo_cost(ftar.topo("2,2", 1), 5, big) > ftar.topo_cost("5", 5, big)
    assert str(ftar.topo_choose(2, big)) == "2"          # ties keep the tree
    # every candidate is a valid factorization of P
    for P in range(2, 17):
        t = ftar.topo_choose(P, 1 << 20)
        if not t.ring:
            prod = 1
            for w in t.widths:
                prod *= w
            assert prod == P


def test_topo_from_env(monkeypatch):
    import ftar
    monkeypatch.setenv("FT_TOPO", "2,2")
    monkeypatch.setenv("FT_LONELY", "1")
    assert str(ftar.topo_from_env(5, 1 << 20)) == "2,2+1"
    monkeypatch.setenv("FT_TOPO", "3")
    with pytest.raises(ftar.FtarError):
        ftar.topo_from_env(5, 1 << 20)
    monkeypatch.delenv("FT_TOPO")
    with pytest.raises(ftar.FtarError):   # FT_LONELY alone is not "unset": reported, not the cost model
        ftar.topo_from_env(5, 1 << 20)
    monkeypatch.setenv("FT_LONELY", "0")  # ... but "0" is
    assert str(ftar.topo_from_env(8, 1 << 30)) == "8"
    monkeypatch.setenv("FT_TOPO", "1")    # the ring at any P, FT_LONELY ignored (mpi_mod.hpp:1461-1464)
    monkeypatch.setenv("FT_LONELY", "3")
    assert str(ftar.topo_from_env(8, 1 << 30)) == "ring"
    monkeypatch.delenv("FT_TOPO")
    monkeypatch.delenv("FT_LONELY")
    assert str(ftar.topo_from_env(8, 1 << 30)) == "8"


def test_reduce_argument_errors_without_gpu():
    """Argument validation happens before any device work."""
    import ftar
    with pytest.raises(ftar.FtarError):
        ftar.reduce([], 1234, 10)                      # k = 0
    with pytest.raises(ftar.FtarError):
        ftar.reduce([1024, 2048], 4096, 10, "f32", "band")   # BAND on float: unsupported (mpi_mod.hpp:1397)


def test_cost_model_candidates_match_reference_getwidth():
    """The candidate set is the reference's getWidth(P) (tests/golden/getwidth.json, dumped from
    cost_model/GetWidth.h), its [1,P]/[P,1] entries being the ring, plus the single-stage
    width-P tree that getWidth never lists although FT_TOPO=P is valid (mpi_mod.hpp:1440-1468)
    and is the all-links schedule on an MI355X node."""
    import json
    import ftar
    with open(os.path.join(ROOT, "tests", "golden", "getwidth.json")) as f:
        ref = json.load(f)
    for P in range(2, 25):
        exp = []
        for w in ref[str(P)]:
            key = "ring" if 1 in w else ",".join(map(str, w))
            if key not in exp:
                exp.append(key)
                if key == "ring":
                    exp.append(str(P))
        got = [str(t) for t in ftar.topo_candidates(P)]
        assert got == exp, (P, got, exp)


def test_mpi_library_exports_ftar_mpi_h():
    """libftar_mpi.so (built where MPICH is present) exports every include/ftar_mpi.h entry point."""
    import ctypes
    lib_path = os.path.join(ROOT, "allreduce-over-mpi_amd", "lib", "libftar_mpi.so")
    if not os.path.exists(lib_path):
        pytest.skip("libftar_mpi.so not built (no MPI here)")
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "ftar_mpi.h")).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b((?:MPI_Allreduce_FT\w*|ftar_mpi_\w+))\s*\(", src)))
    assert "MPI_Allreduce_FT" in names and len(names) >= 5
    import ftar  # noqa: F401  (loads libftar.so first, as the loader would)
    lib = ctypes.CDLL(lib_path)
    assert all(hasattr(lib, n) for n in names), names


def test_header_is_plain_c99(tmp_path):
    """include/ftar.h compiles as C99 and links against libftar.so (the FFI boundary needs no C++)."""
    import subprocess
    import ftar  # noqa: F401  (library is built)
    lib_dir = os.path.join(ROOT, "allreduce-over-mpi_amd", "lib")
    exe = str(tmp_path / "abi_c99")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-pedantic", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_c99.c"), "-o", exe, "-L", lib_dir, "-lftar",
                    f"-Wl,-rpath,{lib_dir}"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, (out.returncode, out.stdout, out.stderr)
    assert "c99 ok" in out.stdout


def _costmodel_golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "costmodel.jsonl")) as f:
        return [json.loads(line) for line in f]


def test_reference_cost_model_matches_reference_output():
    """The reference's cost model restated in libftar (ftar_cost_reference, ftar_topo_choose_reference) against
    what the reference itself prints (tests/golden/costmodel.jsonl, oracle/ref_costmodel.cpp around the
    unmodified cost_model/CostModel.h + GetWidth.h): every candidate list in getWidth's order, every
    candidate's score to the last bit (printed at 17 digits), and the argmin, for P = 2..48, 60, 64, 72, 96,
    128, 256, 512 and chunk 100 (cost_model/main.cpp:23), 1 and 1000."""
    import ftar
    rows = _costmodel_golden()
    assert len(rows) >= 150
    for d in rows:
        P, ch = d["P"], d["chunk"]
        cands = ftar.reference_candidates(P)
        assert cands == d["candidates"], P
        for w, c in zip(cands, d["costs"]):
            assert ftar.cost_reference(w, P, ch) == float(c), (P, ch, w)
        t, idx = ftar.topo_choose_reference(P, ch)
        assert "*".join(map(str, cands[idx])) == d["chosen"], (P, ch, cands[idx], d["chosen"])
        assert ftar.cost_reference(cands[idx], P, ch) == float(d["cost"])
        want = "ring" if 1 in cands[idx] else ",".join(map(str, cands[idx]))
        assert str(t) == want, (P, str(t), want)


def test_reference_cost_model_picks_the_ring_at_2_4_8():
    """with chunk 100 the reference's model chooses 1*2, 1*4, 1*8 -- the ring."""
    import ftar
    for P in (2, 4, 8):
        t, idx = ftar.topo_choose_reference(P)
        assert str(t) == "ring" and ftar.reference_candidates(P)[idx] == [1, P]


def test_cost_model_selector(monkeypatch):
    """FTAR_COST_MODEL=reference makes ftar_topo_choose (and so FT_TOPO-less communicators) take the
    reference's argmin; the default stays the xGMI model (width 8 at P = 8); anything else is refused."""
    import ftar
    monkeypatch.delenv("FT_TOPO", raising=False)
    monkeypatch.setenv("FTAR_COST_MODEL", "reference")
    assert str(ftar.topo_choose(8, 1 << 30)) == "ring"
    monkeypatch.setenv("FTAR_COST_REF_CHUNK", "100")
    assert str(ftar.topo_choose(12, 1 << 30)) == "2,6"
    monkeypatch.setenv("FTAR_COST_MODEL", "xgmi")
    assert str(ftar.topo_choose(8, 1 << 30)) == "8"
    monkeypatch.setenv("FTAR_COST_MODEL", "bogus")
    with pytest.raises(ftar.FtarError):
        ftar.topo_choose(8, 1 << 30)


def test_cost_params_set_and_restore(monkeypatch):
    """ftar_cost_set_params (bench.py fits it from the xGMI probe) changes the xGMI model's constants and
    its costs; 0 restores the defaults; the environment still overrides."""
    import ftar
    for k in ("FTAR_COST_ALPHA_US", "FTAR_COST_LINK_GBPS", "FTAR_COST_HBM_GBPS"):
        monkeypatch.delenv(k, raising=False)
    base = ftar.cost_params()
    c0 = ftar.topo_cost("8", 8, 1 << 30)
    try:
        p = ftar.cost_params(alpha_us=5.0, link_gbps=2 * base["link_GBps"])
        assert p["alpha_us"] == pytest.approx(5.0) and p["link_GBps"] == pytest.approx(2 * base["link_GBps"])
        assert ftar.topo_cost("8", 8, 1 << 30) < c0
        monkeypatch.setenv("FTAR_COST_LINK_GBPS", "10")
        assert ftar.cost_params()["link_GBps"] == pytest.approx(10.0)
    finally:
        ftar.cost_params(0.0, 0.0, 0.0)
    monkeypatch.delenv("FTAR_COST_LINK_GBPS")
    assert ftar.cost_params() == base and ftar.topo_cost("8", 8, 1 << 30) == c0


def test_mpi_dropin_type_and_op_mapping(tmp_path):
    """libftar_mpi.so's MPI datatype/op mapping against the reference's handle_reduce dispatch list
    (mpi_mod.hpp:1363-1412), its error classes, and MPI_Allreduce_FT's P <= 1 copy (mpi_mod.hpp:1739) for
    every type, from a C program under mpiexec -n 1 (no GPU)."""
    import subprocess
    lib_dir = os.path.join(ROOT, "allreduce-over-mpi_amd", "lib")
    if not (os.path.exists(os.path.join(lib_dir, "libftar_mpi.so")) and os.path.exists("/opt/conda/bin/mpiexec")):
        pytest.skip("libftar_mpi.so or MPICH not available")
    exe = str(tmp_path / "mpi_dtypes")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-I", "/opt/conda/include",
                    os.path.join(ROOT, "tests", "c", "mpi_dtypes.c"), "-o", exe, "-L", lib_dir, "-lftar_mpi", "-lftar",
                    f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath-link,/usr/lib/x86_64-linux-gnu", "-Wl,-rpath-link,/opt/rocm/lib",
                    "/opt/conda/lib/libmpi.so", "-Wl,-rpath,/opt/conda/lib"], check=True)
    out = subprocess.run(["/opt/conda/bin/mpiexec", "-n", "1", exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "mpi dtypes ok" in out.stdout, (out.returncode, out.stdout, out.stderr)


def test_stress_drivers_are_built_against_the_product_library():
    """build() makes the engine and MPI drop-in stress drivers (harness/engine_stress.cpp, harness/mpi_stress.cpp)
    next to libftar.so, linked to it (their GPU runs: tests/test_gpu_engine_stress.py, test_mpi_drop_in_random_calls)"""
    import subprocess
    lib = os.path.join(ROOT, "allreduce-over-mpi_amd", "lib")
    for exe in ("ftar_engine_stress", "ftar_mpi_stress"):
        path = os.path.join(lib, exe)
        if exe == "ftar_mpi_stress" and not os.path.exists("/opt/conda/include/mpi.h"):
            continue
        assert os.access(path, os.X_OK), path
        deps = subprocess.run(["ldd", path], capture_output=True, text=True).stdout
        assert "libftar.so" in deps and os.path.join(lib, "libftar.so") in deps, deps


def test_group_thread_pool_runs_every_rank_at_once():
    """The in-process group calls' host threads are pooled (engine_api.cpp RankPool): the ranks of a call
    meet in the transport, so every job of a call must start at once even while other callers' jobs hold
    workers.  Four caller threads, group sizes 1..8, each job waiting at a rendezvous of its call."""
    import ctypes
    import threading
    import ftar
    fn = ftar.lib().ftar_debug_rank_pool
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_int, ctypes.c_int]
    assert fn(0, 1) == -1
    got = {}

    def caller(i):
        got[i] = [(n, fn(n, 20)) for n in (8, 1, 3, 7, 2, 5)]
    th = [threading.Thread(target=caller, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert all(not t.is_alive() for t in th)
    assert all(done == 20 for runs in got.values() for _, done in runs), got
