"""The engine stress driver (allreduce-over-mpi_amd/harness/engine_stress.cpp, built as lib/ftar_engine_stress)
on the production library: seeded random calls with every result checked against the exact sum of
small-integer inputs -- in-process groups created and destroyed (P = 2..8; some calls captured into HIP graphs
and replayed), and P processes of one RCCL communicator or of the host-bootstrapped transport each (loopback
sockets; two communicators in turn); per-call knobs and a steered execution model.  The
same source built against a host-sanitized libftar.so is tools/asan/ (profiles/r04/asan_*.log); the RCCL mode
found the peer-write race that test_peer_write_waits_for_every_copy_out now pins."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "allreduce-over-mpi_amd", "lib", "ftar_engine_stress")


def _run(args, timeout, **extra_env):
    env = dict(os.environ, NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", **extra_env)
    p = subprocess.run([EXE] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout, env=env)
    return p


@pytest.mark.parametrize("calls", [500, pytest.param(1500, marks=pytest.mark.wide)])
def test_in_process_groups(calls):
    # 500 calls of seed 5 bring up and tear down at least 8 groups (the bar round 5 lowered to 3),
    # so the in-process transport's pooled threads, batched events and broken-group state see several
    # lifecycles in the default suite
    p = _run([calls, 5], 240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    stats = json.loads(p.stdout.strip().splitlines()[-1])
    assert stats["checked"] == stats["calls"] >= calls and stats["groups"] >= 8 and stats["captured"] > 0, stats


def test_in_process_groups_multi_segment_receives():
    """The in-process transport's batched receive (one multi-segment copy per stream and flush: the path
    receives from other devices take on a multi-GPU box) on every receive, forced by FTAR_LOCAL_COPY=gather
    on this one-GPU box: the same random calls, every result checked, captures included."""
    p = _run([120, 7], 240, FTAR_LOCAL_COPY="gather")
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    stats = json.loads(p.stdout.strip().splitlines()[-1])
    assert stats["checked"] == stats["calls"] >= 120 and stats["captured"] > 0, stats


@pytest.mark.parametrize("mode,P,calls,seed", [pytest.param("rccl", 4, 40, 41, marks=pytest.mark.wide), ("rccl", 8, 10, 12),
                                               ("host", 4, 30, 43), pytest.param("host", 4, 60, 43, marks=pytest.mark.wide)])
def test_processes(mode, P, calls, seed):
    p = _run([mode, P, calls, seed, 2], 240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    ranks = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{"rank"')]
    assert len(ranks) == P and all(r["checked"] == 2 * calls for r in ranks), ranks
    assert f"{mode}: P={P}" in p.stdout and p.stdout.rstrip().endswith("ok"), p.stdout[-500:]
