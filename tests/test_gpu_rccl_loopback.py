"""RCCL point-to-point between ranks, on the box's one GPU (tests/rccl_loopback_child.py under torchrun).

The product's RcclTransport (ncclSend/ncclRecv in ncclGroupStart/End; the replacement of the reference's
handle_send/handle_recv, mpi_mod.hpp:1254-1305) has otherwise only ever run on a 1-rank communicator here,
because RCCL refuses two ranks of one communicator on the same device.  Giving every rank its own
NCCL_HOSTID makes RCCL treat them as separate nodes, so its socket transport over the loopback interface
carries the bytes: every golden case of the world size (per-rank reference bits) in the direct, staged and
collective forms, plus ragged 2^20 buckets against the oracle through device and host buffers.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_loopback(world, env_extra=None, timeout=170):
    """(completed process, every rank's result dict, by rank); each rank writes its own result file"""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(HERE, "rccl_loopback_child.py")]
    with tempfile.TemporaryDirectory() as out:
        env = dict(os.environ, FTAR_LOOPBACK_OUT=out, **(env_extra or {}))
        p = subprocess.run(cmd, cwd=os.path.dirname(HERE), env=env, capture_output=True, text=True, timeout=timeout)
        res = []
        for r in range(world):
            path = os.path.join(out, f"rank{r}.json")
            if os.path.exists(path):
                with open(path) as f:
                    res.append(json.load(f))
    return p, res


WIDE = pytest.mark.wide


@pytest.mark.parametrize("world", [2, pytest.param(3, marks=WIDE), pytest.param(4, marks=WIDE), 8,
                                   pytest.param(12, marks=WIDE)])
def test_rccl_p2p_between_ranks_matches_reference(world):
    # P = 8: the direct and staged forms; the collective all-gather runs every golden case at P = 2 (and at
    # P = 8 with FTAR_RUN_WIDE=1), and at full size in-process (test_gpu_full_size.py)
    forms = "direct,stages" if world == 8 and os.environ.get("FTAR_RUN_WIDE") != "1" else None
    p, res = run_loopback(world, {"FTAR_LOOPBACK_FORMS": forms} if forms else None)
    assert p.returncode == 0 and len(res) == world, (p.returncode, p.stdout[-3000:], p.stderr[-4000:])
    for r in res:
        assert not r["fail"], r["fail"][:10]
        assert r["golden"] > 0 and r["oracle"] == 4 and r["nccl_allreduce"] == "ok", r
    assert len({r["golden"] for r in res}) == 1


@pytest.mark.parametrize("world", [2, pytest.param(4, marks=WIDE)])   # one default case
def test_rccl_p2p_allreduce_captures_into_a_hip_graph(world):
    """One rank per process over RCCL (the product's process model), P > 1, under torch.cuda.graph: the
    ring and the width-P tree in the direct form and the ring in the reference's staged rounds, each captured
    once and replayed on three new input sets, bit-exact against the oracle on every rank.  torch's bundled HIP
    7.0 runtime died in hipStreamEndCapture on the forked comm/reduce streams (profiles/r03/loopback/
    capture_py_relaxed.log), so on runtimes before 7.2 a captured call issues serially on its stream
    (serial_capture, engine.cpp); from C++ on 7.2 the forked form captures
    (test_harness_rccl_allreduce_captured_in_a_hip_graph)."""
    p, res = run_loopback(world, {"FTAR_LOOPBACK_MODE": "capture"})
    assert p.returncode == 0 and len(res) == world, (p.returncode, p.stdout[-3000:], p.stderr[-4000:])
    for r in res:
        assert not r["fail"] and r["captured"] == 3, r


@pytest.mark.parametrize("world", [pytest.param(w, marks=WIDE) if w != 5 else w for w in (2, 3, 5, 6, 7, 8)])
def test_rccl_p2p_random_soak(world):
    """Seeded random cases of the world size over RCCL, each with its own piece size, data-movement form and
    device, pinned or pageable host buffers, bit-exact against the oracle (lonely layouts at P = 5, 6, 7 and 8)."""
    p, res = run_loopback(world, {"FTAR_LOOPBACK_MODE": "soak"})
    assert p.returncode == 0 and len(res) == world, (p.returncode, p.stdout[-3000:], p.stderr[-4000:])
    for r in res:
        assert not r["fail"] and r["soak"] == 40, r


@pytest.mark.parametrize("world,dtype", [pytest.param(2, "bf16", marks=WIDE), (2, "f32"),   # one default
                                         pytest.param(4, "f32", marks=WIDE), pytest.param(4, "bf16", marks=WIDE)])
def test_ddp_comm_hook_over_rccl(world, dtype):
    """torch DistributedDataParallel with ftar as the gradient AllReduce (ftar.ddp.allreduce_hook, one rank
    per process over RCCL) against DDP's own AllReduce on the same model and batches, fp32 and bf16 models:
    bit-identical gradients at P = 2, close at P = 4, every rank with the same parameters after 3 SGD steps."""
    p, res = run_loopback(world, {"FTAR_LOOPBACK_MODE": "ddp", "FTAR_LOOPBACK_DDP_DTYPE": dtype})
    assert p.returncode == 0 and len(res) == world, (p.returncode, p.stdout[-3000:], p.stderr[-4000:])
    for r in res:
        assert not r["fail"] and r["ddp_hook_calls"] >= 3, r   # at least one bucket per step


@pytest.mark.parametrize("world", [2, pytest.param(3, marks=WIDE)])
def test_peer_write_waits_for_every_copy_out(world):
    """Consecutive peer-write calls over RCCL with the last rank's copy-out enqueued 150 ms late: a peer that
    returned early would scatter its next call into that rank's exchange buffer before the copy-out read it
    (found by tools/asan/engine_stress rccl, profiles/r04/asan_engine_stress_rccl_*.log)."""
    env = {"FTAR_LOOPBACK_MODE": "write_race", "FTAR_LOOPBACK_LATE_RANK": str(world - 1)}
    p, res = run_loopback(world, env)
    assert p.returncode == 0 and len(res) == world, (p.returncode, p.stdout[-3000:], p.stderr[-4000:])
    for r in res:
        assert not r["fail"] and r["write_race"] == 8, r


def test_first_contact_with_a_missing_peer_times_out():
    """the first call on an RCCL communicator runs the settings agreement and connects the peers on
    a helper thread with a deadline, so a peer that never calls fails the call with FTAR_ERR_TIMEOUT
    (FTAR_FIRST_CONTACT_TIMEOUT_S) instead of hanging it; later calls fail at once; destroy aborts RCCL."""
    p, res = run_loopback(2, {"FTAR_LOOPBACK_MODE": "first_contact", "FTAR_FIRST_CONTACT_TIMEOUT_S": "4"},
                          timeout=120)
    assert p.returncode == 0 and len(res) == 2, (p.returncode, p.stdout[-3000:], p.stderr[-4000:])
    r0 = res[0]
    assert not r0["fail"], r0
    assert r0["first_call"]["status"] == 7 and "first contact" in r0["first_call"]["error"], r0
    assert r0["second_call"]["status"] == 7, r0


def test_rccl_p2p_baseline_c4_c5_full_size():
    """BASELINE configs[3] (8 ranks x 2^28 fp32, the ring, direct and staged, default pieces and pieces that
    divide no block) and configs[4] (8 ranks x 2^29 bf16, the width-8 tree) over RCCL between 8 processes,
    random inputs per rank: every rank's WHOLE output bit for bit against the reference's fold of all P inputs
    (tests/whole_fold.py, each rank regenerating every rank's input from its seed)."""
    p, res = run_loopback(8, {"FTAR_LOOPBACK_MODE": "full"})
    assert p.returncode == 0 and len(res) == 8, (p.returncode, p.stdout[-3000:], p.stderr[-4000:])
    for r in res:
        assert not r["fail"] and len(r["full"]) == (5 if os.environ.get("FTAR_RUN_WIDE") == "1" else 3), r
