"""bench.py's N > 1 path, end to end, on the box's one GPU: P ranks under torchrun share it, the communicator
is bootstrapped over gloo (--host-comm, or RCCL refusing the shared GPU and every rank falling back), and the
peer-direct forms move the data through IPC.  Everything the driver's 8-GPU run executes except the RCCL forms:
the timed default, the validated sweep with registration and tuning variants, the xGMI probe, phase timelines,
the 256 MiB (80 Mi elements > 2^26) and C5 line items, and the single JSON line."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(ranks, extra, env_extra=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--steps", "2", "--warmup", "1", "--elements", str(5 << 24), "--elements-c5", str(1 << 22)] + extra
    env = dict(os.environ, FTAR_BENCH_BUDGET_S="100", FTAR_BENCH_SWEEP_S="60")
    env.update(env_extra or {})
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and len(lines) == 1, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    return json.loads(lines[0])


@pytest.mark.parametrize("ranks,extra", [(2, ["--host-comm"]), pytest.param(4, ["--host-comm"], marks=pytest.mark.wide),
                                         (2, [])])
def test_bench_n_gt_1_rehearsal(ranks, extra):
    d = _bench(ranks, extra)
    assert d["n_gpus"] == ranks and d["check"] == "ok" and d["config"]["form"].startswith("peer-")
    assert "watchdog" not in d
    ok = [r for r in d["sweep"] if r.get("check") == "ok"]
    assert len(ok) >= 8 and not [r for r in d["sweep"] if r.get("check") == "MISMATCH"], d["sweep"]
    assert d["c5_bf16"]["check"] == "ok", d["c5_bf16"]
    assert "ms" in d["bucket_256MiB"], d["bucket_256MiB"]
    assert d["xgmi_probe_GBps"]["read_all_peers"][0] > 0
    assert set(d["stage_wall_s"]) >= {"init", "default", "sweep core", "headline", "C5 bf16", "host e2e"}, d["stage_wall_s"]
    assert "stages_skipped_for_budget" in d and d["budget_s"] > 0, d.get("stages_skipped_for_budget")
    if not extra:   # RCCL refused the shared GPU on every rank and every rank fell back
        assert "rccl_init_error" in d
        assert [e["rank"] for e in d["rccl_error_by_rank"]] == list(range(ranks)), d["rccl_error_by_rank"]


# the hang case (~24 s: the spinning wave holds the box until its preflight times out) runs with the wide
# rehearsals; the failing-call case of the same fallback stays in the default suite
@pytest.mark.parametrize("env_extra,why", [pytest.param({"FTAR_BENCH_PREFLIGHT_HANG": "1"}, "not complete",
                                                        marks=pytest.mark.wide),
                                           ({"FTAR_BENCH_FAIL_DEFAULT": "1"}, "FTAR_BENCH_FAIL_DEFAULT")])
def test_bench_rccl_failure_paths_at_world_size_one(env_extra, why):
    """The first-contact failure paths of the 8-GPU run, at world size 1 over a real RCCL communicator: an RCCL
    call that never completes or fails makes every rank fall back to the IPC peer forms; the line names every
    rank's error and the stage times, and rccl_p2p_best is absent because no RCCL configuration was measured.
    The hang is real: a spinning wave keeps the bench's stream from draining until the run ends,
    and the fallback runs on a fresh stream -- still blocked when the fallback's default was measured."""
    # the fallback's sweep is not what is tested here: a short budget (the spinning wave of the hang case
    # slows every later kernel until the run ends)
    d = _bench(1, ["--force-dist", "--no-cpu-baseline", "--no-c5", "--no-host"],
               dict(env_extra, FTAR_BENCH_PREFLIGHT_S="3", FTAR_BENCH_SWEEP_S="5"))
    assert d["check"] == "ok" and d["config"]["form"].startswith("peer-"), d["config"]
    assert why in d["rccl_init_error"], d["rccl_init_error"]
    assert len(d["rccl_error_by_rank"]) == 1 and why in d["rccl_error_by_rank"][0]["error"]
    assert "default" in d["stage_wall_s"] and d.get("rccl_p2p_best") is None
    if "FTAR_BENCH_PREFLIGHT_HANG" in env_extra:
        assert d["fallback_stream"] == {"fresh": True, "stuck_stream_still_blocked": True}, d.get("fallback_stream")


@pytest.mark.parametrize("ranks", [2, pytest.param(4, marks=pytest.mark.wide)])
def test_bench_n_gt_1_rehearsal_over_rccl(ranks, tmp_path):
    """The same N > 1 run with RCCL itself carrying the default configuration and every RCCL form of the sweep
    (--rccl-loopback: one NCCL_HOSTID per rank, ncclSend/ncclRecv over loopback sockets, the ranks sharing the
    box's GPU): no fallback is taken, the default configuration is RCCL p2p and validates, and rccl_p2p_best is
    in the line with a validated entry -- the fields the driver's 8-GPU run reports, produced by a real
    multi-rank RCCL communicator."""
    cost_file = str(tmp_path / "node.cost")
    d = _bench(ranks, ["--rccl-loopback", "--no-cpu-baseline", "--save-cost", cost_file], {"FTAR_BENCH_BUDGET_S": "160"})
    assert d["n_gpus"] == ranks and d["check"] == "ok" and "watchdog" not in d, d
    assert "rccl_init_error" not in d and "rccl_error_by_rank" not in d, d.get("rccl_init_error")
    # the default configuration is the execution model's: form "auto", which ran the one-round RCCL forms
    assert d["default_config"]["form"] == "auto" and d["default_config"]["check"] == "ok", d["default_config"]
    assert d["default_config"]["ran"]["form"] == "direct" and d["default_config"]["enqueue_ms"] > 0
    cm = d["cost_model"]
    assert "error" not in cm and cm["prediction_error_refit"]["entries"] >= 5, cm
    assert cm["choice_refit_measured_ms"] and cm["regret_refit"] is not None, cm
    assert all("model_ms_refit" in r for r in d["sweep"] if r.get("check") == "ok"), d["sweep"]
    best = d["rccl_p2p_best"]
    assert best and best["form"].split(":")[0] in ("direct", "stages") and best["ms"] > 0, best
    # every form says in words what moved (a gather never reads as a ring)
    assert best["form_label"].startswith(best["form"].split(":")[0] + " ("), best
    assert d["config"]["form_label"].startswith(d["config"]["form"].split(":")[0].replace("-reg", "")), d["config"]
    for form, item in (d.get("c4_ring") or {}).items():
        assert item["form_label"] in ("direct (gather + ring-order fold)", "stages (reference ring steps)"), item
        assert item["judged"] == (form == "direct")
    # the refit leaves no constant on a search bound: such a constant is flagged and keeps its prior
    p2p = cm["refit_p2p"]
    assert p2p is None or all(lo * 1.01 < p2p["params"][k] < hi / 1.01 or k in p2p["unidentified"]
                              for k, lo, hi in (("alpha_us", 0.1, 1e5), ("link_gbps", 0.5, 5e3))), p2p
    rccl_ok = [r for r in d["sweep"] if r.get("check") == "ok" and r["form"].split(":")[0] in ("direct", "stages",
                                                                                                "collective")]
    assert rccl_ok and not [r for r in d["sweep"] if r.get("check") == "MISMATCH"], d["sweep"]
    assert "RCCL over loopback" in d["config"]["parallelism"], d["config"]
    # the node's calibration file: the re-fitted constants, in the format FTAR_COST_FILE loads
    assert cm["saved_to"] == cost_file
    with open(cost_file) as f:
        saved = dict((ln.split()[0], float(ln.split()[1])) for ln in f if ln.strip() and not ln.startswith("#"))
    for k, v in saved.items():
        assert v == pytest.approx(cm["constants_refit"][k], rel=1e-3, abs=1e-3), (k, v, cm["constants_refit"])
