"""Child process of tests/test_gpu_allreduce.py::test_allreduce_group_captures_into_a_hip_graph (run in its
own process so that a HIP runtime abort cannot take the test runner down).

One in-process group of P ranks on cuda:0: a warm-up call outside capture (sizes scratch and events), then
the group call captured into one HIP graph -- torch.cuda.graph in relaxed mode on stream s0, every rank's
stream forked from s0 and joined back -- then replayed on fresh inputs written in place.  Writes every
replay's per-rank outputs to OUT.npz.

usage: capture_child.py OUT P TOPO N CHUNK RS AG REPLAYS   (CAPTURE_SHARED=1: every rank's call on the
capture stream itself instead of a stream forked per rank)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "allreduce-over-mpi_amd"), os.path.join(ROOT, "tests")]


def step(msg):
    sys.stderr.write(f"[capture_child] {msg}\n")
    sys.stderr.flush()


def main():
    if os.environ.get("SEGV_BT"):   # diagnostic: native backtrace on a crash (tools/capture/segv_bt.c)
        import ctypes
        import resource
        ctypes.CDLL(os.environ["SEGV_BT"])
        sys.stderr.write(f"[capture_child] stack limit {resource.getrlimit(resource.RLIMIT_STACK)}\n")
    else:
        import faulthandler
        faulthandler.enable()
    out, P, topo, n, chunk, rs, ag, replays = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), \
        int(sys.argv[5]), sys.argv[6], sys.argv[7], int(sys.argv[8])
    import torch
    import ftar
    import ftar_inputs as fi
    torch.cuda.set_device(0)
    g = ftar.Comm.init_local(P)
    g.set_chunk_bytes(chunk)
    g.set_reduce_scatter(rs)
    g.set_allgather(ag)
    xs = [torch.from_numpy(fi.fill("f32", 99, r, n).copy()).cuda() for r in range(P)]
    ys = [torch.empty_like(x) for x in xs]
    g.allreduce(xs, ys, n, "f32", "sum", topo_=topo)   # warm-up: every buffer and event exists before capture
    torch.cuda.synchronize()
    step("warm-up done")
    if os.environ.get("CAPTURE_RAW"):
        replay = raw_capture(g, xs, ys, n, topo, P)
    else:
        replay = torch_capture(g, xs, ys, n, topo, P)
    res = {}
    for it in range(replays):
        for r in range(P):
            xs[r].copy_(torch.from_numpy(fi.fill("f32", 1000 + it, r, n)))
            ys[r].fill_(float("nan"))
        torch.cuda.synchronize()
        replay()
        torch.cuda.synchronize()
        step(f"replay {it} done")
        for r in range(P):
            res[f"it{it}_r{r}"] = ys[r].cpu().numpy()
    np.savez(out, **res)
    g.destroy()
    print("capture ok", flush=True)


def raw_capture(g, xs, ys, n, topo, P):
    """hipStreamBeginCapture (relaxed) / hipStreamEndCapture / hipGraphInstantiate / hipGraphLaunch via ctypes:
    the HIP runtime's own capture, no torch in the way."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p

    def ck(rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: hip error {rc}")
    s0, fork = vp(), vp()
    ck(hip.hipStreamCreateWithFlags(ctypes.byref(s0), 1), "stream")
    ck(hip.hipEventCreateWithFlags(ctypes.byref(fork), 2), "event")
    rs, joins = [], []
    for _ in range(P):
        s, e = vp(), vp()
        ck(hip.hipStreamCreateWithFlags(ctypes.byref(s), 1), "stream")
        ck(hip.hipEventCreateWithFlags(ctypes.byref(e), 2), "event")
        rs.append(s)
        joins.append(e)
    ck(hip.hipStreamBeginCapture(s0, 2), "hipStreamBeginCapture")   # hipStreamCaptureModeRelaxed
    step("capture begun (raw)")
    ck(hip.hipEventRecord(fork, s0), "record")
    for s in rs:
        ck(hip.hipStreamWaitEvent(s, fork, 0), "fork")
    g.allreduce(xs, ys, n, "f32", "sum", topo_=topo, streams=[s.value for s in rs])
    step("group call issued")
    for s, e in zip(rs, joins):
        ck(hip.hipEventRecord(e, s), "record")
        ck(hip.hipStreamWaitEvent(s0, e, 0), "join")
    graph, exe = vp(), vp()
    ck(hip.hipStreamEndCapture(s0, ctypes.byref(graph)), "hipStreamEndCapture")
    step("capture ended")
    ck(hip.hipGraphInstantiate(ctypes.byref(exe), graph, None, None, 0), "hipGraphInstantiate")

    def replay():
        ck(hip.hipGraphLaunch(exe, s0), "hipGraphLaunch")
        ck(hip.hipStreamSynchronize(s0), "sync")
    return replay


def torch_capture(g, xs, ys, n, topo, P):
    import torch
    s0 = torch.cuda.Stream()
    shared = bool(os.environ.get("CAPTURE_SHARED"))
    rank_streams = [s0] * P if shared else [torch.cuda.Stream() for _ in range(P)]
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s0):
        with torch.cuda.graph(graph, stream=s0, capture_error_mode="relaxed"):
            step("capture begun")
            for s in rank_streams:
                if s is not s0:
                    s.wait_stream(s0)
            g.allreduce(xs, ys, n, "f32", "sum", topo_=topo, streams=rank_streams)
            step("group call issued")
            for s in rank_streams:
                if s is not s0:
                    s0.wait_stream(s)
    step("capture ended")
    torch.cuda.synchronize()
    return graph.replay


if __name__ == "__main__":
    main()
