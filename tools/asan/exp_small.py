"""Peer forms on tiny ragged buckets (blocks of 0..2 elements) in an in-process group: which shapes differ."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "allreduce-over-mpi_amd"))
import torch
import ftar

bad = []
for P in (8, 5, 3):
    g = ftar.Comm.init_local(P)
    for form in ("peer-write", "peer-read"):
        g.set_form(form)
        for dt, tdt in (("f64", torch.float64), ("f32", torch.float32), ("i32", torch.int32), ("bf16", torch.bfloat16)):
            for n in (1, P - 1, P, P + 1, 2 * P + 1, 3 * P - 1, 100):
                for topo in ("1", str(P)):
                    for oop in (True, False):
                        xs = [torch.arange(n, device="cuda").to(tdt) % 7 - 3 + r for r in range(P)]
                        want = sum(x.to(torch.float64) for x in xs)
                        ys = [torch.full_like(x, 55) for x in xs] if oop else [x.clone() for x in xs]
                        g.allreduce(xs if oop else None, ys, n, dt, "sum", topo_=topo)
                        torch.cuda.synchronize()
                        ran = g.comms[0].last_exec()["form"]
                        for r, y in enumerate(ys):
                            if not torch.equal(y.to(torch.float64), want):
                                bad.append((P, form, dt, n, topo, oop, r, ran, y.tolist()[:12]))
                                break
    g.destroy()
for b in bad:
    print("BAD", b)
print("checked; bad =", len(bad))
