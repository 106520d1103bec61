#!/usr/bin/env python3
"""Which NaN does a float sum return when several NaNs meet?  Prints a handful of elements where the
one-round ring fold (4 in-process ranks) and the oracle's staged ring differ, with every rank's input, and
the GPU's 2-source reduce of NaN pairs in both orders."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "allreduce-over-mpi_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ftar  # noqa: E402
import ftar_inputs as fi  # noqa: E402
import oracle_lib  # noqa: E402
from test_gpu_reduce import _bf16_specials, _f32_specials  # noqa: E402


def main():
    for dt in ("f32", "bf16"):
        P, n = 4, 50_001
        view = np.int16 if dt == "bf16" else np.int32
        uview = np.uint16 if dt == "bf16" else np.uint32
        xs = [(_bf16_specials if dt == "bf16" else _f32_specials)(11, r, n) for r in range(P)]
        g = ftar.Comm.init_local(P)
        g.set_reduce_scatter("direct")
        bufs = [torch.from_numpy(x.view(view).copy()).cuda() for x in xs]
        g.allreduce(None, bufs, n, dt, "sum", topo_="1")
        torch.cuda.synchronize()
        got = bufs[0].cpu().numpy().view(uview)
        ref = oracle_lib.allreduce(xs, "1", dtype=fi.BY_NAME[dt])[0].view(uview)
        bad = np.nonzero(got != ref)[0]
        split = (n + P - 1) // P
        print(dt, "mismatches", bad.size)
        for i in bad[:8]:
            b = i // split
            print(f"  elem {i} block {b}: inputs x_b..x_b+3 =", [hex(int(xs[(b + j) % P].view(uview)[i])) for j in range(P)],
                  "gpu", hex(int(got[i])), "oracle", hex(int(ref[i])))
        g.destroy()
        # 2-source reduce: which NaN wins
        nan_a = np.array([0x7FC01234 if dt == "f32" else 0x7FC1], dtype=uview)
        nan_b = np.array([0xFFC05678 if dt == "f32" else 0xFFC3], dtype=uview)
        for a_, b_ in ((nan_a, nan_b), (nan_b, nan_a)):
            ta = torch.from_numpy(a_.view(view).copy()).cuda()
            tb = torch.from_numpy(b_.view(view).copy()).cuda()
            out = torch.empty_like(ta)
            ftar.reduce([ta, tb], out, 1, dt, "sum")
            torch.cuda.synchronize()
            o = oracle_lib.reduce(fi.BY_NAME[dt], 0, [a_.view(fi.DTYPES[fi.BY_NAME[dt]][1]), b_.view(fi.DTYPES[fi.BY_NAME[dt]][1])])
            print(f"  {dt} reduce({hex(int(a_[0]))}, {hex(int(b_[0]))}) gpu {hex(int(out.cpu().numpy().view(uview)[0]))}"
                  f" oracle {hex(int(np.asarray(o).view(uview)[0]))}")


if __name__ == "__main__":
    main()
