"""tests/host_comm_cases.gather_forensics on synthetic records (CPU): a wrong tile is traced to the gather
workgroup that copies it -- workgroup w copies tiles w / nsegs + j * grid / nsegs of segment w % nsegs
(reduce_impl.h gather_body) -- and that workgroup's records are reported."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import host_comm_cases as hc  # noqa: E402

TILE = 8192          # 2 x 256 threads x 16 B
ESZ = 4


class FakeComm:
    """Two pieces; piece p gathers 3 segments of 4 tiles each (grid 6: 2 workgroups per segment, each 2 tiles)
    at element offsets seg * 10 tiles + p * 4 tiles."""

    def __init__(self, lost_xcc=None, dev_lost=False):
        self.records = []
        for p in range(2):
            grid, m = 6, 3
            host = np.zeros((grid, 4), dtype=np.uint32)
            for w in range(grid):
                host[w] = [0x80000000 | (w % 8), (1 << 30) | (2 << 24) | (w % 4), 100 + w, 200 + w]
            dev = np.zeros(2 * grid, dtype=np.uint32)     # per id: how many times it ran, on which XCDs
            dev[0::2] = 1
            dev[1::2] = [1 << (w % 8) for w in range(grid)]
            if dev_lost and p == 1:   # id lost_xcc never ran; id lost_xcc - 4's workgroups ran it a second time
                dev[2 * lost_xcc] = 0
                dev[2 * lost_xcc + 1] = 0
                dev[2 * (lost_xcc - 4)] = 2
                dev[2 * (lost_xcc - 4) + 1] |= 1 << lost_xcc
            self.records.append({"pieces": 2, "grid": grid, "nsegs": m, "tile_bytes": TILE,
                                 "off": [(s * 10 + p * 4) * TILE for s in range(m)], "bytes": [4 * TILE] * m,
                                 "host": host, "dev_ptr": p, "dev": dev})

    def gather_log(self, k):
        return self.records[k] if k < len(self.records) else None


def tiles_of(w, grid=6, m=3, tiles=4):
    """the (segment, tile) pairs workgroup w copies"""
    nb = grid // m
    return [(w % m, t) for t in range(tiles) if t % nb == w // m]


def test_wrong_tiles_name_their_workgroups_and_xcd():
    comm = FakeComm(lost_xcc=4, dev_lost=True)
    n = 40 * TILE // ESZ
    exp = torch.arange(n, dtype=torch.float32)
    y = exp.clone()
    # piece 1: workgroup 4 (4 % 8 = XCD 4) left its tiles holding something else
    for s, t in tiles_of(4):
        lo = ((s * 10 + 4) + t) * TILE // ESZ
        y[lo:lo + TILE // ESZ] = -1
    out = hc.gather_forensics(comm, y, exp, torch.float32, read_dev=lambda ptr, words: comm.records[ptr]["dev"])
    assert out["pieces"] == 2 and out["wgs"] == 12 and out["host_missing"] == 0 and out["dev_missing"] == 1
    assert out["xcc_is_w_mod_8"] == 12 and out["queues"] == {"me1.pipe0.q2": 12}
    [b] = out["bad"]
    assert b["piece"] == 1 and b["first_wgs"] == [4] and b["bad_tiles"] == 2
    assert b["xcc"] == {4: 1} and b["w_mod_8"] == {4: 1} and b["host_present"] == 1 and b["dev_present"] == 0
    assert b["piece_runs"] == 6 and b["piece_ids_run_twice"] == 1 and out["runs"] == 12
    assert b["twice_w_mod_8"] == {0: 1} and b["twice_xcds"] == {"0,4": 1}
    assert b["end_ticks_of_bad"] == [104, 104] and b["piece_span_ticks"] == 105
    assert b["piece_queues"] == {"me1.pipe0.q2": 6} and b["rotation"] == {0: 6} and b["largest_start_gap"] == 1
    assert b["end_pct"][0] == 100 and b["end_pct"][-1] == 105 and out["split_pieces"] == 0


def test_right_result_lists_no_bad_piece():
    comm = FakeComm()
    n = 40 * TILE // ESZ
    exp = torch.arange(n, dtype=torch.float32)
    out = hc.gather_forensics(comm, exp.clone(), exp, torch.float32,
                              read_dev=lambda ptr, words: comm.records[ptr]["dev"])
    assert out["bad"] == [] and out["host_missing"] == 0 and out["dev_missing"] == 0 and out["split_pieces"] == 0
    comm.records[0]["host"][5, 1] = (1 << 30) | (5 << 24) | 64     # one workgroup ran from another queue slot
    out = hc.gather_forensics(comm, exp.clone(), exp, torch.float32,
                              read_dev=lambda ptr, words: comm.records[ptr]["dev"])
    assert out["split_pieces"] == 1 and out["queues"] == {"me1.pipe0.q2": 11, "me1.pipe1.q5": 1}
