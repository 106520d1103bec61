#!/usr/bin/env python3
"""Per-kernel medians of rocprofv3 --pmc counters (TOOL): which HBM-side counters separate the k = 2 reduce
from pure read and pure write streams.  Reads run_counter_collection.csv files, groups dispatches by kernel
name (and grid size), and prints per-dispatch medians plus derived ratios:
  stall/cycle   = TCC_EA0_{RD,WR}REQ_DRAM_CREDIT_STALL / GRBM_GUI_ACTIVE   (EA waiting on DRAM credits)
  level/request = TCC_EA0_{RD,WR}REQ_LEVEL / TCC_EA0_{RD,WR}REQ           (mean cycles a request is queued)
  outstanding   = TCC_EA0_{RD,WR}REQ_LEVEL / GRBM_GUI_ACTIVE               (mean requests in flight, all channels)

    python tools/pmc_stalls.py CSV [CSV ...]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))   # (kernel, grid) -> counter -> [per-dispatch values]
    for path in sys.argv[1:]:
        per = defaultdict(dict)
        with open(path) as f:
            for row in csv.DictReader(f):
                key = (path, row["Dispatch_Id"])
                per[key]["__k"] = (row["Kernel_Name"][:60], int(row["Grid_Size"]))
                per[key][row["Counter_Name"]] = float(row["Counter_Value"])
        for d in per.values():
            k = d.pop("__k")
            for c, v in d.items():
                vals[k][c].append(v)
    for (kern, grid), cs in sorted(vals.items(), key=lambda t: t[0]):
        if grid < 1 << 20:
            continue
        med = {c: statistics.median(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        out = [f"{kern} grid={grid} n={n}"]
        cyc = med.get("GRBM_GUI_ACTIVE")
        for side in ("RD", "WR"):
            st = med.get(f"TCC_EA0_{side}REQ_DRAM_CREDIT_STALL_sum")
            if st is not None and cyc:
                out.append(f"{side} credit-stall/cycle={st / cyc:.3f}")
            lv, rq = med.get(f"TCC_EA0_{side}REQ_LEVEL_sum"), med.get(f"TCC_EA0_{side}REQ_sum")
            if lv is not None and rq:
                out.append(f"{side} level/req={lv / rq:.1f}")
            if lv is not None and cyc:
                out.append(f"{side} outstanding={lv / cyc:.0f}")
        for c in ("TCC_TOO_MANY_EA_WRREQS_STALL_sum", "TCC_EA0_WRREQ_STALL_sum"):
            if c in med and cyc:
                out.append(f"{c.replace('TCC_', '').replace('_sum', '')}/cycle={med[c] / cyc:.3f}")
        if cyc:
            out.append(f"cycles={cyc:.0f}")
        print("  ".join(out))


if __name__ == "__main__":
    main()
