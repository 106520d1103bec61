#!/usr/bin/env python3
"""Summarise bench.py N > 1 lines (a driver SCALE_rNN.json, or log files holding the JSON lines) into the
calibration facts DESIGN §13 #1 asks for: per N the headline (form, topology, chunk, busBW, frac of the xGMI
spec and of the probe), the best RCCL p2p configuration beside it, the best validated entry of every form,
the xGMI probe's link rates, the fitted cost model and C5's widths, host_e2e, and any RCCL failure or
watchdog cut with the stage times.

    python tools/scale_report.py SCALE_r03.json
    python tools/scale_report.py profiles/r03/dist/*.log
"""
import json
import sys


def lines_from(path):
    """Every bench JSON line in the file: a driver record ({..., "parsed": {...}} or a list of them) or a log."""
    text = open(path).read()
    try:
        d = json.loads(text)
    except ValueError:
        d = None
    out = []

    def walk(x):
        if isinstance(x, dict):
            if "metric" in x and "n_gpus" in x:
                out.append(x)
            else:
                for v in x.values():
                    walk(v)
        elif isinstance(x, list):
            for v in x:
                walk(v)
    if d is not None:
        walk(d)
    else:
        for ln in text.splitlines():
            ln = ln.strip()
            if ln.startswith("{"):
                try:
                    walk(json.loads(ln))
                except ValueError:
                    pass
    return out


def fmt(x, nd=1):
    return "-" if x is None else (f"{x:.{nd}f}" if isinstance(x, float) else str(x))


def report(d):
    c, roof = d.get("config", {}), d.get("roofline") or {}
    print(f"== N={d['n_gpus']}: value {fmt(d.get('value'))} GB/s, {fmt(d.get('ms_per_step'), 3)} ms/call "
          f"[{c.get('form_label') or c.get('form')} topo {c.get('topology')} chunk {c.get('chunk_bytes')}] "
          f"check {d.get('check')}")
    print(f"   busBW {fmt(d.get('busbw_GBps_per_rank'))} GB/s/rank; roofline {roof.get('bound')} frac {roof.get('frac')}"
          f" (probe {roof.get('frac_of_probe')})  selection: {d.get('config_selection')}")
    if d.get("watchdog"):
        print(f"   WATCHDOG: {d['watchdog']}")
    if d.get("rccl_init_error"):
        print(f"   RCCL FAILURE: {d['rccl_init_error']}")
        for e in d.get("rccl_error_by_rank") or []:
            print(f"     rank {e.get('rank')}: {e.get('error')} | {e.get('ftar_last_error')}")
    rb = d.get("rccl_p2p_best")
    if rb:
        print(f"   rccl_p2p_best: {rb['form']} topo {rb['topology']} chunk {rb['chunk_bytes']}: {rb['ms']} ms, "
              f"busBW {rb['busbw_GBps_per_rank']} (frac {(rb.get('roofline') or {}).get('frac')})"
              f"{' = headline' if rb.get('is_headline') else ''}")
    for form, item in (d.get("c4_ring") or {}).items():
        print(f"   c4_ring {item.get('form_label')}: {item.get('ms')} ms, busBW {item.get('busbw_GBps_per_rank')} "
              f"(frac {(item.get('roofline') or {}).get('frac')}){'  <- judged (>= 70 % target)' if item.get('judged') else ''}")
    best = {}
    for r in d.get("sweep") or []:
        if r.get("check") == "ok" and "ms" in r:
            f = r["form"]
            if f not in best or r["ms"] < best[f]["ms"]:
                best[f] = r
    if best:
        print("   best per form: " + "; ".join(f"{f} {r['topology']}/{r['chunk_bytes'] >> 20}M {r['ms']}ms"
                                               for f, r in sorted(best.items(), key=lambda kv: kv[1]["ms"])))
    bad = [r for r in d.get("sweep") or [] if r.get("error") or str(r.get("check", "ok")) != "ok"]
    for r in bad[:8]:
        print(f"   sweep problem: {r.get('form')} {r.get('topology')} {r.get('chunk_bytes')}: "
              f"{r.get('error') or r.get('check')}")
    pr = d.get("xgmi_probe_GBps")
    if isinstance(pr, dict) and "error" not in pr:
        keys = [k for k in pr if k not in ("note", "by_workgroups_per_peer")]
        print("   xGMI probe [min,max over ranks]: " + ", ".join(f"{k} {pr[k]}" for k in keys))
        if pr.get("by_workgroups_per_peer"):
            print("   probe by workgroups/peer: " + ", ".join(
                f"{w}: r{v['read_all_peers']}/w{v['write_all_peers']}" for w, v in pr["by_workgroups_per_peer"].items()))
    fit = d.get("cost_model_fit")
    if isinstance(fit, dict) and "fitted" in fit:
        print(f"   cost model fitted {fit['fitted']} -> {fit.get('choice_fitted')} (reference model: "
              f"{fit.get('choice_reference_model')})")
    cm = d.get("cost_model")
    if isinstance(cm, dict) and "constants_refit" in cm:
        p2p = cm.get("refit_p2p") or {}
        print(f"   cost model refit {cm['constants_refit']}; unidentified (prior kept): {p2p.get('unidentified')}"
              f"{'; kept the prior whole' if p2p.get('kept_prior') else ''}; regret {cm.get('regret_refit')}"
              f"{'; saved to ' + cm['saved_to'] if cm.get('saved_to') else ''}")
        for f, r in (cm.get("refit_rates") or {}).items():
            if r and r.get("unidentified"):
                print(f"     {f}: unidentified ({r['unidentified']}), prior {r.get('value')} kept")
    c5 = d.get("c5_bf16")
    if isinstance(c5, dict) and "ms" in c5:
        ow = ", ".join(f"{k} {v.get('ms')}ms" for k, v in (c5.get("other_widths") or {}).items())
        tie = (f"; the model's width was a tie of {c5.get('model_tied')} broken by {c5.get('model_tie_broken_by')}"
               if (c5.get("model_tied") or 1) > 1 else "")
        print(f"   C5 bf16: {c5['topology']} {c5['ms']} ms ({c5.get('check')}){tie}; other widths: {ow}")
    he = d.get("host_e2e")
    if isinstance(he, dict) and "ms" in he:
        print(f"   host e2e: {he['ms']} ms = {he.get('algbw_GBps_per_rank')} GB/s/rank ({he.get('check')})")
    y = d.get("rccl_native_allreduce")
    if isinstance(y, dict):
        print(f"   RCCL ncclAllReduce: {y.get('ms')} ms, busBW {y.get('busbw_GBps')}")
    if d.get("stage_wall_s"):
        print("   stages (s): " + ", ".join(f"{k} {v}" for k, v in d["stage_wall_s"].items()))


def main():
    found = []
    for p in sys.argv[1:]:
        found += lines_from(p)
    for d in sorted(found, key=lambda x: x.get("n_gpus", 0)):
        if d.get("n_gpus", 1) > 1 or "sweep" in d:
            report(d)
    if not found:
        print("no bench lines found")


if __name__ == "__main__":
    main()
