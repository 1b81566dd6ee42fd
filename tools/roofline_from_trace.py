#!/usr/bin/env python3
"""Recompute bench.py's `roofline` from a rocprofv3 kernel trace of the same
command (the reproducibility check of the bench line).

bench.py prices the dominant kernel of ONE device batch replayed alone
(tbg_replay_profile, after its timed region).  In the trace of that command
the kernel's dispatches of the full device-batch grid that overlap NO other
dispatch are those exclusive runs (the replay_profile pass, and the
one-at-a-time first submits of the bench's setup); their mean duration,
with the work model of profiles/work_model.json, gives achieved / frac.

  python tools/roofline_from_trace.py <run_kernel_trace.csv> <bench.json> [--out summary.json]

Prints (and writes with --out) the kernel's exclusive dispatches, their mean
duration, the recomputed frac and its ratio to the bench line's frac.
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _grid(r):
    for k in ("Grid_Size", "Grid_Size_X", "Grid_Sizes"):
        if k in r and r[k] not in (None, ""):
            try:
                return int(str(r[k]).split(",")[0].strip("[( "))
            except ValueError:
                pass
    return 0


def exclusive_dispatches(rows, symbol):
    """Dispatches of `symbol` with the largest grid that overlap no other dispatch."""
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], _grid(r)) for r in rows))
    mine = [e for e in ev if e[2] == symbol]
    if not mine:
        return [], 0
    g = max(e[3] for e in mine)
    out = []
    for s, t, name, grid in mine:
        if grid != g:
            continue
        overlap = any(o is not None and o[0] < t and o[1] > s and not (o[0] == s and o[1] == t and o[2] == name)
                      for o in ev)
        if not overlap:
            out.append((s, t))
    return out, g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    a = ap.parse_args()
    bench = None
    with open(a.bench) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{") and '"roofline"' in line:
                bench = json.loads(line)
    if bench is None or not bench.get("roofline"):
        sys.exit("no bench line with a roofline in " + a.bench)
    rl = bench["roofline"]
    rows = list(csv.DictReader(open(a.trace)))
    disp, grid = exclusive_dispatches(rows, rl["rocprof_name"])
    if not disp:
        sys.exit(f"no exclusive dispatch of {rl['rocprof_name']} in {a.trace}")
    durs = [(t - s) / 1e6 for s, t in disp]
    mean_ms = sum(durs) / len(durs)
    ach = rl["algorithmic_mads_per_launch"] / (mean_ms * 1e-3) / 1e12
    frac = ach / rl["peak"]
    out = {"kernel": rl["rocprof_name"], "grid": grid, "exclusive_dispatches": len(durs),
           "durations_ms": [round(d, 4) for d in durs], "mean_ms": round(mean_ms, 4),
           "bench_launch_ms": rl["launch_ms"], "algorithmic_mads_per_launch": rl["algorithmic_mads_per_launch"],
           "achieved_T": round(ach, 3), "frac_from_trace": round(frac, 4), "frac_bench": rl["frac"],
           "ratio": round(frac / rl["frac"], 4)}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
