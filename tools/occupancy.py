#!/usr/bin/env python3
"""Wave-slot occupancy of the pipelined bench from a rocprofv3 kernel trace.

For every dispatch in the window [t_start, end] (ms from the first
dispatch), the grid's waves are counted as resident from its start to its end
timestamp (an upper bound: a dispatch's waves do not all run for its whole
span).  Prints the mean number of waves demanded, the same capped at the
machine's capacity (256 CUs x 4 SIMDs = 1024 waves at one wave per SIMD,
which is what the big kernels get: 256 VGPRs + AGPRs; 2048 at two), and each
kernel's share of the window.

  python tools/occupancy.py run_kernel_trace.csv T_START_MS
"""
import collections
import csv
import sys

import numpy as np


def main(path, t_start_ms):
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].replace("tbg::", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"]) // 64, n))
    t0 = min(e[0] for e in ev)
    lo = t0 + int(float(t_start_ms) * 1e6)
    ev = [e for e in ev if e[0] >= lo]
    hi = max(e[1] for e in ev)
    ts = np.linspace(lo, hi, 50000)
    occ = np.zeros_like(ts)
    busy = collections.Counter()
    for s, e, w, n in ev:
        m = (ts >= s) & (ts < e)
        occ[m] += w
        busy[n] += w * (e - s)
    span = hi - lo
    print(f"window {span / 1e6:.1f} ms, {len(ev)} dispatches")
    print(f"mean waves demanded {occ.mean():.0f}; capped at 1024 (1 wave/SIMD): {np.minimum(occ, 1024).mean():.0f} "
          f"({np.minimum(occ, 1024).mean() / 1024:.1%}); time with < 1024 waves demanded: {(occ < 1024).mean():.1%}")
    tot = sum(busy.values())
    for n, v in busy.most_common():
        print(f"  {n:24s} {v / span:8.1f} waves avg  {v / tot:6.1%}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
