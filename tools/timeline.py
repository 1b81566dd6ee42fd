#!/usr/bin/env python3
"""Timeline of bench.py's timed region from a rocprofv3 kernel trace.

The driver's command (`bench.py --steps 20 --warmup 5`) times ONE replay
plan: three launches (7 + 7 + 6 caller batches of 10k DVs) in flight
together.  This finds those three chains in the trace (the k_decode_sigs
dispatches whose grids cover 20 batches' partials, started together), then
prints each chain's kernels in order with start / end (ms from the region's
start) and wave count, and a coarse fill curve: per 0.5 ms bin, the waves of
the dispatches running in it (capped at the 2,048 wave slots of two waves
per SIMD), so latency-bound stretches where the three chains leave the GPU
idle stand out.

  python tools/timeline.py <run_kernel_trace.csv> [--steps 20] [--batch-partials 40000]
"""
import argparse
import csv
import collections


def grid(r):
    for k in ("Grid_Size", "Grid_Size_X", "Grid_Sizes"):
        if k in r and r[k] not in (None, ""):
            try:
                return int(str(r[k]).split(",")[0].strip("[( "))
            except ValueError:
                pass
    return 0


def short(name):
    return name.split("(")[0].replace("void ", "").replace("tbg::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch-partials", type=int, default=40000)
    ap.add_argument("--bin", type=float, default=0.5)
    ap.add_argument("--per-lane", type=int, default=1, help="signatures per k_decode_sigs lane")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), grid(r),
                 r.get("Queue_Id", r.get("Stream_Id", ""))) for r in rows)
    dec = [e for e in ev if e[2] == "k_decode_sigs"]
    # groups of decode dispatches that start within 30 ms of each other
    groups, cur = [], []
    for e in dec:
        if cur and e[0] - cur[0][0] > 30e6:
            groups.append(cur)
            cur = []
        cur.append(e)
    if cur:
        groups.append(cur)
    want = a.steps * a.batch_partials // a.per_lane
    timed = None
    for g in groups:
        if abs(sum(x[3] for x in g) - want) <= 64 * len(g) * 16:
            timed = g  # the last matching group (the warmup plan is smaller)
    if timed is None:
        raise SystemExit(f"no group of decode dispatches covers {want} partials: {[sum(x[3] for x in g) for g in groups]}")
    queues = {x[4] for x in timed}
    # each chain starts with its per-message kernels (hash_to_G2, H(m) lines)
    # before its decode: walk back over dispatches of the same queue that
    # follow each other within 2 ms; the chain ends at its last aggregation
    # kernel (k_aggregate_exc<false>) after the decode
    t0, t1 = float("inf"), 0
    region = []
    for d in timed:
        q = d[4]
        mine = [e for e in ev if e[4] == q]
        i = mine.index(d)
        j = i
        while j > 0 and mine[j][0] - mine[j - 1][1] < 2e6:
            j -= 1
        k = i
        while k + 1 < len(mine) and mine[k][2] != "k_aggregate_exc<false>":
            k += 1
        region += mine[j:k + 1]
        t0, t1 = min(t0, mine[j][0]), max(t1, mine[k][1])
    region.sort()
    print(f"timed region: {len(timed)} chains, {(t1 - t0) / 1e6:.3f} ms, queues {sorted(queues)}")
    for q in sorted(queues):
        print(f"\n-- chain on queue {q}")
        for s, t, n, gsz, qq in region:
            if qq != q:
                continue
            print(f"  {(s - t0) / 1e6:8.3f} {(t - t0) / 1e6:8.3f} {(t - s) / 1e6:7.3f}  {gsz // 64:7d}w  {n}")
    nb = int((t1 - t0) / 1e6 / a.bin) + 1
    fill = [0.0] * nb
    who = [collections.Counter() for _ in range(nb)]
    for s, t, n, gsz, qq in region:
        for b in range(int((s - t0) / 1e6 / a.bin), min(nb, int((t - t0) / 1e6 / a.bin) + 1)):
            fill[b] += min(2048, gsz // 64)
            who[b][n] += 1
    print("\n-- fill (waves running, capped at 2048 per dispatch) per bin")
    for b in range(nb):
        top = ", ".join(k for k, _ in who[b].most_common(3))
        print(f"  {b * a.bin:7.1f} ms {min(fill[b], 9999):6.0f}  {'#' * int(min(fill[b], 4096) / 128)}  {top}")


if __name__ == "__main__":
    main()
