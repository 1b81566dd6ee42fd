#!/usr/bin/env python3
"""Where a kernel's wave time goes, from one rocprofv3 SQ counter pass
(tools/gpu_pmc_stall.sh): SQ_WAIT_ANY (parked at s_waitcnt / barrier --
memory), SQ_WAIT_INST_ANY (issue stalls), SQ_ACTIVE_INST_ANY (issuing);
the three are disjoint and add up to SQ_WAVE_CYCLES (MI355X_MICROARCH.md,
PMC table).  Summed over each kernel's dispatches.

  python tools/pmc_stall.py gpurun_out/stall/run_counter_collection.csv [out.json]
"""
import collections
import csv
import json
import sys

COUNTERS = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
            "SQ_INSTS_VALU", "SQ_WAVES", "SQ_BUSY_CYCLES")


def main(src, dst=None):
    agg = collections.defaultdict(lambda: collections.Counter())
    calls = collections.Counter()
    seen = set()
    with open(src) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0].replace("tbg::", "").replace("void ", "")
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (name, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            if key not in seen:
                seen.add(key)
                calls[name] += 1
    out = {}
    for k, c in agg.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0:
            continue
        out[k] = {"calls": calls[k], "wave_cycles": wc,
                  "wait_any": round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
                  "wait_inst_any": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                  "active_inst_any": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
                  "active_valu": round(c.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
                  "valu_insts": c.get("SQ_INSTS_VALU", 0), "waves": c.get("SQ_WAVES", 0)}
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["wave_cycles"])[:20]:
        print(f"{k[:40]:40s} waves {v['waves']:>9.0f} wait {v['wait_any']:.3f} issue-stall {v['wait_inst_any']:.3f} "
              f"active {v['active_inst_any']:.3f} valu {v['active_valu']:.3f}")
    if dst:
        json.dump({"source": src, "kernels": out}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
