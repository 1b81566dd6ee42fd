#!/usr/bin/env python3
"""Per-kernel VALU utilisation from the rocprofv3 PMC pass of
tools/pmc_valu.sh (SQ_WAVES, SQ_INSTS_VALU, SQ_INSTS_VALU_INT32/INT64,
SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE; one
isolated 10k-DV batch chain, --inflight 1) -> JSON for profiles/.

  valu_busy       = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the share of a
                    resident wave's cycles in which it issues VALU work
  int64_share     = SQ_INSTS_VALU_INT64 / SQ_INSTS_VALU (v_mad_u64_u32 and
                    the 64-bit adds of the product columns)
  valu_per_wave   = SQ_INSTS_VALU / SQ_WAVES

  python tools/valu_summary.py gpurun_out/valu/pmc/run_counter_collection.csv OUT.json
"""
import collections
import csv
import json
import sys


def main(src, dst):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(src)):
        k = r["Kernel_Name"].split("(")[0].replace("tbg::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, v in agg.items():
        d = {c: sum(x) / len(x) for c, x in v.items()}
        if d.get("SQ_INSTS_VALU", 0) < 1e6:
            continue  # empty fallback launches, fills
        out[k] = {
            "launches": len(next(iter(v.values()))),
            "waves": round(d["SQ_WAVES"]),
            "valu_per_wave": round(d["SQ_INSTS_VALU"] / max(d["SQ_WAVES"], 1)),
            "int64_share": round(d.get("SQ_INSTS_VALU_INT64", 0) / d["SQ_INSTS_VALU"], 3),
            "valu_busy": round(d["SQ_ACTIVE_INST_VALU"] / max(d["SQ_WAVE_CYCLES"], 1), 3),
        }
    doc = {"command": "rocprofv3 --pmc " + " ".join(sorted(next(iter(agg.values())).keys())) +
                      " -f csv -- python3 bench.py --no-cpu --steps 4 --inflight 1 (tools/pmc_valu.sh)",
           "kernels": out}
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in out.items():
        print(f"{k:24s} {v}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
