#!/usr/bin/env python3
"""Per-kernel HBM traffic (KB per launch) from the two rocprofv3 PMC passes
of tools/gpu_round.sh (FETCH_SIZE and WRITE_SIZE in separate runs, as
MI355X_MICROARCH.md prescribes) -> JSON for profiles/ and bench.py.

  python tools/pmc_traffic.py gpurun_out/round profiles/rNN/traffic.json [batches_per_launch]
"""
import collections
import csv
import json
import os
import sys


def main(src, dst, batches=1):
    out = {}
    for sub, c in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        agg = collections.defaultdict(list)
        with open(os.path.join(src, sub, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == c:
                    agg[r["Kernel_Name"].split("(")[0].replace("tbg::", "")].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            out.setdefault(k, {})[c + "_KB_per_launch"] = round(sum(v) / len(v), 1)
            out[k]["launches"] = len(v)
    doc = {"command": "rocprofv3 --pmc FETCH_SIZE (resp. WRITE_SIZE) -f csv -- python3 bench.py --no-cpu "
                      "--inflight 1 --merge %d --steps %d --warmup 0 --api-batches 0 (tools/gpu_pmc.sh)" % (batches, batches),
           "note": "one counter group per pass; raw values in KB per launch.  bench.py counts FETCH_SIZE x 2 (the "
                   "gfx950 correction of MI355X_MICROARCH.md, calibrated for 16-B/lane streaming reads) + WRITE_SIZE; "
                   "a launch here covers batches_per_launch batches of 10k 3-of-4 DVs",
           "batches_per_launch": batches,
           "kernels": out}
    with open(dst, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1)
