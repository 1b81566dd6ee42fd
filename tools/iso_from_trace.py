#!/usr/bin/env python3
"""Durations of the isolated-batch chain bench.py replays last (after its
timed region), from a rocprofv3 --kernel-trace CSV: the rocprof side of the
roofline's per-launch time (bench.py "isolated_batch_ms").

  python tools/iso_from_trace.py gpurun_out/round/prof/run_kernel_trace.csv
"""
import csv
import json
import sys

CHAIN = ["k_decode_sigs", "k_rlc_partial", "k_rlc_duty_sum", "k_rlc_group_lines", "k_hash_msgs", "k_lines_h",
         "k_rlc_miller_chunks", "k_rlc_group_final"]


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = {}
    for r in rows:  # the last launch of each kernel is the isolated chain's
        k = r["Kernel_Name"].split("(")[0].replace("tbg::", "")
        last[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    out = {k: round(last[k], 3) for k in CHAIN if k in last}
    out["verify_stage_ms(chunks+final)"] = round(last.get("k_rlc_miller_chunks", 0) + last.get("k_rlc_group_final", 0), 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
