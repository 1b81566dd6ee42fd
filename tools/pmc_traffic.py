#!/usr/bin/env python3
"""Per-kernel HBM traffic (KB per launch) from the two rocprofv3 PMC passes
of tools/gpu_pmc.sh (driven by tools/gpu_r04_bench.sh) (FETCH_SIZE and WRITE_SIZE in separate runs, as
MI355X_MICROARCH.md prescribes) -> JSON for profiles/ and bench.py.

  python tools/pmc_traffic.py gpurun_out/round profiles/rNN/traffic.json [batches_per_launch]
"""
import collections
import csv
import json
import os
import sys


# kernels that only load keys / generate test vectors (not part of the chain)
NOT_CHAIN = {"k_sign", "k_sk_to_pk", "k_decode_pubkeys", "k_pubkey_tables"}
# chain kernels that vector generation also launches (on one batch at a time):
# only their largest-grid calls belong to the chain
SHARED = {"k_hash_map", "k_hash_sswu", "k_hash_clear_x1", "k_hash_clear_x2", "k_hash_clear_fin", "k_hash_affine"}


def _grid(r):
    for k in ("Grid_Size", "Grid_Size_X", "Grid_Sizes"):
        if k in r:
            try:
                return int(str(r[k]).split(",")[0].strip("[( "))
            except ValueError:
                pass
    return 0


def main(src, dst, batches=1):
    """KB per CHAIN launch for every kernel: the sum over the kernel's calls in
    the chain launches (several per launch for k_msm_sum, k_l0_tree, the two
    k_rlc_miller_chunks modes, ...) / the number of chain launches (the calls
    of k_decode_sigs, which runs once per chain and nowhere else)."""
    out = {}
    for sub, c in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        agg = collections.defaultdict(list)
        with open(os.path.join(src, sub, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == c:
                    name = r["Kernel_Name"].split("(")[0].replace("tbg::", "").replace("void ", "")
                    agg[name].append((_grid(r), float(r["Counter_Value"])))
        chains = max(1, len(agg.get("k_decode_sigs", [])))
        for k, v in agg.items():
            if k in NOT_CHAIN:
                continue
            if k in SHARED:
                g = max(x for x, _ in v)
                v = [x for x in v if x[0] == g]
            out.setdefault(k, {})[c + "_KB_per_launch"] = round(sum(y for _, y in v) / chains, 1)
            out[k]["calls_per_launch"] = round(len(v) / chains, 2)
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
