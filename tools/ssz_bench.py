"""Host signing-root throughput (include/tbls_ssz.h): AttestationData ->
hash_tree_root -> SigningData root, the step in front of every verify.

  python tools/ssz_bench.py [--n 1000000] [--threads 1,8,16]

Prints one JSON line per thread count (roots/s); run_rate() is also called by
bench.py for its `host_signing_roots` field."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_batch(n: int, seed: int = 1):
    """n serialized AttestationData objects (128 B each) with distinct slots /
    roots, and 4 domains (4 forks of a chain)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    buf = rng.integers(0, 256, size=(n, 128), dtype=np.uint8)
    buf[:, 0:8] = np.arange(n, dtype=np.uint64).view(np.uint8).reshape(n, 8)
    domains = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(4)]
    idx = (np.arange(n) % 4).astype(np.uint32)
    return buf.tobytes(), domains, idx


def run_rate(n: int = 1_000_000, threads: int = 0, reps: int = 3):
    import ctypes
    from charon_amd import _native, ssz
    lib = _native.load()
    buf, domains, idx = make_batch(n)
    out = ctypes.create_string_buffer(32 * n)
    dom = b"".join(domains)
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        rc = lib.tbg_signing_roots(ssz.ATTESTATION_DATA, buf, n, dom, len(domains), idx.ctypes.data, out, threads)
        dt = time.perf_counter() - t0
        assert rc == 0
        best = dt if best is None else min(best, dt)
    return {"roots_per_s": round(n / best), "objects": n, "threads": threads, "kind": "attestation_data",
            "sha": "portable" if os.environ.get("TBG_SHA_PORTABLE") == "1" else "auto (x86 SHA extensions if present)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--threads", default="1,8,16")
    a = ap.parse_args()
    for t in [int(x) for x in a.threads.split(",")]:
        print(json.dumps(run_rate(a.n, t)), flush=True)


if __name__ == "__main__":
    main()
