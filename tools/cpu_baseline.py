"""CPU baseline for bench.py: the oracle (a CPU restatement of the reference
tbls path, kind "port") timed on the host cores over a bounded sample of the
bench batch.  The reference Go/kryptology path cannot be built here (no Go
toolchain, kryptology not vendored), so this is the labelled
fallback of BASELINE.md.

Per DV-duty the CPU does what the GPU step does: decode the n partial
signatures (SigFromCore), H(m), n pairing checks, Lagrange combine, compress.
Pubshares are decoded once outside the timed region (startup in Charon,
app/app.go:334-376).
"""
from __future__ import annotations

import os
import time
from concurrent.futures import ProcessPoolExecutor

_STATE = {}


def _init(pubshares_hex, t, n):
    from oracle import bls12_381 as bls
    _STATE["pk"] = [bls.g1_decompress(bytes.fromhex(h)) for h in pubshares_hex]
    _STATE["t"], _STATE["n"] = t, n


def _one(args):
    from oracle import bls12_381 as bls
    from oracle import tbls_oracle as tb
    d, msg, sigs = args
    n = _STATE["n"]
    pks = _STATE["pk"][d * n:(d + 1) * n]
    tss = tb.TSS({i + 1: pks[i] for i in range(n)}, n, _STATE["t"])
    partials = [(i + 1, bls.g2_decompress(s)) for i, s in enumerate(sigs)]
    agg, _ = tb.verify_and_aggregate(tss, partials, msg)
    return bls.g2_compress(agg)


def host_cores():
    n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(n, cap))


def run_cpu_baseline(batch, seconds: float = 15.0, max_dvs: int = 4096):
    cores = host_cores()
    n_dv = min(batch.n_dv, max_dvs)
    n = batch.n
    pks = [bytes(batch.pubshares[i]).hex() for i in range(n_dv * n)]
    tasks = [(d, batch.msgs[d], [bytes(batch.sigs[d * n + i]) for i in range(n)]) for d in range(n_dv)]
    done = 0
    mismatches = 0
    with ProcessPoolExecutor(max_workers=cores, initializer=_init, initargs=(pks, batch.t, n)) as ex:
        # warm the workers (imports, pubshare decode) outside the timed region
        list(ex.map(_init_probe, range(cores)))
        t0 = time.perf_counter()
        i = 0
        while i < n_dv and time.perf_counter() - t0 < seconds:
            chunk = tasks[i:i + cores]
            for d_out, agg in zip(range(i, i + len(chunk)), ex.map(_one, chunk)):
                mismatches += agg != bytes(batch.group_sig[d_out])
            done += len(chunk)
            i += len(chunk)
        dt = time.perf_counter() - t0
    return {"value": round(done / dt, 3), "unit": "DV-duties/s", "cores": cores, "kind": "port",
            "sample": f"first {done} DVs of the rank-0 bench batch ({batch.t}-of-{n}, Python oracle, "
                      f"{cores} processes, {dt:.1f}s); CPU restatement, not the Go reference",
            "mismatches": mismatches}


def _init_probe(_):
    return len(_STATE.get("pk", []))
