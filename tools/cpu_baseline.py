"""CPU baseline for bench.py: the C restatement of the reference tbls path
(oracle/c, kind "port") timed on the host cores over a bounded sample of the
bench batch.  The reference Go/kryptology path cannot be built here (no Go
toolchain, kryptology not vendored), so this is the labelled
fallback of BASELINE.md.

Per DV-duty the CPU does what the reference does per tbls.VerifyAndAggregate
call: decode the n partial signatures (SigFromCore, with subgroup checks),
H(m), n two-pair pairing checks, Lagrange combination, compression.
Pubshares are decoded once outside the timed region (startup in Charon,
app/app.go:334-376).  One host thread per core, duties handed out
dynamically (the reference runs one goroutine per peer message / duty).
"""
from __future__ import annotations

import os
import time

import numpy as np


def host_cores():
    """Threads for the CPU baseline: every core this process may use.

    On the GPU pool one GPU's job gets a 16-core share of a 256-core machine
    (the harness sets OMP_NUM_THREADS=16 there; os.cpu_count() and the
    affinity mask still report the whole machine).  The share is the host
    a one-GPU Charon node would have, so that is what is timed; the machine
    count and the per-core rate are reported beside it so the rate can be
    scaled.  Elsewhere (no OMP_NUM_THREADS) every core in the affinity mask."""
    machine = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = machine
    quota = cgroup_cpus()
    if quota:
        avail = min(avail, quota)
    share = os.environ.get("OMP_NUM_THREADS")
    n = min(avail, int(share)) if share and share.isdigit() and int(share) > 0 else avail
    return max(1, n), machine


def cgroup_cpus():
    """CPUs the cgroup's CFS quota allows (cgroup v2 cpu.max), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q == "max":
            return None
        return max(1, -(-int(q) // int(p)))
    except (OSError, ValueError):
        return None


def run_cpu_baseline(batch, seconds: float = 15.0, chunk: int = 512):
    from oracle import c as oc
    oc.build()
    cores, machine = host_cores()
    n = batch.n
    # startup decode (untimed) of the pubshares of the DVs the sample can reach:
    # the first `cap` DVs (the oracle's table decodes on one thread)
    cap = min(batch.n_dv, max(chunk, 12000))
    table = oc.PubkeyTable(np.asarray(batch.pubshares[:cap * n], dtype=np.uint8))
    first_id = int(batch.pubkey_ids[0])
    done = mismatches = 0
    t0 = time.perf_counter()
    d0 = 0
    while d0 < cap and time.perf_counter() - t0 < seconds:
        d1 = min(d0 + chunk, cap)
        nd = d1 - d0
        sigs = np.asarray(batch.sigs[d0 * n:d1 * n], dtype=np.uint8)
        ids = batch.identifiers[d0 * n:d1 * n]
        pk_ids = (np.asarray(batch.pubkey_ids[d0 * n:d1 * n], dtype=np.int64) - first_id).astype(np.uint32)
        msgs = np.asarray(batch.msg_data[d0 * 32:d1 * 32], dtype=np.uint8)
        ps, ds, agg = oc.run(3, np.arange(nd + 1) * n, sigs, ids, table, msgs=msgs, msg_off=np.arange(nd + 1) * 32,
                             duty_msg=np.arange(nd), pubkey_ids=pk_ids, duty_threshold=batch.threshold[d0:d1],
                             threads=cores)
        mismatches += int((ds != 0).sum()) + int((ps != 1).sum())
        mismatches += int((agg != np.asarray(batch.group_sig[d0:d1])).any(axis=1).sum())
        done += nd
        d0 = d1
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 3), "unit": "DV-duties/s", "cores": cores, "kind": "port",
            "per_core": round(done / dt / cores, 3), "machine_cores": machine,
            "cgroup_cpus": cgroup_cpus(),
            "sample": f"first {done} DVs of the rank-0 bench batch ({batch.t}-of-{n}); C restatement of the "
                      f"reference per-item schedule (oracle/c), {cores} threads = every core this job may use "
                      f"(affinity, cgroup quota, OMP_NUM_THREADS; the machine has {machine}), {dt:.1f}s; "
                      f"not the Go reference",
            "mismatches": mismatches}
