#!/usr/bin/env python3
"""Benchmark: verified+aggregated 3-of-4 threshold BLS signatures per second.

One step = one pass of the hot path (decode -> hash_to_G2 -> per-partial
pairing check -> Lagrange -> G2 MSM -> compress) over one batch of
BASELINE config 2: 10,000 DVs x 1 attestation, 3-of-4 (40,000 partial
verifies + 10,000 aggregates) with inputs resident in HBM.  Multi-GPU is
weak scaling: every rank runs its own 10k-DV shard (independent validators,
no cross-GPU math; BASELINE config 4 is this at 125k DVs per GPU).

Single GPU:  python bench.py
N GPUs:      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
             or python bench.py --gpus N (starts the N rank processes itself)
Ranks meet on gloo (barrier + max over ranks); each holds one HIP runtime,
the engine library's.  Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# GPU_MAX_HW_QUEUES (hardware queues per process, HIP's default 4) is read
# once, at HIP initialisation.  The engine no longer needs more than the
# default: concurrent batches are packed into one device batch per launch
# (tbg_submit_group), so a few streams fill the GPU.  --hw-queues still sets
# it (before anything touches the GPU) for comparisons.
def _hw_queues(argv):
    v = None  # default: leave the environment alone (HIP's own default is 4)
    for i, a in enumerate(argv):
        if a == "--hw-queues" and i + 1 < len(argv):
            v = argv[i + 1]
        elif a.startswith("--hw-queues="):
            v = a.split("=", 1)[1]
    if v is None:
        return None
    if not v.isdigit() or not 1 <= int(v) <= 32:  # HIP refuses > 32; checked before HIP initialises
        sys.exit(f"bench.py: --hw-queues must be an integer in 1..32, got {v!r}")
    return v


if _hw_queues(sys.argv) is not None:
    os.environ["GPU_MAX_HW_QUEUES"] = _hw_queues(sys.argv)

METRIC = "verified+aggregated 3-of-4 threshold BLS sigs/sec at 1/2/4/8 MI355X"
# Best measured v_mad_u64_u32 rate on MI355X (tools/microbench/valu_rates.hip,
# profiles/r02/valu_rates.txt: 19.0 / 32.8 / 32.2 / 30.4 T lane-ops/s at
# 1 / 2 / 4 / 8 waves per SIMD); the 4-cycle issue model gives 39.3 T at
# 2.4 GHz (256 CU x 4 SIMD x 32 lanes / 2).  See DESIGN.md.
PEAK_MAD_TOPS = 32.8
# The clock-derived ceiling of a half-rate 64-bit multiply-add: 256 CU x 4
# SIMD x 16 lanes per cycle x 2.4 GHz (MI355X_MICROARCH.md gives no integer
# multiply peak); the measured 32.8 T is 83 % of it.  Both fractions are printed.
PEAK_MAD_TOPS_CLOCK = 39.3


def rank_env():
    """(world size, rank, local rank) from the launcher's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


_JSON_FD = None


def emit(obj) -> None:
    """Print the one JSON line (rank 0) on the process's original stdout."""
    line = (json.dumps(obj) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


def quiet_stdout() -> None:
    """Keep stdout for the JSON line alone: everything else the process
    writes to fd 1 (gloo's C++ connection messages among it) goes to stderr."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def dist_setup():
    """Join the rank group on gloo (CPU).  The ranks exchange only a barrier
    and the max of their elapsed times -- no data-path collective (DV-duties
    shard with no cross-GPU math) -- so nothing here touches the
    GPU: torch is imported for torch.distributed only, after the engine
    library holds the process's one HIP runtime."""
    ws, rank, local = rank_env()
    if ws > 1:
        quiet_stdout()
        import torch.distributed as dist
        dist.init_process_group(backend="gloo")
    return ws, rank, local


def launch_ranks(n: int, argv) -> int:
    """`--gpus N` without a launcher (WORLD_SIZE unset): start N fresh rank
    processes of this script, one per GPU (LOCAL_RANK = rank), with the
    environment torch.distributed.run would give them, before this process
    touches the GPU; wait for all of them and return the first failure's exit
    code (the others are stopped).  Rank 0 prints the JSON line."""
    import signal
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.send_signal(signal.SIGTERM)
    return rc


def barrier_sync(ws, sync=None):
    """Device synchronisation (the engine's streams) then the rank barrier;
    errors propagate."""
    if sync is not None:
        sync()
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, ws: int) -> float:
    if ws == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(step_fn, steps: int, ws: int, sync=None):
    """Barrier + sync on both sides of exactly `steps` steps; max over ranks."""
    barrier_sync(ws, sync)
    t0 = time.perf_counter()
    out = step_fn(steps)
    barrier_sync(ws, sync)
    dt = time.perf_counter() - t0
    return max_over_ranks(dt, ws), out


def launch_check(args):
    """--launch-check: the rank plumbing alone (no engine, no GPU): every rank
    joins the gloo group, runs a timed region of rank-dependent length, and
    rank 0 prints the ranks it saw with the max-over-ranks time."""
    ws, rank, local = dist_setup()

    def step(k):
        time.sleep(0.05 * (rank + 1) * k)
        return k

    dt, _ = timed_steps(step, args.steps, ws)
    seen = [(rank, local, os.getpid())]
    if ws > 1:
        import torch.distributed as dist
        allv = [None] * ws
        dist.all_gather_object(allv, seen[0])
        seen = allv
        dist.destroy_process_group()
    if rank == 0:
        emit({"launch_check": True, "n_gpus": ws, "ranks": [list(x) for x in seen],
                          "elapsed_max_s": round(dt, 4)})


def work_model():
    """Algorithmic u32 mul-add counts of the engine's per-item schedule,
    frozen by tools/count_work.py (host build with operation counters)."""
    path = os.path.join(ROOT, "profiles", "work_model.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


# Stages of the kernel chain (tbg_last_timings order) and their kernels.
STAGE_KERNELS = {
    "decode": ["k_decode_sigs", "k_sgb_sort", "k_sgb_bucket", "k_sgb_fold", "k_sgb_combine", "k_sgb_test", "k_subgroup_sigs"],
    "hash": ["k_hash_map", "k_hash_sswu", "k_hash_clear_x1", "k_hash_clear_x2", "k_hash_clear_fin", "k_hash_affine"],
    "combine": ["k_rlc_g1_l0", "k_msm_bucket", "k_msm_bucket_part", "k_msm_tree", "k_msm_tree_final", "k_msm_scan", "k_msm_scatter",
                "k_rlc_duty_sum<DSUM_L0_P>", "k_rlc_duty_sum<DSUM_BOTH>", "k_rlc_duty_sum<DSUM_FALLBACK_S>",
                "k_l0_lines", "k_rlc_partial2", "k_rlc_group_lines", "k_lines_fold<FOLD_GROUPS>",
                "k_rlc_g1", "k_rlc_duty_sum<DSUM_P>", "k_gm_sort", "k_gm_bucket", "k_gm_window", "k_gm_combine",
                "k_gm_failed_list", "k_rlc_partial2_list"],
    "h_lines": ["k_lines_h"],
    "verify": ["k_miller_hex<MILLER_L0>", "k_miller_hex<MILLER_GROUPS>", "k_miller_hex<MILLER_GROUP_S>", "k_l0_fold", "k_l0_tree", "k_l0_final", "k_l0_inv", "k_l0_fe", "k_l0_after",
               "k_rlc_group_final", "k_rlc_resolve_groups", "k_rlc_gident_lines", "k_lines_fold<FOLD_GID>",
               "k_rlc_gident_miller", "k_rlc_gident_check", "k_rlc_chunk_lines", "k_lines_fold<FOLD_CHUNKS>",
               "k_rlc_check_chunks", "k_rlc_cident_lines", "k_lines_fold<FOLD_CID>", "k_rlc_cident_check",
               "k_rlc_ident_lines", "k_lines_fold<FOLD_IDENT>", "k_rlc_ident_check", "k_lines_sig_list",
               "k_verify_list"],
    # (the speculative pass <true> runs mid-chain while level 0 is on; the
    # regular pass <false> then returns at once after a level-0 pass)
    "aggregate": ["k_lagrange<true>", "k_aggregate<true>", "k_aggregate_finish<true>", "k_aggregate_exc<true>",
                  "k_lagrange<false>", "k_aggregate<false>", "k_aggregate_finish<false>", "k_aggregate_exc<false>"],
}
# profile name (launch site) -> the symbol rocprofv3 prints for it
ROCPROF_NAME = {
    "k_miller_hex<MILLER_L0>": "void tbg::k_miller_hex<1>(tbg::DevBatch)",
    "k_miller_hex<MILLER_GROUPS>": "void tbg::k_miller_hex<0>(tbg::DevBatch)",
    "k_miller_hex<MILLER_GROUP_S>": "void tbg::k_miller_hex<2>(tbg::DevBatch)",
}
# one Fp product of the engine's 14 x 28-bit limbs = 392 u32 mul-adds (196 for
# the product, 196 for the REDC); SURVEY.md 8(d) prices one at 300 (12 x 32-bit
# CIOS): frac_fp300 states the same measured Fp-product rate on that basis
MADS_PER_FP_MUL = 392
SURVEY_MADS_PER_FP_MUL = 300


def rocprof_name(k):
    """The symbol rocprofv3 prints for a launch-site name."""
    return ROCPROF_NAME.get(k, "tbg::" + k + "(...)")


def traffic_key(k):
    """The key tools/pmc_traffic.py files a kernel under: rocprofv3's symbol
    without 'void tbg::' and the argument list (k_miller_hex<1>, k_lagrange<true>)."""
    return rocprof_name(k).split("(")[0].replace("void ", "").replace("tbg::", "")


def kernel_profile(prof):
    """[(kernel, ms)] of one device batch replayed alone -> {kernel: (ms, launches)}."""
    out = {}
    for name, ms in prof:
        t, n = out.get(name, (0.0, 0))
        out[name] = (t + ms, n + 1)
    return out


def launch_items(groups, shape):
    """Items of one device batch (the `merge` caller batches of a slot);
    `shape` = Engine.shape of its last submit (duties per group / chunk)."""
    nd = sum(b.n_dv for b in groups)
    np_ = sum(len(b.identifiers) for b in groups)
    nm = sum(len(b.msg_off) - 1 for b in groups)
    G = shape.get("group") or 16
    ng = -(-nd // G)  # level-1 groups are cut from the packed device batch
    chunks = shape.get("chunks") or ng * -(-G // 4)
    return {"partial": np_, "message": nm, "duty": nd, "group": ng, "chunk": chunks, "launch": 1}


def kernel_roofline(wm, kp, items, tm, batches):
    """roofline: the dominant kernel of one device batch replayed ALONE (every
    kernel timed by its own HIP event pair on its stream, tbg_replay_profile)
    -- its algorithmic u32 mul-adds (per-kernel work model of
    tools/count_work.py x the launch's items) / its measured duration."""
    if not wm or "kernels" not in wm:
        return None
    model = wm["kernels"]
    dom = max(kp, key=lambda k: kp[k][0])
    priced = [k for k in sorted(kp, key=lambda k: -kp[k][0]) if k in model]
    if not priced:
        return None
    k = dom if dom in model else priced[0]
    m = model[k]
    mads = m["mads"] * items[m["per"]] + sum(v * items[u] for u, v in m.get("plus", {}).items()) \
        + m.get("plus_per_launch", 0)
    ms, launches = kp[k]
    ach = mads / (ms * 1e-3) / 1e12
    traffic = None
    kk = (tm or {}).get("kernels", {}).get(traffic_key(k))
    if kk:
        traffic = int(1024 * (2 * kk.get("FETCH_SIZE_KB_per_launch", 0) + kk.get("WRITE_SIZE_KB_per_launch", 0))
                      * batches / max(1, tm.get("batches_per_launch", 1)))
    fp_mul_per_s = ach * 1e12 / MADS_PER_FP_MUL
    return {"bound": "valu-int-mul", "kernel": k, "rocprof_name": rocprof_name(k),
            "achieved": round(ach, 3), "peak": PEAK_MAD_TOPS, "unit": "T u32-mad/s",
            "frac": round(ach / PEAK_MAD_TOPS, 4),
            "frac_fp300": round(fp_mul_per_s * SURVEY_MADS_PER_FP_MUL / 1e12 / PEAK_MAD_TOPS, 4),
            "peak_clock_derived": PEAK_MAD_TOPS_CLOCK,
            "frac_clock_derived": round(ach / PEAK_MAD_TOPS_CLOCK, 4),
            "frac_fp300_clock_derived": round(fp_mul_per_s * SURVEY_MADS_PER_FP_MUL / 1e12 / PEAK_MAD_TOPS_CLOCK, 4),
            "fp_mul_per_s": round(fp_mul_per_s, 1),
            "traffic": traffic, "traffic_unit": "bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, "
                                                "profiles/traffic_latest.json)" if traffic is not None else None,
            "algorithmic_mads_per_launch": int(mads), "work_model": f"{m['mads']} mads per {m['per']}"
            + "".join(f" + {v} per {u}" for u, v in m.get("plus", {}).items())
            + (f" + {m['plus_per_launch']} per launch" if m.get("plus_per_launch") else ""),
            "items_per_launch": items[m["per"]], "launch_ms": round(ms / launches, 4),
            "batches_per_launch": batches, "dominant_by_exclusive_time": dom,
            "measured": "HIP event pair around every kernel of ONE device batch replayed alone on its stream "
                        "(tbg_replay_profile, after the timed region); rocprofv3 --kernel-trace of the same "
                        "command: tools/roofline_from_trace.py"}


def pipeline_roofline(wm, value, l0, t, n, sgb=True, items=None):
    """roofline_pipeline: the whole chain, work model x rate (config 2 shape;
    `items` = launch_items of one launch: its level-0 P chunks, when the
    launch shape is not the model's G = 16, C = 4)."""
    if not wm or (t, n) != (3, 4):
        return None
    mm = wm["mads"]
    unit = mm["unit_3of4_l0" if l0 else "unit_3of4_rlc"]
    if l0 and items and "l0_chunk_base" in mm:  # P-chunk hexads (+ their fold products) per duty
        unit += (items["chunk"] / items["duty"] - 0.25) * (mm["l0_chunk_base"] + mm["quad_mul"])
    if not sgb:  # every signature's subgroup test alone
        unit += 4 * (wm["mads"]["decode_sig"] - wm["mads"]["decode_sig_batched_subgroup"])
    ach = value * unit / 1e12
    return {"bound": "valu-int-mul", "kernel": "the whole kernel chain (launches in flight together)",
            "achieved": round(ach, 3), "peak": PEAK_MAD_TOPS, "unit": "T u32-mad/s",
            "frac": round(ach / PEAK_MAD_TOPS, 4), "frac_clock_derived": round(ach / PEAK_MAD_TOPS_CLOCK, 4),
            "work_per_unit_mads": unit,
            "schedule": "level 0 (batch-wide check, bucket MSM)" if l0 else "level-1 groups",
            "reference_schedule_mads_per_unit": wm["mads"]["unit_3of4_single_lane_schedule"],
            "reference_schedule_equivalent_tmads": round(value * wm["mads"]["unit_3of4_single_lane_schedule"] / 1e12,
                                                         3)}


def traffic_model():
    """Per-kernel HBM bytes per launch from the committed PMC passes of this
    build (profiles/traffic_latest.json, written by tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "traffic_latest.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return None


def cpu_baseline(batch, seconds: float):
    """The oracle (CPU restatement, 'port') on a bounded sample of the same
    workload: whole DV-duties (n verifies + 1 combine), all host threads."""
    from tools.cpu_baseline import run_cpu_baseline
    return run_cpu_baseline(batch, seconds)


def api_pipeline(e, eng, batches, inflight, n_batches, merge):
    """Side measurement of the product path: n_batches batches pushed through
    tbg_submit_group (`merge` at a time, as a coalescing call site would) and
    tbg_collect, with up to `inflight` groups outstanding: host packing into
    pinned staging, H2D, the kernel chain, D2H and the unpacking all inside
    the clock.  Not the headline (inputs are not HBM-resident); every result
    is checked."""
    import collections
    pending = collections.deque()
    done = 0
    results = []  # (result, batch): checked after the clock stops (test work, not product work)
    groups = [batches[k:k + merge] for k in range(0, n_batches, merge)]

    def drain_one():
        nonlocal done
        ts, grp = pending.popleft()
        for t, b in zip(ts, grp):
            results.append((e.collect(t), b))
            done += b.n_dv

    # untimed pass over every slot first: a slot's first submit allocates its
    # pinned staging and device arenas (hipHostMalloc / hipMalloc of ~20 GB)
    for k in range(inflight):
        grp = [batches[(k * merge + j) % len(batches)] for j in range(merge)]
        pending.append((e.submit_group(eng.OP_VERIFY_AGGREGATE, [
            dict(duty_first=b.duty_first, sigs=b.sigs, identifiers=b.identifiers, msgs=(b.msg_data, b.msg_off),
                 duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold) for b in grp]), grp))
    while pending:
        drain_one()
    results.clear()
    done = 0
    t0 = time.perf_counter()
    for k in range(len(groups)):
        if len(pending) >= inflight:
            drain_one()
        grp = [batches[(k * merge + j) % len(batches)] for j in range(merge)]
        ts = e.submit_group(eng.OP_VERIFY_AGGREGATE, [
            dict(duty_first=b.duty_first, sigs=b.sigs, identifiers=b.identifiers, msgs=(b.msg_data, b.msg_off),
                 duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold) for b in grp])
        pending.append((ts, grp))
    while pending:
        drain_one()
    dt = time.perf_counter() - t0
    ok = all(batch_exact(r, b, eng) for r, b in results)
    return {"value": round(done / dt, 2), "unit": "DV-duties/s", "batches": done // batches[0].n_dv,
            "batches_per_submit": merge, "inflight": inflight, "exact": bool(ok),
            "path": "tbg_submit_group + tbg_collect (pinned staging, H2D, chain, D2H); results checked after the clock"}


def latency_probe(e_load, eng, load_plan, sizes=(1, 64, 1024, 10000), reps=(30, 30, 12, 6)):
    """Submit -> collect latency of small batches (the reference verifies a
    peer's set inside a 5 s handler context, core/parsigex/parsigex.go:70-71,
    and the local VC's submission synchronously, core/validatorapi/
    validatorapi.go:228-287; tbls.Verify of one partial is a one-duty batch):
    p50 / p99 over `reps` tbg_submit + tbg_collect of each size on an idle
    context, then again on a second context while the first replays the
    headline launches (`load_plan`) in a background thread.  Every result is
    checked; the first call of each size (arena allocation) is not counted."""
    import threading
    from tools.workload import make_batch
    e = eng.Engine(e_load.device, slots=2)  # + the express slot (tbg_config.express_partials)
    e_plain = eng.Engine(e_load.device, slots=2, express_partials=eng.EXPRESS_OFF)
    try:
        bs = {n: make_batch(e, n, 3, 4, seed=7000 + n, load=lambda pk: _load_both(e, e_plain, pk)) for n in sizes}

        def one(b, e=e):
            t0 = time.perf_counter()
            r = e.run(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                      duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
            dt = (time.perf_counter() - t0) * 1e3
            if not batch_exact(r, b, eng):
                raise RuntimeError("latency probe: result differs")
            return dt

        def series(e=e):
            out = {}
            for n, k in zip(sizes, reps):
                one(bs[n], e)
                t = np.array([one(bs[n], e) for _ in range(k)])
                out[str(n)] = {"p50_ms": round(float(np.percentile(t, 50)), 3),
                               "p99_ms": round(float(np.percentile(t, 99)), 3), "samples": k}
            return out

        idle = series()
        stop = threading.Event()

        def load():
            while not stop.is_set():
                e_load.replay_plan(*load_plan)

        th = threading.Thread(target=load, daemon=True)
        th.start()
        try:
            time.sleep(0.2)
            loaded = series()
            loaded_plain = series(e_plain)
        finally:
            stop.set()
            th.join()
        return {"idle": idle, "under_headline_load": loaded, "under_headline_load_no_express": loaded_plain,
                "path": "tbg_submit + tbg_collect of one VERIFY_AGGREGATE batch (3-of-4) on its own context "
                        "(batches up to 4096 partials on its high-priority express slot; *_no_express: a context "
                        "without one); load = the headline launches replayed on another context of the same GPU"}
    finally:
        e.close()
        e_plain.close()


def _load_both(e1, e2, pk):
    """Load pubshares into two contexts at the same ids (the latency probe's
    batches run on either)."""
    f1, st = e1.load_pubkeys(pk)
    f2, _ = e2.load_pubkeys(pk)
    assert f1 == f2
    return f1, st


def batch_exact(res, b, eng):
    """Every partial verifies iff it was not injected, every duty with t
    valid partials aggregates to the group signature, the others fail."""
    if not np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected):
        return False
    ok = res.duty_status == eng.DS_OK
    if not np.array_equal(ok, b.expect_ok):
        return False
    return bool(np.array_equal(res.agg[ok], b.group_sig[ok]))


def host_side(hs, duties, wall_s):
    """The host share of the multi-context product path, timed inside the
    library (tbg_multi_host_stats): CPU time of the sub-batch builds, the
    packing into pinned staging and the gather (copy-out + counts), and the
    DV-duty rate those would sustain spread over the box's 16 cores -- host
    side only, no scaling curve (the GPUs are not involved in the figure)."""
    ms = lambda ns: round(ns / 1e6, 3)  # noqa: E731
    cpu_ns = hs["build_ns"] + hs["ctx_pack_ns"] + hs["ctx_gather_ns"]
    return {
        "label": "host side only, no scaling curve",
        "duties": duties, "wall_ms": round(wall_s * 1e3, 3),
        "submit_wall_ms": ms(hs["submit_wall_ns"]), "collect_wall_ms": ms(hs["collect_wall_ns"]),
        "build_cpu_ms": ms(hs["build_ns"]), "pack_cpu_ms": ms(hs["ctx_pack_ns"]),
        "enqueue_cpu_ms": ms(hs["ctx_enqueue_ns"]), "gather_cpu_ms": ms(hs["ctx_gather_ns"]),
        "device_wait_ms": ms(hs["ctx_wait_ns"]),
        "dv_duties_per_host_cpu_s": round(duties / (cpu_ns / 1e9), 1) if cpu_ns else None,
        "dv_duties_per_s_on_16_cores": round(16 * duties / (cpu_ns / 1e9), 1) if cpu_ns else None,
        "workers": "persistent per-context host workers (tbls_multi.hip Pool); pack / gather per context",
    }


def config4_multi(args):
    """BASELINE config 4 through the one-process multi-device product path:
    the 1M-DV 3-of-4 batch (1 % invalid partials of every kind when
    --inject > 0) as `--multi-batches` caller batches handed to
    tbg_multi_submit_group, cut over `--multi-contexts` contexts (one per
    visible GPU, or several per GPU when fewer GPUs are visible -- on a
    one-GPU box eight contexts share it), gathered into caller order by
    tbg_multi_collect.  Host packing, H2D, the chains and D2H are all inside
    the clock (the product path, not HBM-resident); every result is checked."""
    from charon_amd import engine as eng
    from tools.workload import make_mixed_batch
    from charon_amd.shard import sub_batch
    ndev = max(1, eng.device_count())
    devs = [i % ndev for i in range(args.multi_contexts)]
    m = eng.MultiEngine(devs, slots=1)
    try:
        t0 = time.perf_counter()
        b = make_mixed_batch(m.context(0), args.dvs, seed=args.seed, inject=args.inject, thresholds=((3, 4),),
                             load=m.load_pubkeys)
        gen_s = time.perf_counter() - t0
        K = max(1, args.multi_batches)
        cuts = [args.dvs * k // K for k in range(K + 1)]
        calls, subs = [], []
        for k in range(K):
            sb = sub_batch(cuts[k], cuts[k + 1], b.duty_first, b.sigs, b.identifiers, pubkey_ids=b.pubkey_ids,
                           duty_threshold=b.threshold, msg_data=b.msg_data, msg_off=b.msg_off, duty_msg=b.duty_msg)
            subs.append(sb)
            calls.append(dict(duty_first=sb.duty_first, sigs=sb.sigs, identifiers=sb.identifiers,
                              msgs=(sb.msg_data, sb.msg_off), duty_msg=sb.duty_msg, pubkey_ids=sb.pubkey_ids,
                              duty_threshold=sb.duty_threshold))

        def one_round():
            ts = m.submit_group(eng.OP_VERIFY_AGGREGATE, calls)
            return [m.collect(t) for t in ts]

        res = one_round()  # untimed: the first round allocates every context's arenas
        rounds = max(1, args.steps)
        m.host_stats(reset=True)
        t0 = time.perf_counter()
        for _ in range(rounds):
            res = one_round()
        dt = time.perf_counter() - t0
        hs = m.host_stats()
        ps = np.concatenate([r.partial_status for r in res])
        ds = np.concatenate([r.duty_status for r in res])
        agg = np.concatenate([r.agg for r in res])
        ok = ds == eng.DS_OK
        exact = bool(np.array_equal(ps == eng.PS_VALID, ~b.injected) and np.array_equal(ok, b.expect_ok)
                     and np.array_equal(agg[ok], b.group_sig[ok]))
        return {"metric": METRIC, "value": round(args.dvs * rounds / dt, 2),
                "unit": "DV-duties/s (n verifies + 1 aggregate each)", "n_gpus": ndev, "steps": rounds,
                "warmup": 1, "ms_per_step": round(dt * 1e3 / rounds, 3), "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "u32 (Fp 14x28-bit limbs)",
                "data": f"synthetic (seeded, generated on the GPU), {args.inject:.2%} injected invalid partials",
                "config": {"workload": f"config4 via tbg_multi: {args.dvs}-DV 3-of-4 batch as {K} caller batches, "
                                       f"cut over {len(devs)} contexts on {ndev} GPU(s)",
                           "contexts": len(devs), "caller_batches": K,
                           "path": "tbg_multi_submit_group + tbg_multi_collect (host packing, PCIe, chains, "
                                   "gather); one step = the whole batch"},
                "exact": exact, "generation_s": round(gen_s, 1),
                "host_side": host_side(hs, args.dvs * rounds, dt)}
    finally:
        m.close()


WORKLOADS = {
    "config2": "config2: 3-of-4, {dvs} DVs x 1 attestation per GPU",
    "config3": "config3: 7-of-10, {dvs} DVs x 1 attestation per GPU",
    "config4": "config4: 3-of-4, {dvs}-DV shard per GPU of the 1M-DV batch",
    "config5": "config5: {dvs} mixed DV-duties per GPU (attestation / sync / randao / proposal, thresholds 3-of-4, "
               "5-of-7, 7-of-10), {inject:.0%} invalid partials of every kind",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one GPU each (default: WORLD_SIZE, else 1).  Without a launcher (WORLD_SIZE "
                         "unset) N > 1 starts N rank processes itself; under one, N must equal WORLD_SIZE")
    ap.add_argument("--launch-check", action="store_true",
                    help="run only the rank plumbing (gloo barrier, max-over-ranks) and print the ranks seen")
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--dvs", type=int, default=10000)
    ap.add_argument("--t", type=int, default=3)
    ap.add_argument("--n", type=int, default=4)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--inflight", type=int, default=3, help="engine slots replayed round-robin (launches in flight)")
    ap.add_argument("--merge", type=int, default=16,
                    help="caller batches per slot, submitted together as one device batch (tbg_submit_group)")
    ap.add_argument("--launches", type=int, default=0,
                    help="spread the timed steps over at least this many launches (default: one per slot)")
    ap.add_argument("--verify-mode", type=int, default=0, help="0 = RLC groups with fallback, 1 = per-partial checks")
    ap.add_argument("--split", type=lambda v: [int(x) for x in v.split(",")], default=None,
                    help="batches per launch of a plan whose total is that many steps (launch-size experiments)")
    ap.add_argument("--rlc-group", type=int, default=0, help="duties per RLC group (0 = engine default)")
    ap.add_argument("--rlc-chunk", type=int, default=0, help="duties per Miller quad (0 = engine default)")
    ap.add_argument("--streams-per-slot", type=int, default=0, help="1 (default) or 2")
    ap.add_argument("--latency", type=int, default=1, help="1: the small-batch latency side key (latency_probe)")
    ap.add_argument("--subgroup-batch", type=int, default=0,
                    help="tbg_config.subgroup_batch: 0 auto (batched G2 subgroup test while clean), 1 on, 2 off")
    ap.add_argument("--gident", type=int, default=0,
                    help="level 1g (tbg_config.gident): 0 off, 1 unresolved groups to level 3, 2 to level 1.5")
    ap.add_argument("--inject", type=float, default=None,
                    help="fraction of partials replaced by invalid ones (side measurement; the headline is 0; "
                         "config5 defaults to 0.01)")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (read at HIP init); default: the environment's / HIP's 4")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="config2",
                    help="config2: 10k 3-of-4 DVs per step (the headline); config3: 100k 7-of-10 DVs per step; "
                         "config4: each GPU's 125k-DV shard of the 1M-DV 3-of-4 batch; config5: 10k mixed duties "
                         "with 1%% invalid partials of every kind per step")
    ap.add_argument("--multi-contexts", type=int, default=0,
                    help="config4 only: run the 1M-DV batch through tbg_multi_* over this many contexts in ONE "
                         "process (one per visible GPU, repeated when fewer are visible) instead of the "
                         "per-rank 125k-DV shard")
    ap.add_argument("--multi-batches", type=int, default=8,
                    help="caller batches the 1M-DV batch is handed over as (tbg_multi_submit_group)")
    ap.add_argument("--api-batches", type=int, default=192,
                    help="batches pushed through the product path (tbg_submit / tbg_collect, host packing and PCIe "
                         "included) for the api_pipeline side key; 0 skips it")
    args = ap.parse_args()
    ws_env = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(ws_env) if ws_env else 1
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if ws_env is None and args.gpus > 1:
        # no launcher: this process only starts the ranks (it never touches the GPU)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if ws_env is not None and int(ws_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws_env} ranks were launched")
    if args.launch_check:
        launch_check(args)
        return
    if args.workload == "config4" and args.multi_contexts:
        if args.gpus != 1:
            sys.exit("bench.py: --multi-contexts drives every GPU from one process (no torch.distributed launch)")
        args.dvs = 1_000_000 if args.dvs == 10000 else args.dvs
        args.inject = 0.0 if args.inject is None else args.inject
        emit(config4_multi(args))
        return
    if args.workload == "config4":
        args.dvs, args.t, args.n = 125000, 3, 4
        args.inflight, args.merge = min(args.inflight, 2), 1  # ~19 GB of HBM per resident 125k-DV batch
    elif args.workload == "config3":
        args.dvs, args.t, args.n = 100000, 7, 10
        args.inflight, args.merge = min(args.inflight, 3), 1  # one 100k-DV batch (1M partials) per launch
    if args.inject is None:
        args.inject = 0.01 if args.workload == "config5" else 0.0
    if args.workload != "config2":
        args.api_batches = 0  # the product-path side key is measured on the headline shape

    # The engine library is loaded first: its HIP runtime (ROCm's
    # libamdhip64.so.7) is the one the process initialises; torch comes in
    # afterwards for torch.distributed on gloo only and never touches the GPU.
    from charon_amd import engine as eng
    from tools.workload import make_batch, make_mixed_batch
    ndev = eng.device_count()
    if ndev < 1:
        sys.exit("bench.py: no HIP device visible to the engine")
    ws, rank, local = dist_setup()
    # one GPU per rank (LOCAL_RANK); modulo the visible count so N ranks can
    # share one card on a one-GPU box (identity on an 8-GPU node)
    device = local % ndev
    # one slot more than the replayed launches: the product-path side key packs
    # the next group into it while `inflight` launches run (the replay uses
    # only the first `inflight` slots)
    e = eng.Engine(device, slots=max(args.inflight, 1) + (1 if args.api_batches else 0),
                   verify_mode=args.verify_mode, rlc_group=args.rlc_group,
                   rlc_chunk=args.rlc_chunk, streams_per_slot=args.streams_per_slot, gident=args.gident,
                   subgroup_batch=args.subgroup_batch)
    # `inflight` engine slots each hold `merge` independent caller batches
    # submitted together (tbg_submit_group: one device batch, one launch per
    # kernel for all of them) and stay resident; the timed region replays the
    # slots round-robin, so `merge` steps run per launch and `inflight`
    # launches overlap -- what back-to-back submits of a serving node do.
    M = max(1, args.merge)

    def mk(seed, inject):
        if args.workload == "config5":
            return make_mixed_batch(e, args.dvs, seed=seed, inject=inject)
        return make_batch(e, args.dvs, args.t, args.n, seed=seed, inject=inject)

    def as_call(b):
        return dict(duty_first=b.duty_first, sigs=b.sigs, identifiers=b.identifiers, msgs=(b.msg_data, b.msg_off),
                    duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)

    batches, tickets = [], []
    pcie_ms = None
    if args.verify_mode == 0 and args.inject > 0:
        # the adaptive group size (tbg_config.rlc_group = 0) follows the invalid
        # share of collected batches: one untimed pass puts it in the state a
        # node serving this traffic is in before the resident slots are built
        for b in [mk(args.seed + 999_983 + k, args.inject) for k in range(2)]:
            e.collect(e.submit(eng.OP_VERIFY_AGGREGATE, **as_call(b)))
    for j in range(args.inflight):
        group = [mk(args.seed + 1000 * rank + M * j + k, args.inject) for k in range(M)]
        ts = e.submit_group(eng.OP_VERIFY_AGGREGATE, [as_call(b) for b in group])
        for b, t in zip(group, ts):
            first = e.collect(t)
            if pcie_ms is None:
                pcie_ms = e.timings()["total"]
            if not batch_exact(first, b, eng):
                print(json.dumps({"error": "parity check failed on the bench batch"}), file=sys.stderr)
                sys.exit(2)
        batches.append(group)
        tickets.append(ts[0])

    def plan(n):
        """Launches for exactly n steps: the n batches split as evenly as the
        slots allow over L = max(ceil(n / M), min(inflight, n)) launches
        round-robin over the slots (a prefix of a packed device batch is a
        batch of its own), so a short run still has `inflight` launches
        overlapping instead of a full launch plus a small remainder."""
        if args.split and sum(args.split) == n and len(args.split) <= len(tickets) and max(args.split) <= M:
            return [tickets[k] for k in range(len(args.split))], [0 if x == M else x for x in args.split]
        L = max(-(-n // M), min(len(tickets), n), min(args.launches, n))
        base, extra = divmod(n, L)
        ts, ps = [], []
        for k in range(L):
            size = base + (1 if k < extra else 0)
            ts.append(tickets[k % len(tickets)])
            ps.append(0 if size == M else size)
        return ts, ps

    if args.warmup:
        e.replay_plan(*plan(args.warmup))
    kernel_ms = {}

    def step_fn(k):
        kernel_ms.update(e.replay_plan(*plan(k)))

    elapsed, _ = timed_steps(step_fn, args.steps, ws, sync=e.synchronize)
    # outputs of the timed replays must still be exact (every batch of every slot)
    exact_after = True
    for group, t0 in zip(batches, tickets):
        for k, b in enumerate(group):
            again = e.fetch(t0 + k, b.n_dv, len(b.identifiers))
            exact_after = exact_after and batch_exact(again, b, eng)
    if ws > 1:  # every rank's re-check, reported by rank 0
        import torch.distributed as dist
        allx = [None] * ws
        dist.all_gather_object(allx, {"rank": rank, "device": device, "exact": bool(exact_after)})
    else:
        allx = [{"rank": 0, "device": device, "exact": bool(exact_after)}]
    if not all(x["exact"] for x in allx):
        print(json.dumps({"error": "timed replays' outputs differ", "ranks": allx}), file=sys.stderr)
        sys.exit(3)
    b = batches[0][0]
    flat = [x for g in batches for x in g]
    group_used = e.stats(tickets[0])["group_size"]  # before api_pipeline reuses the slots (tickets expire)
    l0_state = e.level0(tickets[0])
    fallback = e.fallback(tickets[0])  # per-level fallback work of the slot's last run
    slot_dev, slot_pinned = e.slot_bytes(tickets[0])
    subgroup = e.subgroup(tickets[0])  # batched subgroup test of the slot's last run

    units = args.dvs * args.steps * ws
    value = units / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # Per-kernel pass (untimed): one resident device batch (`merge` batches)
    # replayed alone, an event pair around every kernel -- the exclusive
    # durations the roofline prices; the stage sums are isolated_batch_ms.
    kp = kernel_profile(e.replay_profile(tickets[0]))
    shape = e.shape(tickets[0])  # the shape that profiled replay ran (the whole device batch)
    iso = {st: round(sum(kp[k][0] for k in ks if k in kp), 3) for st, ks in STAGE_KERNELS.items()}
    iso["total"] = round(sum(v[0] for v in kp.values()), 3)
    wm = work_model()
    items = launch_items(batches[0], shape)
    roofline = kernel_roofline(wm, kp, items, traffic_model(), M)
    # the roofline is per GPU: whole-job rate / ranks against one GPU's peak
    roofline_pipeline = pipeline_roofline(wm, value / ws, l0_state == eng.L0_PASSED, args.t, args.n,
                                          subgroup["groups"] > 0, items) \
        if args.workload in ("config2", "config4") else None
    # (before api_pipeline: the load replays the resident launches)
    lat = latency_probe(e, eng, plan(3 * M)) if args.latency and rank == 0 and args.workload == "config2" else None
    # (reuses the engine's slots: after the replays and the isolated pass)
    api = api_pipeline(e, eng, flat, args.inflight + 1, args.api_batches, M) if args.api_batches else None

    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "DV-duties/s (n verifies + 1 aggregate each)",
        "n_gpus": ws, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32 (Fp 14x28-bit limbs)",
        "data": "synthetic (seeded shares/pubshares/signatures generated on the GPU)"
                + (f", {args.inject:.2%} injected invalid partials" if args.inject else ""),
        "config": {"workload": WORKLOADS[args.workload].format(dvs=args.dvs, inject=args.inject),
                   "partials_per_step_per_gpu": int(len(b.identifiers)), "parallelism": f"shard{ws}",
                   "inflight_launches": args.inflight, "batches_per_launch": M,
                   "rlc_group": group_used, "rlc_chunk": shape["chunk"], "gident": args.gident, "subgroup_batch": args.subgroup_batch,
                   "level0": {eng.L0_NOT_RUN: "not run", eng.L0_PASSED: "passed", eng.L0_FAILED: "failed"}[l0_state],
                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))},
        "ranks_exact_after_clock": allx,
        "fallback_levels": fallback,
        "subgroup_batch": subgroup,
        "slot_bytes": {"device": int(slot_dev), "pinned_host": int(slot_pinned), "batches_per_slot": M},
        "kernel_ms_per_step": {k: round(v / args.steps, 3) for k, v in kernel_ms.items()},
        "pcie_inclusive_ms_first_batch": round(pcie_ms, 3),
        "api_pipeline": api,
        "small_batch_latency": lat,
        "isolated_batch_ms": iso,
        "isolated_kernel_ms": {k: round(v[0], 4) for k, v in sorted(kp.items(), key=lambda kv: -kv[1][0])
                               if v[0] >= 0.05},
        "roofline": roofline,
        "roofline_pipeline": roofline_pipeline,
        "cpu_baseline": None,
        "host_signing_roots": None,
    }
    if rank == 0:
        # the host step in front of the GPU path: AttestationData -> signing
        # root (include/tbls_ssz.h), 16 threads -- must outpace `value`
        from tools.ssz_bench import run_rate
        result["host_signing_roots"] = run_rate(1 << 18, 16, reps=2)
    if rank == 0 and not args.no_cpu and ws == 1 and args.workload in ("config2", "config3", "config4"):
        result["cpu_baseline"] = cpu_baseline(b, args.cpu_seconds)
    if rank == 0:
        emit(result)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    e.close()


if __name__ == "__main__":
    main()
