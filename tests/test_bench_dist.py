"""bench.py's multi-process plumbing (barrier, max-over-ranks timing, weak
scaling value) with world_size 2 on the gloo backend (CPU)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), TBG_DIST_BACKEND="gloo")
    import time
    import bench
    w, r, _ = bench.dist_setup()
    assert (w, r) == (ws, rank)

    def step(k):
        time.sleep(0.05 * (rank + 1) * k)  # rank 1 is slower: max over ranks must see it
        return k

    dt, out = bench.timed_steps(step, 2, ws)
    q.put((rank, dt, out))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_two_rank_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dts = {r: dt for r, dt, _ in res}
    # both ranks report the same (max) elapsed time, at least the slow rank's 0.2 s
    assert abs(dts[0] - dts[1]) < 1e-9
    assert dts[0] >= 0.2


def test_roofline_fields_from_work_model():
    """bench.py's roofline arithmetic (no GPU): the pipelined chain's
    achieved rate is units/s x algorithmic mul-adds per unit; the isolated
    stage's is its mul-adds per launch / its launch time."""
    import argparse
    import bench
    wm = bench.work_model()
    assert wm is not None
    args = argparse.Namespace(dvs=10000, t=3, n=4, merge=16)
    iso = {"decode": 22.8, "hash": 16.6, "combine": 28.4, "h_lines": 6.5, "verify": 41.2, "aggregate": 2.8}
    timed = {k: 3 * 1.5 * v for k, v in iso.items()}  # 3 launches of 16 batches, 1.5x slower when shared
    stage, iso_r, pipe = bench.stage_rooflines(wm, iso, timed, args, 1.0e6, 48)
    assert stage["kernel"].startswith("verify stage") and iso_r["kernel"].startswith("verify stage")
    # timed-region form: work of the 48 steps over the summed launch time
    assert abs(stage["achieved"] - stage["algorithmic_mads_per_launch"] * 3 / (timed["verify"] * 1e-3) / 1e12) < 1e-2
    assert abs(iso_r["achieved"] - iso_r["algorithmic_mads_per_launch"] / 41.2e-3 / 1e12) < 1e-2
    assert abs(iso_r["achieved"] / stage["achieved"] - 1.5) < 1e-3
    assert abs(pipe["achieved"] - 1.0e6 * wm["mads"]["unit_3of4_rlc"] / 1e12) < 1e-2
    assert 0 < pipe["frac"] < 1


def test_batch_exact_follows_injection():
    """bench.py's exactness check under --inject (no GPU): a partial must
    verify iff it was not injected, a duty aggregates iff it kept t valid
    partials, and only those duties' aggregates are compared."""
    import types
    import numpy as np
    import bench
    eng = types.SimpleNamespace(PS_VALID=1, DS_OK=0)
    injected = np.array([False, True, False, False, True, True, False, False])  # 2 duties x 4
    expect_ok = np.array([True, False])                                      # t = 3
    group_sig = np.arange(2 * 96, dtype=np.uint8).reshape(2, 96)
    b = types.SimpleNamespace(injected=injected, expect_ok=expect_ok, group_sig=group_sig)
    agg = group_sig.copy()
    agg[1] = 0  # a failed duty's aggregate is not compared
    good = types.SimpleNamespace(partial_status=np.where(injected, 0, 1).astype(np.int32),
                                 duty_status=np.array([0, 3], dtype=np.int32), agg=agg)
    assert bench.batch_exact(good, b, eng)
    flipped = types.SimpleNamespace(**{**vars(good), "partial_status": np.ones(8, dtype=np.int32)})
    assert not bench.batch_exact(flipped, b, eng)
    wrong_duty = types.SimpleNamespace(**{**vars(good), "duty_status": np.zeros(2, dtype=np.int32)})
    assert not bench.batch_exact(wrong_duty, b, eng)
    bad_agg = agg.copy()
    bad_agg[0, 5] ^= 1
    assert not bench.batch_exact(types.SimpleNamespace(**{**vars(good), "agg": bad_agg}), b, eng)
