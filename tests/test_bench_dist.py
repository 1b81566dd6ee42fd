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
                      MASTER_PORT=str(port))
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


def _bench(args, env_extra=None, timeout=180):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_gpus_n_without_launcher_spawns_n_ranks():
    """`bench.py --gpus 2` with WORLD_SIZE unset starts two
    rank processes itself (gloo barrier, max over ranks); rank 0 prints one
    JSON line naming both ranks, each its own process on LOCAL_RANK = rank."""
    import json
    r = _bench(["--gpus", "2", "--steps", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout  # stdout carries the JSON line alone (gloo's own messages go to stderr)
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    ranks = sorted(tuple(x) for x in out["ranks"])
    assert [(x[0], x[1]) for x in ranks] == [(0, 0), (1, 1)]
    assert ranks[0][2] != ranks[1][2]  # two processes
    assert out["elapsed_max_s"] >= 0.2  # the slower rank's 2 x 0.1 s


def test_gpus_must_match_world_size():
    """Under a launcher --gpus N must equal WORLD_SIZE (a mismatch would time
    one GPU and call it N)."""
    r = _bench(["--gpus", "8", "--launch-check"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_roofline_fields_from_work_model():
    """bench.py's roofline arithmetic (no GPU): the dominant kernel by
    exclusive time is priced with its own per-item work model x the launch's
    items over its measured duration; the pipeline form is units/s x the
    algorithmic mul-adds per unit."""
    import types
    import numpy as np
    import bench
    wm = bench.work_model()
    assert wm is not None and "kernels" in wm
    b = types.SimpleNamespace(n_dv=10000, identifiers=np.zeros(40000), msg_off=np.zeros(10001))
    items = bench.launch_items([b] * 16, {"group": 16, "chunk": 4, "level0": 1, "chunks": 40000})
    assert items == {"partial": 640000, "message": 160000, "duty": 160000, "group": 10000, "chunk": 40000,
                     "launch": 1}
    # the level-0 launch shape (16, 8): half the P chunks, same duties
    items8 = bench.launch_items([b] * 16, {"group": 16, "chunk": 8, "level0": 1, "chunks": 20000})
    assert items8["chunk"] == 20000 and items8["group"] == 10000
    prof = [("k_decode_sigs", 9.0), ("k_subgroup_sigs", 13.4), ("k_miller_hex<MILLER_L0>", 15.9),
            ("k_miller_hex<MILLER_GROUP_S>", 0.005), ("k_msm_sum", 0.4), ("k_msm_sum", 0.1)]
    kp = bench.kernel_profile(prof)
    assert kp["k_msm_sum"] == (0.5, 2)
    # the PMC model files kernels under rocprofv3's symbol (k_miller_hex<1>):
    # the dominant kernel's traffic is found by that key and scaled per launch
    tm = {"batches_per_launch": 16, "kernels": {"k_miller_hex<1>": {"FETCH_SIZE_KB_per_launch": 100.0,
                                                                     "WRITE_SIZE_KB_per_launch": 10.0}}}
    r = bench.kernel_roofline(wm, kp, items, tm, 16)
    m = wm["kernels"]["k_miller_hex<MILLER_L0>"]
    mads = m["mads"] * 40000 + m["plus"]["duty"] * 160000 + m["plus_per_launch"]
    # the per-chunk + per-duty form equals count_work's measured 4-duty chunk
    assert abs(4 * m["plus"]["duty"] + m["mads"] - wm["mads"]["rlc_miller_chunk"]) <= 4
    assert r["kernel"] == "k_miller_hex<MILLER_L0>" == r["dominant_by_exclusive_time"]
    assert r["rocprof_name"] == "void tbg::k_miller_hex<1>(tbg::DevBatch)"
    assert r["traffic"] == 1024 * 210
    assert abs(r["frac_fp300"] - r["frac"] * 300 / 392) < 1e-3
    assert bench.traffic_key("k_lagrange<true>") == "k_lagrange<true>"
    assert bench.traffic_key("k_miller_hex<MILLER_GROUP_S>") == "k_miller_hex<2>"
    assert r["algorithmic_mads_per_launch"] == mads
    assert abs(r["achieved"] - mads / 15.9e-3 / 1e12) < 1e-2
    assert abs(r["frac"] - r["achieved"] / bench.PEAK_MAD_TOPS) < 1e-3
    # an unpriced dominant kernel falls to the longest priced one, and says so
    kp2 = dict(kp, k_mystery=(99.0, 1))
    r2 = bench.kernel_roofline(wm, kp2, items, None, 16)
    assert r2["dominant_by_exclusive_time"] == "k_mystery" and r2["kernel"] == "k_miller_hex<MILLER_L0>"
    pipe = bench.pipeline_roofline(wm, 1.0e6, True, 3, 4)
    assert abs(pipe["achieved"] - 1.0e6 * wm["mads"]["unit_3of4_l0"] / 1e12) < 1e-2
    assert bench.pipeline_roofline(wm, 1.0e6, True, 3, 4, items=items)["achieved"] == pipe["achieved"]
    # 8-duty chunks: fewer squarings per duty, less algorithmic work per unit
    pipe8 = bench.pipeline_roofline(wm, 1.0e6, True, 3, 4, items=items8)
    assert pipe8["work_per_unit_mads"] < pipe["work_per_unit_mads"]
    assert 0 < pipe["frac"] < 1
    assert bench.pipeline_roofline(wm, 1.0e6, True, 7, 10) is None


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
