"""Sharding and gather order across processes (world_size 2, gloo on CPU).

Each rank takes its contiguous duty range of one batch (charon_amd.shard, the
rule tbg_multi_submit uses inside the library), runs it through the C oracle
(the CPU checker; no GPU here) as its own sub-batch -- messages re-indexed,
duty_first rebased -- and the ranks' results are gathered on rank 0 back into
caller order.  The gathered arrays must equal the golden fixtures of the
whole batch, which mixes thresholds, duties sharing nothing and every
injected failure kind (cfg5 / va_id_modes / cfg2)."""
import json
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
PS = {"valid": 1, "invalid": 0, "err_flags": -1, "err_field": -2, "err_curve": -3, "err_subgroup": -4,
      "err_identity": -5, "err_pubkey": -6}
DS = {"ok": 0, "insufficient": -20, "insufficient_valid": -21}


def _batch():
    vecs = []
    for name in ("cfg5_mixed_invalid.json", "va_id_modes.json", "cfg2_3of4_sample.json"):
        with open(os.path.join(HERE, "golden", name)) as f:
            vecs += json.load(f)["vectors"][:12]
    pks, sigs, ids, pk_ids, duty_first, thr = [], [], [], [], [0], []
    for v in vecs:
        for p in v["partials"]:
            sigs.append(bytes.fromhex(p["sig"]))
            ids.append(p["identifier"])
            share = v["tss"]["pubshares"].get(str(p["identifier"]))
            pk_ids.append(0xFFFFFFFF if share is None else len(pks))
            if share is not None:
                pks.append(bytes.fromhex(share))
        duty_first.append(duty_first[-1] + len(v["partials"]))
        thr.append(v["tss"]["threshold"])
    # two duties share each signing root where the fixture allows it: here every
    # duty has its own; make the message table non-trivial by reversing it
    msgs = [bytes.fromhex(v["msg"]) for v in vecs][::-1]
    duty_msg = np.arange(len(vecs))[::-1].copy()
    off = np.concatenate([[0], np.cumsum([len(m) for m in msgs])])
    return dict(vecs=vecs, pks=b"".join(pks), sigs=np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 96),
                ids=np.array(ids, np.uint8), pk_ids=np.array(pk_ids, np.uint32), duty_first=np.array(duty_first),
                thr=np.array(thr, np.uint32), msg_data=np.frombuffer(b"".join(msgs) + b"\0", np.uint8), msg_off=off,
                duty_msg=duty_msg)


def _rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from charon_amd import shard
        from oracle import c as oc
        b = _batch()
        lo = shard.shard_bounds(b["duty_first"], world)
        sb = shard.sub_batch(lo[rank], lo[rank + 1], b["duty_first"], b["sigs"], b["ids"], pubkey_ids=b["pk_ids"],
                             duty_threshold=b["thr"], msg_data=b["msg_data"], msg_off=b["msg_off"],
                             duty_msg=b["duty_msg"])
        table = oc.PubkeyTable(b["pks"])
        res = oc.run(3, sb.duty_first, sb.sigs, sb.identifiers, table, msgs=sb.msg_data, msg_off=sb.msg_off,
                     duty_msg=sb.duty_msg, pubkey_ids=sb.pubkey_ids, duty_threshold=sb.duty_threshold)
        parts = [None] * world
        dist.all_gather_object(parts, (sb, *res))
        if rank == 0:
            nd = len(b["duty_first"]) - 1
            ps, ds, agg = shard.gather(parts, nd, int(b["duty_first"][-1]))
            ok = True
            for d, v in enumerate(b["vecs"]):
                exp = v["expect"]
                lo_, hi_ = b["duty_first"][d], b["duty_first"][d + 1]
                if exp["status"] != "insufficient":
                    ok &= ps[lo_:hi_].tolist() == [PS[s] for s in exp["partial_status"]]
                ok &= int(ds[d]) == DS.get(exp["status"], 99)
                if exp["status"] == "ok":
                    ok &= bytes(agg[d]).hex() == exp["agg"]
            out.put((ok, lo))
    finally:
        dist.destroy_process_group()


def test_two_rank_shard_gather_matches_whole_batch():
    from oracle import c as oc
    oc.build()
    import random
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, lo = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert 0 < lo[1] < lo[2], lo
    assert ok


def test_shard_bounds_rules():
    from charon_amd.shard import shard_bounds
    assert shard_bounds([0, 4, 4, 8], 4) == [0, 1, 1, 3, 3]          # an empty duty never opens a shard
    assert shard_bounds([0, 0, 0, 0], 2) == [0, 1, 3]                # no partials: duties split evenly
    assert shard_bounds(np.arange(11) * 4, 3) == [0, 4, 7, 10]       # 40 partials: cuts at 13, 26
    lo = shard_bounds(np.cumsum([0] + [4, 7, 10] * 50), 8)
    assert lo[0] == 0 and lo[-1] == 150 and all(a <= b for a, b in zip(lo, lo[1:]))


def test_group_shard_bounds_cut_the_concatenation():
    """tbg_multi_submit_group's cut (host mirror): several caller batches taken
    back to back are cut like ONE batch, each ticket's layout is that cut
    clamped to its own duties, and empty / zero-partial batches stay valid."""
    from charon_amd.shard import group_shard_bounds, shard_bounds
    rng = np.random.default_rng(5)
    for trial in range(200):
        k = int(rng.integers(1, 6))
        dfs = []
        for _ in range(k):
            nd = int(rng.integers(1, 40))
            counts = rng.integers(0, 11, size=nd) * (rng.random(nd) < 0.9)
            dfs.append(np.concatenate([[0], np.cumsum(counts)]))
        n = int(rng.integers(1, 10))
        lays = group_shard_bounds(dfs, n)
        glob = np.concatenate([d[:-1] + off for d, off in zip(dfs, np.cumsum([0] + [int(d[-1]) for d in dfs])[:-1])]
                              + [[sum(int(d[-1]) for d in dfs)]])
        cut = shard_bounds(glob, n)
        base = 0
        for d, lo in zip(dfs, lays):
            nd = len(d) - 1
            assert len(lo) == n + 1 and lo[0] == 0 and lo[-1] == nd
            assert all(a <= b for a, b in zip(lo, lo[1:]))
            assert lo == [min(max(c - base, 0), nd) for c in cut]
            base += nd
    # the config-4 shape: four batches of 1M 3-of-4 DVs -> eight 125k-DV shards
    dfs = [np.arange(n + 1) * 4 for n in (400_000, 250_000, 250_000, 100_000)]
    lays = group_shard_bounds(dfs, 8)
    assert lays[0] == [0, 125_000, 250_000, 375_000] + [400_000] * 5
    assert lays[3] == [0] * 8 + [100_000]
