"""Full-size GPU parity against the C oracle (oracle/c, the checker) and the
single-process multi-device path (BASELINE config 4).

Every test runs the HIP engine through the C ABI on a batch of BASELINE size
and compares per-partial status, per-duty status and every 96-byte aggregate
bit-exactly with oracle/c's restatement of the reference per-item schedule
(tbls.VerifyAndAggregate, tss.go:153-187) on the same inputs:

  * config 2: 10,000 DVs, 3-of-4, one signing root each;
  * config 3: 10,000 DVs, 7-of-10 (a 10k slice of the 100k configuration);
  * config 5: 10,000 DVs, thresholds {3/4, 5/7, 7/10}, mixed duties with
    committee-shared signing roots, 1 % of partials replaced by every invalid
    kind the reference rejects (tools/workload.INJECT_KINDS);
  * config 4: a 125,000-DV 3-of-4 shard with 1 % mixed injections through
    tbg_multi_* with 3 contexts mapped onto the visible device(s), gathered
    results bit-exact against per-shard single-context runs and against
    oracle/c on a 10,000-DV slice.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share


@pytest.fixture(scope="module")
def engine():
    from charon_amd import engine as eng
    e = eng.Engine(0, slots=2)
    yield e
    e.close()


def oracle_run(b, d0=0, d1=None):
    """oracle/c over duties [d0, d1) of a workload batch (statuses, aggregates)."""
    from oracle import c as oc
    oc.build()
    d1 = b.n_dv if d1 is None else d1
    p0, p1 = int(b.duty_first[d0]), int(b.duty_first[d1])
    pk_ids = np.asarray(b.pubkey_ids[p0:p1], dtype=np.int64)
    # the oracle's table holds the slice's pubshares only (decoding every key of
    # a 1M-partial batch on the host would dominate the test), indexed from 0
    known = pk_ids != 0xFFFFFFFF
    used = np.unique(pk_ids[known] - b.pk_first)
    rel = np.full(len(pk_ids), 0xFFFFFFFF, dtype=np.uint32)
    rel[known] = np.searchsorted(used, pk_ids[known] - b.pk_first).astype(np.uint32)
    table = oc.PubkeyTable(np.asarray(b.pubshares, dtype=np.uint8)[used])
    used = np.unique(b.duty_msg[d0:d1])
    remap = {int(m): i for i, m in enumerate(used)}
    msgs = b"".join(b.msgs[m] for m in used)
    off = np.arange(len(used) + 1, dtype=np.uint32) * 32
    duty_msg = np.array([remap[int(m)] for m in b.duty_msg[d0:d1]], dtype=np.uint32)
    return oc.run(3, np.asarray(b.duty_first[d0:d1 + 1], dtype=np.int64) - p0, b.sigs[p0:p1], b.identifiers[p0:p1],
                  table, msgs=np.frombuffer(msgs, np.uint8), msg_off=off, duty_msg=duty_msg, pubkey_ids=rel,
                  duty_threshold=b.threshold[d0:d1], threads=THREADS)


def engine_run(e, b):
    from charon_amd import engine as eng
    return e.run(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                 duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)


def assert_same(res, ref, lo=0, hi=None, plo=0):
    ps, ds, agg = ref
    hi = len(ds) + lo if hi is None else hi
    n = len(ps)
    assert np.array_equal(res.partial_status[plo:plo + n], ps), np.flatnonzero(res.partial_status[plo:plo + n] != ps)[:8]
    assert np.array_equal(res.duty_status[lo:hi], ds), np.flatnonzero(res.duty_status[lo:hi] != ds)[:8]
    assert np.array_equal(res.agg[lo:hi], agg)


def test_config2_full_batch_matches_oracle(engine):
    from tools.workload import make_batch
    b = make_batch(engine, 10000, 3, 4, seed=202)
    res = engine_run(engine, b)
    assert_same(res, oracle_run(b))
    assert (res.duty_status == 0).all()
    assert np.array_equal(res.agg, b.group_sig)


def test_config3_7of10_matches_oracle(engine):
    from tools.workload import make_batch
    b = make_batch(engine, 10000, 7, 10, seed=303, inject=0.01)
    res = engine_run(engine, b)
    assert_same(res, oracle_run(b))
    ok = res.duty_status == 0
    assert np.array_equal(ok, b.expect_ok) and np.array_equal(res.agg[ok], b.group_sig[ok])


def test_config5_mixed_injections_match_oracle(engine):
    from charon_amd import engine as eng
    from tools.workload import INJECT_KINDS, make_mixed_batch
    b = make_mixed_batch(engine, 10000, seed=505, inject=0.01)
    res = engine_run(engine, b)
    assert_same(res, oracle_run(b))
    # every kind was injected and none verified
    st = res.partial_status[b.injected]
    assert len(st) > 8 * len(INJECT_KINDS) and not (st == eng.PS_VALID).any()
    for code in (eng.PS_INVALID, eng.PS_ERR_SUBGROUP, eng.PS_ERR_CURVE, eng.PS_ERR_FLAGS, eng.PS_ERR_IDENTITY,
                 eng.PS_ERR_PUBKEY):
        assert (st == code).any(), code
    assert (res.partial_status[~b.injected] == eng.PS_VALID).all()
    ok = res.duty_status == 0
    assert np.array_equal(ok, b.expect_ok) and np.array_equal(res.agg[ok], b.group_sig[ok])


def test_multi_device_config4_shard(engine):
    """Config 4's 125k-DV shard through tbg_multi_* (3 contexts on the visible
    device(s)): the gathered results equal per-shard single-context runs
    bit-exactly, and oracle/c on a 10k-DV slice."""
    from charon_amd import engine as eng
    from tools.workload import make_mixed_batch
    ndev = max(1, eng.device_count())
    m = eng.MultiEngine([i % ndev for i in range(3)], slots=1)
    try:
        b = make_mixed_batch(engine, 125000, seed=404, inject=0.01, thresholds=((3, 4),), load=m.load_pubkeys)
        # the single context needs the same pubkey ids: load the table there too
        first, _ = engine.load_pubkeys(b.pubshares)
        shift = np.int64(first) - np.int64(b.pk_first)
        t = m.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                     duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
        lo = m.layout(t)
        assert lo == eng.shard_bounds(b.duty_first, 3)
        res = m.collect(t)
        # per-shard single-context runs
        pk_single = np.where(b.pubkey_ids == 0xFFFFFFFF, b.pubkey_ids, b.pubkey_ids.astype(np.int64) + shift)
        for i in range(3):
            d0, d1 = lo[i], lo[i + 1]
            p0, p1 = int(b.duty_first[d0]), int(b.duty_first[d1])
            used = np.unique(b.duty_msg[d0:d1])
            remap = np.zeros(int(b.duty_msg.max()) + 1, dtype=np.uint32)
            remap[used] = np.arange(len(used), dtype=np.uint32)
            r1 = engine.run(eng.OP_VERIFY_AGGREGATE, b.duty_first[d0:d1 + 1] - p0, b.sigs[p0:p1],
                            b.identifiers[p0:p1], msgs=[b.msgs[k] for k in used], duty_msg=remap[b.duty_msg[d0:d1]],
                            pubkey_ids=pk_single[p0:p1].astype(np.uint32), duty_threshold=b.threshold[d0:d1])
            assert np.array_equal(res.partial_status[p0:p1], r1.partial_status), i
            assert np.array_equal(res.duty_status[d0:d1], r1.duty_status), i
            assert np.array_equal(res.agg[d0:d1], r1.agg), i
        # the oracle on a 10k-DV slice that straddles the first cut
        s0 = max(0, lo[1] - 5000)
        assert_same(res, oracle_run(b, s0, s0 + 10000), s0, s0 + 10000, int(b.duty_first[s0]))
        ok = res.duty_status == 0
        assert np.array_equal(ok, b.expect_ok) and np.array_equal(res.agg[ok], b.group_sig[ok])
        assert not (res.partial_status[b.injected] == eng.PS_VALID).any()
    finally:
        m.close()


def test_multi_device_poll_and_uneven_shards(engine):
    """More contexts than duties, empty partial lists, polling collect."""
    import time
    from charon_amd import engine as eng
    from tools.workload import make_batch
    m = eng.MultiEngine([0, 0, 0, 0], slots=1)
    try:
        b = make_batch(engine, 3, 3, 4, seed=9, load=m.load_pubkeys)
        t = m.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                     duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
        assert m.layout(t) == eng.shard_bounds(b.duty_first, 4)
        deadline = time.time() + 60
        res = None
        while res is None and time.time() < deadline:
            res = m.collect(t, block=False)
        assert res is not None
        assert (res.duty_status == 0).all() and np.array_equal(res.agg, b.group_sig)
        # OP_AGGREGATE with a duty of zero partials among non-empty ones
        df = np.array([0, 4, 4, 8])
        sig = np.concatenate([b.sigs[0:4], b.sigs[4:8]])
        r = m.run(eng.OP_AGGREGATE, df, sig, np.concatenate([b.identifiers[0:4], b.identifiers[4:8]]))
        assert r.duty_status[1] == eng.DS_AGG_TOO_FEW
        assert np.array_equal(r.agg[[0, 2]], b.group_sig[:2])
    finally:
        m.close()


def test_g1_pubkey_rejections_match_oracle(engine):
    """tblsconv.KeyFromBytes (tblsconv.go:30-37): every rejection class of the
    48-byte pubshare decode equals the oracle's, and the startup wiring
    (app/app.go:345-354) aborts on the first bad pubshare."""
    import json
    from charon_amd import tbls
    with open(os.path.join(os.path.dirname(__file__), "golden", "g1_pubkeys.json")) as f:
        vecs = json.load(f)["vectors"]
    names = {0: "valid", 1: "identity", -1: "err_flags", -2: "err_field", -3: "err_curve", -4: "err_subgroup"}
    _, st = engine.load_pubkeys(b"".join(bytes.fromhex(v["pk"]) for v in vecs))
    assert [names[s] for s in st.tolist()] == [v["expect"] for v in vecs]
    keys = tbls.key_from_bytes_batch([bytes.fromhex(v["pk"]) for v in vecs], engine)
    for k, v in zip(keys, vecs):
        if v["expect"] == "valid":
            assert isinstance(k, tbls.PublicKey)
        else:
            assert isinstance(k, tbls.TblsError) and str(k).startswith("unmarshal pubkey")
    good = [bytes.fromhex(v["pk"]) for v in vecs if v["expect"] == "valid"]
    wired = tbls.wire_pubshares({b"dv0": good[:2], b"dv1": good[2:4]}, engine)
    assert sorted(wired[b"dv1"]) == [1, 2]
    bad = bytes.fromhex(next(v["pk"] for v in vecs if v["expect"] == "err_subgroup"))
    with pytest.raises(tbls.TblsError, match="unmarshal pubkey"):
        tbls.wire_pubshares({b"dv0": good[:2], b"dv1": [good[2], bad]}, engine)


def test_submit_group_matches_single_batches(engine):
    """tbg_submit_group packs several callers' batches into one device batch:
    every ticket's statuses and aggregates equal that batch submitted alone
    (index rebasing of duties, partials and messages), including a mixed
    batch whose messages are shared within it, and a single-duty batch."""
    from charon_amd import engine as eng
    from tools.workload import make_batch, make_mixed_batch
    parts = [make_batch(engine, 700, 3, 4, seed=71, inject=0.02), make_mixed_batch(engine, 900, seed=72, inject=0.02),
             make_batch(engine, 1, 7, 10, seed=73), make_batch(engine, 333, 5, 7, seed=74, inject=0.05)]
    args = [dict(duty_first=b.duty_first, sigs=b.sigs, identifiers=b.identifiers, msgs=(b.msg_data, b.msg_off),
                 duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold) for b in parts]
    tickets = engine.submit_group(eng.OP_VERIFY_AGGREGATE, args)
    assert len(set(tickets)) == len(parts)
    # collect out of order
    got = {t: engine.collect(t) for t in reversed(tickets)}
    # prefix replays of the packed device batch (tbg_replay_plan) leave every
    # ticket's results intact (before other submits reuse the slot)
    engine.replay_plan([tickets[0], tickets[0], tickets[0]], [1, 3, 0])
    for b, t in zip(parts, tickets):
        again = engine.fetch(t, b.n_dv, int(b.duty_first[-1]))
        assert np.array_equal(again.partial_status, got[t].partial_status)
        assert np.array_equal(again.agg, got[t].agg)
    for b, a, t in zip(parts, args, tickets):
        alone = engine.run(eng.OP_VERIFY_AGGREGATE, **a)
        g = got[t]
        assert np.array_equal(g.partial_status, alone.partial_status)
        assert np.array_equal(g.duty_status, alone.duty_status)
        assert np.array_equal(g.agg, alone.agg)
        ok = g.duty_status == 0
        assert np.array_equal(ok, b.expect_ok) and np.array_equal(g.agg[ok], b.group_sig[ok])
    # an empty group is refused (and nothing is left pending)
    with pytest.raises(eng.EngineError):
        engine.submit_group(eng.OP_VERIFY_AGGREGATE, [])


@pytest.mark.parametrize("cfg", [
    dict(verify_mode=1),                                                     # level 3 only
    dict(verify_mode=0, rlc_group=8, rlc_chunk=2, rlc_batch=2, rlc_seed=0x64),  # 1 -> 1.5 -> 1.5b -> 2b -> 3
    dict(verify_mode=0, rlc_group=16, rlc_batch=2, rlc_seed=0x65, gident=1),  # level 1g, then level 3
    dict(verify_mode=0, rlc_group=7, rlc_chunk=3, rlc_batch=1, rlc_seed=0x66, gident=2),  # level 0 fails; 1g -> 1.5
], ids=["each", "g8c2", "g16_gid", "l0_g7c3_gid2"])
def test_fallback_window_passes_match_oracle(cfg):
    """The fallback levels share one line buffer of fb_window list positions,
    consumed in passes (tbls_engine.hip, k_rlc.hip fb_passes).  With a
    64-position window every level's list spans many passes (5 % invalid
    partials: hundreds of chunks, duties and partials per level), and the
    verdicts and aggregates must equal the one-pass default and oracle/c."""
    from charon_amd import engine as eng
    from tools.workload import make_batch
    small = eng.Engine(0, slots=1, fb_window=64, **cfg)
    wide = eng.Engine(0, slots=1, **cfg)
    try:
        b = make_batch(small, 3000, 3, 4, seed=64, inject=0.05)
        wide.load_pubkeys(b.pubshares)  # same ids in both contexts (each loaded once)
        t = small.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                         duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
        r_small = small.collect(t)
        fb = small.fallback(t)
        # at least one fallback list crossed the window
        assert max(fb["chunks"], fb["chunk_searches"], fb["duty_searches"], fb["partial_checks"],
                   fb["group_searches"]) > 64, fb
        r_wide = engine_run(wide, b)
        ref = oracle_run(b)
        assert_same(r_small, ref)
        assert_same(r_wide, ref)
        assert np.array_equal(r_small.partial_status == eng.PS_VALID, ~b.injected)
    finally:
        small.close()
        wide.close()


def test_verify_each_past_the_default_window(engine):
    """TBG_VERIFY_EACH with more partials than the default window (32,768):
    level 3's list runs in two passes, invalid partials sit past position
    32,768, and every verdict equals oracle/c."""
    from charon_amd import engine as eng
    from tools.workload import make_batch
    each = eng.Engine(0, slots=1, verify_mode=eng.VERIFY_EACH)
    try:
        b = make_batch(each, 9000, 3, 4, seed=65, inject=0.01)
        assert len(b.identifiers) > 32768 and b.injected[32768:].sum() >= 3
        res = engine_run(each, b)
        assert_same(res, oracle_run(b))
        assert np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected)
    finally:
        each.close()
