"""GPU parity: the HIP engine (through the C ABI) against the oracle's golden
fixtures and against size-independent properties at full batch sizes.

Bar: bit-exact 96-byte aggregates and identical accept/reject (and error
class) on every partial signature."""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")

PS_NAMES = {1: "valid", 0: "invalid", -1: "err_flags", -2: "err_field", -3: "err_curve", -4: "err_subgroup",
            -5: "err_identity", -6: "err_pubkey"}
DS_NAMES = {0: "ok", -20: "insufficient", -21: "insufficient_valid", -22: "too_few", -23: "duplicate",
            -24: "identity", -25: "decode"}


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)["vectors"]


SCHEDULES = {
    # exact per-partial CoreVerify for every candidate
    "each": dict(verify_mode=1),
    # random linear combinations: one duty per group (levels 1 -> 3)
    "rlc1": dict(verify_mode=0, rlc_group=1, rlc_seed=0x5EED),
    # the default: adaptive group size (16 while clean, 8 / 4 after invalid
    # batches), 4 duties per Miller quad, fresh OS randomness per batch
    "rlc16": dict(verify_mode=0),
    # the previous default: 8 duties per group, 2 per quad; no level 0 (the
    # group levels alone, with their r = 1 group leads)
    "rlc8c2": dict(verify_mode=0, rlc_group=8, rlc_chunk=2, rlc_seed=0x8C2, rlc_batch=2),
    # level 0 on every batch: one batch-wide check (bucket MSM of the
    # signatures), injected batches fall through to the group levels
    "l0g16": dict(verify_mode=0, rlc_group=16, rlc_batch=1, rlc_seed=0x10),
    "l0g7c3": dict(verify_mode=0, rlc_group=7, rlc_chunk=3, rlc_batch=1, rlc_seed=0x703),
    # large groups: most injected failures fall back through all three levels
    "rlc64": dict(verify_mode=0, rlc_group=64, rlc_seed=0xC0FFEE),
    # odd group / chunk sizes: ragged last group, chunks of 3 duties
    "rlc7c3": dict(verify_mode=0, rlc_group=7, rlc_chunk=3, rlc_seed=77),
}


@pytest.fixture(scope="module", params=list(SCHEDULES))
def engine(request):
    from charon_amd import engine as eng
    e = eng.Engine(0, **SCHEDULES[request.param])
    yield e
    e.close()


def test_native_library_is_the_hip_engine(engine):
    from charon_amd import _native
    assert os.path.exists(_native.LIB_PATH)
    assert engine._lib._name == _native.LIB_PATH


def test_kat_verify(engine):
    from charon_amd import tbls
    vecs = load("kat_verify.json")
    items = [(tbls.PublicKey(bytes.fromhex(v["pk"])), bytes.fromhex(v["msg"]), tbls.Signature(bytes.fromhex(v["sig"])))
             for v in vecs]
    got = tbls.verify_batch(items, engine)
    assert got == [v["expect"] == "valid" for v in vecs]
    # single-item Go-API form
    assert tbls.verify(*items[0], engine=engine) is True


def _va_batch(engine, vecs):
    from charon_amd import tbls
    duties = []
    for v in vecs:
        t = v["tss"]
        tss = tbls.TSS({int(k): tbls.PublicKey(bytes.fromhex(pk)) for k, pk in t["pubshares"].items()},
                       t["num_shares"], t["threshold"], tbls.PublicKey(bytes.fromhex(t["public_key"])))
        parts = [tbls.PartialSignature(p["identifier"], tbls.Signature(bytes.fromhex(p["sig"]))) for p in v["partials"]]
        duties.append({"tss": tss, "partials": parts, "msg": bytes.fromhex(v["msg"])})
    return duties


@pytest.mark.parametrize("name", ["cfg1_3of4_single.json", "cfg2_3of4_sample.json", "cfg3_7of10_sample.json",
                                  "cfg5_mixed_invalid.json", "va_id_modes.json"])
def test_verify_and_aggregate_golden(engine, name):
    from charon_amd import engine as eng, tbls
    vecs = load(name)
    duties = _va_batch(engine, vecs)
    # raw engine call: per-partial status + per-duty status + bytes
    from charon_amd.tbls import _duty_arrays, _pk_cache
    duty_first, sigs, ids, msgs, thr, pk_keys = _duty_arrays(duties, True)
    present = [k for k in pk_keys if k is not None]
    it = iter(_pk_cache.ids_for(engine, present))
    pk_ids = [next(it) if k is not None else eng.NO_PUBKEY for k in pk_keys]
    res = engine.run(eng.OP_VERIFY_AGGREGATE, duty_first, sigs, ids, msgs=msgs, duty_msg=np.arange(len(duties)),
                     pubkey_ids=pk_ids, duty_threshold=thr)
    for d, v in enumerate(vecs):
        lo, hi = duty_first[d], duty_first[d + 1]
        got_ps = [PS_NAMES[s] for s in res.partial_status[lo:hi].tolist()]
        exp = v["expect"]
        # a duty rejected for too few partials is decided before verification
        if exp["status"] != "insufficient":
            assert got_ps == exp["partial_status"], v["label"]
        assert DS_NAMES[int(res.duty_status[d])] == exp["status"], v["label"]
        if exp["status"] == "ok":
            assert bytes(res.agg[d]).hex() == exp["agg"], v["label"]
            assert bytes(res.agg[d]).hex() == exp["group_sig"]
    # Go-API mirror form
    out = tbls.verify_and_aggregate_batch(duties, engine)
    for r, v in zip(out, vecs):
        if v["expect"]["status"] == "ok":
            sig, signers = r
            assert sig.raw.hex() == v["expect"]["agg"] and signers == v["expect"]["signers"]
        else:
            assert isinstance(r, tbls.TblsError)


def test_aggregate_golden(engine):
    from charon_amd import engine as eng, tbls
    vecs = load("aggregate_edges.json")
    duties = [[tbls.PartialSignature(p["identifier"], tbls.Signature(bytes.fromhex(p["sig"]))) for p in v["partials"]]
              for v in vecs]
    duty_first = np.cumsum([0] + [len(d) for d in duties])
    sigs = b"".join(p.signature.raw for d in duties for p in d)
    ids = [p.identifier for d in duties for p in d]
    res = engine.run(eng.OP_AGGREGATE, duty_first, sigs, ids)
    for d, v in enumerate(vecs):
        assert DS_NAMES[int(res.duty_status[d])] == v["expect"]["status"], v["label"]
        if v["expect"]["status"] == "ok":
            assert bytes(res.agg[d]).hex() == v["expect"]["agg"], v["label"]
    # Go-API mirror
    for d, v in zip(duties, vecs):
        if v["expect"]["status"] == "ok":
            assert tbls.aggregate(d, engine).raw.hex() == v["expect"]["agg"]
        else:
            with pytest.raises(tbls.TblsError):
                tbls.aggregate(d, engine)


def test_engine_sign_matches_oracle(engine):
    """GPU test-vector generation (tbls.Sign) agrees with the oracle."""
    from oracle import bls12_381 as bls
    from oracle import tbls_oracle as tb
    rng = random.Random(7)
    sks = [rng.randrange(1, bls.R) for _ in range(3)]
    msgs = [b"Hello Obol", bytes(32), bytes(range(32))]
    sk32 = b"".join(s.to_bytes(32, "big") for s in sks)
    sigs = engine.sign(sk32, msgs, [0, 1, 2])
    pks = engine.sk_to_pk(sk32)
    for i, s in enumerate(sks):
        assert bytes(sigs[i]) == bls.g2_compress(tb.sign(s, msgs[i]))
        assert bytes(pks[i]) == bls.g1_compress(tb.sk_to_pk(s))


def _make_cluster_batch(engine, n_dv, t, n, seed, inject=0.0):
    """Full-size synthetic batch built on the GPU (keys, shares, signatures)."""
    from tools.workload import make_batch
    return make_batch(engine, n_dv, t, n, seed, inject=inject)


@pytest.mark.parametrize("n_dv,t,n,inject", [(2000, 3, 4, 0.02), (300, 7, 10, 0.02), (512, 3, 4, 0.5)])
def test_full_size_properties(engine, n_dv, t, n, inject):
    """At batch scale: every honest partial verifies, every aggregate equals
    the group signature sk * H(m) computed independently on the GPU, and an
    injected invalid partial is rejected without changing the aggregate."""
    from charon_amd import engine as eng
    b = _make_cluster_batch(engine, n_dv, t, n, seed=11, inject=inject)
    res = engine.run(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                     duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
    expect_valid = ~b.injected
    assert np.array_equal(res.partial_status == eng.PS_VALID, expect_valid)
    ok = res.duty_status == eng.DS_OK
    assert np.array_equal(ok, b.expect_ok)
    assert np.array_equal(res.agg[ok], b.group_sig[ok])


def test_clean_batch_needs_no_fallback(engine):
    """Honest partials pass at level 1: the RLC combination itself is right
    (a wrong scalar identity would still give right verdicts, via fallback)."""
    from charon_amd import engine as eng
    b = _make_cluster_batch(engine, 1000, 3, 4, seed=5)
    t = engine.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                      duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
    res = engine.collect(t)
    assert (res.partial_status == eng.PS_VALID).all()
    assert engine.level0(t) in (eng.L0_NOT_RUN, eng.L0_PASSED)  # a clean batch never fails level 0
    st = engine.stats(t)
    if st["group_size"]:
        assert st["duty_checks"] == 0 and st["partial_checks"] == 0, st
    else:
        assert st["partial_checks"] == 4000


def test_shared_messages_and_replay(engine):
    """Committee-style batch: 64 duties share each message (the same H(m) is
    paired with many combined keys inside one RLC group); replays of the
    resident batch give the same verdicts and bytes."""
    from charon_amd import engine as eng
    b = _make_cluster_batch(engine, 256, 3, 4, seed=23, inject=0.01)
    duty_msg = (np.arange(256) // 64).astype(np.uint32)
    # re-sign so every duty signs its committee's message
    msgs = [b.msgs[k * 64] for k in range(4)]
    sk32 = b"".join(s.to_bytes(32, "big") for s in b.shares)
    item_msg = np.repeat(duty_msg, 4)
    sigs = engine.sign(sk32, msgs, item_msg)
    wrong = engine.sign(sk32, [m[:-1] + bytes([m[-1] ^ 1]) for m in msgs], item_msg)
    sigs = np.where(b.injected[:, None], wrong, sigs)
    group = engine.sign(b"".join(s.to_bytes(32, "big") for s in b.secrets), msgs, duty_msg)
    from charon_amd.engine import pack_messages
    t = engine.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, sigs, b.identifiers, msgs=pack_messages(msgs),
                      duty_msg=duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
    res = engine.collect(t)
    assert np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected)
    ok = res.duty_status == eng.DS_OK
    assert np.array_equal(ok, b.expect_ok)
    assert np.array_equal(res.agg[ok], group[ok])
    engine.replay(t, 2)
    again = engine.fetch(t, 256, 1024)
    assert np.array_equal(again.partial_status, res.partial_status)
    assert np.array_equal(again.duty_status, res.duty_status)
    assert np.array_equal(again.agg, res.agg)


def test_rlc_cancelling_errors_across_duties_are_rejected(engine):
    """Two invalid partials of different duties whose errors cancel
    (s_a = sig_a + D, s_b = sig_b - D) must not pass a level-1 group check:
    only one candidate per GROUP may carry the fixed coefficient r = 1
    (k_rlc.hip).  Every schedule must return the per-item verdicts."""
    from charon_amd import tbls
    from oracle import bls12_381 as bls
    vecs = [dict(v) for v in load("cfg2_3of4_sample.json")[:4]]
    assert all(v["expect"]["status"] == "ok" for v in vecs)
    delta = bls.g2_mul(bls.G2_GEN, 0x1234567)
    bad = {2: None, 3: None}
    for d, sign in ((0, 1), (1, -1)):
        v = vecs[d]
        parts = [dict(p) for p in v["partials"]]
        k = 0  # the first candidate of each duty
        s = bls.g2_decompress(bytes.fromhex(parts[k]["sig"]))
        s = bls.g2_add(s, delta if sign > 0 else bls.g2_neg(delta))
        parts[k]["sig"] = bls.g2_compress(s).hex()
        v["partials"] = parts
        bad[d] = parts[k]["identifier"]
    duties = _va_batch(engine, vecs)
    out = tbls.verify_and_aggregate_batch(duties, engine)
    for d, (r, v) in enumerate(zip(out, vecs)):
        sig, signers = r
        assert bad[d] not in signers, d
        assert len(signers) >= v["tss"]["threshold"]
        assert sig.raw.hex() == v["expect"]["group_sig"]


def test_adaptive_group_size_follows_invalid_share():
    """tbg_config.rlc_group = 0: 16 duties per group while the collected
    batches are clean, smaller groups once they carry invalid partials, and
    back to 16 after clean ones; verdicts are exact throughout."""
    from charon_amd import engine as eng
    e = eng.Engine(0)
    try:
        def run(seed, inject):
            b = _make_cluster_batch(e, 400, 3, 4, seed=seed, inject=inject)
            t = e.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                         duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
            res = e.collect(t)
            assert np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected)
            return e.stats(t)["group_size"]
        assert run(31, 0.0) == 16
        run(32, 0.05)
        assert run(33, 0.05) in (4, 8)
        sizes = [run(34 + k, 0.0) for k in range(8)]
        assert sizes[-1] == 16
    finally:
        e.close()


def test_level0_pass_and_fall_through():
    """Level 0 (tbg_config.rlc_batch): a clean batch -- also several callers'
    batches packed into one launch -- passes the one batch-wide check; one
    invalid partial anywhere fails it and the group levels return the exact
    per-item verdicts; the adaptive policy stops running level 0 after an
    invalid batch."""
    from charon_amd import engine as eng
    for cfg in (dict(rlc_batch=eng.RLC_L0_ON, rlc_group=16), dict()):
        e = eng.Engine(0, **cfg)
        try:
            def submit(bs):
                ts = e.submit_group(eng.OP_VERIFY_AGGREGATE, [
                    dict(duty_first=b.duty_first, sigs=b.sigs, identifiers=b.identifiers, msgs=(b.msg_data, b.msg_off),
                         duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold) for b in bs])
                for b, t in zip(bs, ts):
                    res = e.collect(t)
                    assert np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected)
                    ok = res.duty_status == eng.DS_OK
                    assert np.array_equal(ok, b.expect_ok)
                    assert np.array_equal(res.agg[ok], b.group_sig[ok])
                return e.level0(ts[0])
            clean = [_make_cluster_batch(e, n, 3, 4, seed=40 + n) for n in (700, 333)]
            assert submit(clean) == eng.L0_PASSED
            one_bad = _make_cluster_batch(e, 500, 3, 4, seed=47, inject=0.002)
            assert one_bad.injected.any()
            assert submit([clean[0], one_bad]) == eng.L0_FAILED
            after = submit(clean[1:])
            assert after == (eng.L0_PASSED if cfg else eng.L0_NOT_RUN)
        finally:
            e.close()


def test_level1g_resolves_single_bad_partials():
    """Level 1g: a failed group holding ONE bad partial is resolved by the
    exponent test over the group's partials (no chunk, duty or per-partial
    level), with verdicts and aggregates exact; groups with several bad
    partials still reach the deeper levels and come out exact too."""
    from charon_amd import engine as eng
    # level 1g is opt-in (tbg_config.gident, fixed at init)
    e = eng.Engine(0, verify_mode=0, rlc_group=8, rlc_chunk=4, rlc_batch=2, rlc_seed=0x1A, gident=eng.GIDENT_L3)
    try:
        b = _make_cluster_batch(e, 2000, 3, 4, seed=23, inject=0.01)
        t = e.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                     duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
        res = e.collect(t)
        assert np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected)
        ok = res.duty_status == eng.DS_OK
        assert np.array_equal(ok, b.expect_ok)
        assert np.array_equal(res.agg[ok], b.group_sig[ok])
        fb = e.fallback(t)
        bad_groups = {int(i) // (4 * 8) for i in np.flatnonzero(b.injected)}
        multi = sum(1 for g in bad_groups if int(b.injected[32 * g:32 * g + 32].sum()) > 1)
        assert fb["group_size"] == 8 and fb["group_searches"] == len(bad_groups), (fb, len(bad_groups))
        # only groups with two or more bad partials go deeper (their chunks)
        assert fb["chunks"] <= 2 * multi, (fb, multi)
        dev, pinned = e.slot_bytes(t)
        assert dev > 0 and pinned > 0
    finally:
        e.close()


def test_level1g_off_by_default_narrows_by_chunks(engine):
    """With the default tbg_config.gident (off) the failed groups take the
    chunk / duty narrowing (level 1g is opt-in) and the verdicts are exact."""
    from charon_amd import engine as eng
    b = _make_cluster_batch(engine, 600, 3, 4, seed=29, inject=0.02)
    t = engine.submit(eng.OP_VERIFY_AGGREGATE, b.duty_first, b.sigs, b.identifiers, msgs=(b.msg_data, b.msg_off),
                      duty_msg=b.duty_msg, pubkey_ids=b.pubkey_ids, duty_threshold=b.threshold)
    res = engine.collect(t)
    assert np.array_equal(res.partial_status == eng.PS_VALID, ~b.injected)
    assert engine.fallback(t)["group_searches"] == 0
