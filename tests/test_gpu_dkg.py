"""GPU parity of the DKG / cluster-lock signature work (charon_amd.dkg,
SURVEY.md §8f rank 4) against the oracle fixtures of
tests/golden/make_dkg_golden.py:

  * aggDepositDataSigs (dkg/dkg.go:545-601): the threshold aggregates of the
    reference's four deposit keys are the golden file's signatures, bit for bit;
  * aggLockHashSig (dkg/dkg.go:428-478): AggregateSignatures /
    AggregatePublicKeys equal the oracle's point sums and verify;
  * Lock.VerifySignatures (cluster/lock.go:137-179): FastAggregateVerify over
    every pubshare; the error paths mirror the reference's strings
    (dkg/dkg_internal_test.go:62-80 for the partial-signature ones)."""
import json
import os
import random

import numpy as np
import pytest

from charon_amd import dkg
from charon_amd import engine as eng
from oracle import bls12_381 as bls

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "dkg_vectors.json")))
H = bytes.fromhex


@pytest.fixture(scope="module")
def engine():
    e = eng.Engine(0)
    yield e
    e.close()


def _deposit_inputs():
    data, shares, msgs = {}, {}, {}
    for dv in G["deposit"]:
        pk = H(dv["pubkey"])
        data[pk] = [dkg.DKGPartial(int(i), H(s)) for i, s in dv["partials"].items()]
        shares[pk] = {int(i): H(s) for i, s in dv["pubshares"].items()}
        msgs[pk] = H(dv["signing_root"])
    return data, shares, msgs


def test_deposit_aggregates_are_the_golden_signatures(engine):
    data, shares, msgs = _deposit_inputs()
    aggs = dkg.agg_deposit_data_sigs(data, shares, msgs, engine)
    assert {k.hex(): v.hex() for k, v in aggs.items()} == {dv["pubkey"]: dv["aggregate"] for dv in G["deposit"]}
    dkg.verify_deposit_aggregates(aggs, msgs, engine)
    # three of four partials give the same aggregate (any threshold subset)
    data3 = {k: v[1:] for k, v in data.items()}
    assert dkg.agg_deposit_data_sigs(data3, shares, msgs, engine) == aggs


def test_deposit_error_paths(engine):
    data, shares, msgs = _deposit_inputs()
    k0, k1 = list(data)[:2]
    bad = dict(data)
    bad[k0] = [data[k0][0], dkg.DKGPartial(data[k0][1].share_idx, data[k1][1].signature)] + data[k0][2:]
    with pytest.raises(dkg.DKGError, match="^invalid deposit data partial signature from peer$"):
        dkg.agg_deposit_data_sigs(bad, shares, msgs, engine)
    bad = dict(data)
    bad[k0] = data[k0] + [dkg.DKGPartial(9, data[k0][0].signature)]
    with pytest.raises(dkg.DKGError, match="^invalid pubshare$"):
        dkg.agg_deposit_data_sigs(bad, shares, msgs, engine)
    with pytest.raises(dkg.DKGError, match="^invalid pubkey in deposit data partial signature from peer$"):
        dkg.agg_deposit_data_sigs({b"\x01" * 48: data[k0]}, shares, msgs, engine)
    raw = bytearray(data[k0][0].signature)
    raw[0] &= 0x7F  # compression flag cleared
    bad = dict(data)
    bad[k0] = [dkg.DKGPartial(data[k0][0].share_idx, bytes(raw))] + data[k0][1:]
    with pytest.raises(dkg.DKGError, match="^signature from core: uncompress sig: "):
        dkg.agg_deposit_data_sigs(bad, shares, msgs, engine)
    # the aggregate of one DV claimed for another
    aggs = dkg.agg_deposit_data_sigs(data, shares, msgs, engine)
    aggs[k0], aggs[k1] = aggs[k1], aggs[k0]
    with pytest.raises(dkg.DKGError, match="^invalid deposit data aggregated signature$"):
        dkg.verify_deposit_aggregates(aggs, msgs, engine)


def _lock_inputs():
    L = G["lock"]
    dvs = {d["pubkey"]: d for d in G["deposit"]}
    data, shares = {}, {}
    for p in L["partials"]:
        pk = H(p["pubkey"])
        data.setdefault(pk, []).append(dkg.DKGPartial(p["share_idx"], H(p["sig"])))
        shares[pk] = {int(i): H(s) for i, s in dvs[p["pubkey"]]["pubshares"].items()}
    return data, shares, H(L["hash"])


def test_lock_hash_multisignature(engine):
    data, shares, h = _lock_inputs()
    sig, pk = dkg.agg_lock_hash_sig(data, shares, h, engine)
    assert sig.hex() == G["lock"]["aggregate_signature"] and pk.hex() == G["lock"]["aggregate_pubkey"]
    assert dkg.verify_multi_signature(pk, h, sig, engine)
    assert not dkg.verify_multi_signature(pk, h[:-1] + bytes([h[-1] ^ 1]), sig, engine)
    k0 = list(data)[0]
    bad = dict(data)
    bad[k0] = [dkg.DKGPartial(data[k0][0].share_idx, data[k0][1].signature)] + data[k0][1:]
    with pytest.raises(dkg.DKGError, match="^invalid lock hash partial signature from peer$"):
        dkg.agg_lock_hash_sig(bad, shares, h, engine)


def test_lock_verify_signatures(engine):
    data, shares, h = _lock_inputs()
    lock = {"cluster_definition": {"version": "v1.4.0"}, "lock_hash": "0x" + h.hex(),
            "signature_aggregate": "0x" + G["lock"]["aggregate_signature"],
            "distributed_validators": [{"public_shares": ["0x" + shares[pk][p.share_idx].hex() for p in data[pk]]}
                                       for pk in data]}
    dkg.lock_verify_signatures(lock, h, engine)
    # the aggregate is checked over the caller's recomputed hash, never the JSON's
    with pytest.raises(ValueError, match="recomputed hashLock"):
        dkg.lock_verify_signatures(lock, None, engine)
    # VerifySignatures never reads the JSON's lock_hash (lock.go:137-179): an
    # edited JSON hash still verifies; VerifyHashes (lock_verify_hashes) rejects it
    edited = dict(lock, lock_hash="0x" + bytes(32).hex())
    dkg.lock_verify_signatures(edited, h, engine)
    with pytest.raises(dkg.DKGError, match="^invalid lock hash$"):
        dkg.lock_verify_hashes(edited, h)
    dkg.lock_verify_hashes(lock, h)
    wrong = bytes(32)  # a lock whose fields hash differently: same JSON and aggregate
    with pytest.raises(dkg.DKGError, match="^invalid lock signature aggregate$"):
        dkg.lock_verify_signatures(lock, wrong, engine)
    missing = dict(lock, distributed_validators=lock["distributed_validators"][:-1])
    with pytest.raises(dkg.DKGError, match="^invalid lock signature aggregate$"):
        dkg.lock_verify_signatures(missing, h, engine)
    badkey = json.loads(json.dumps(lock))
    badkey["distributed_validators"][0]["public_shares"][0] = "0x" + (b"\x00" * 48).hex()
    with pytest.raises(dkg.DKGError, match="^unmarshal pubkey: "):
        dkg.lock_verify_signatures(badkey, h, engine)
    badsig = dict(lock, signature_aggregate="0x" + (b"\x00" * 96).hex())
    with pytest.raises(dkg.DKGError, match="^uncompress sig: "):
        dkg.lock_verify_signatures(badsig, h, engine)


def test_key_upload_is_deduplicated(engine):
    """KeyFromBytes over keys already resident uploads nothing more (the
    device table does not grow with repeated lock / wiring checks), and a bad
    key keeps reporting its decode error from the cached status."""
    from charon_amd import tbls
    _, shares, _ = _deposit_inputs()
    raws = [k for per in shares.values() for k in per.values()]
    tbls.key_from_bytes_batch(raws, engine)
    n0 = engine.pubkey_count
    bad = b"\x00" * 47 + b"\x2a"  # no compression flag: a decode error (not uploaded by any other test)
    r1 = tbls.key_from_bytes_batch(raws + [bad] + raws, engine)
    assert engine.pubkey_count == n0 + 1
    r2 = tbls.key_from_bytes_batch([bad] + raws, engine)
    assert engine.pubkey_count == n0 + 1
    assert isinstance(r1[len(raws)], tbls.TblsError) and str(r1[len(raws)]) == str(r2[0])
    assert all(isinstance(k, tbls.PublicKey) for k in r2[1:])


def test_sum_edge_cases(engine):
    """tbg_sum_sigs / tbg_sum_pubkeys: the identity encoding adds nothing, a bad
    encoding fails its set only, an empty set is the identity."""
    L = G["lock"]
    s = [H(p["sig"]) for p in L["partials"][:3]]
    ident = b"\xc0" + bytes(95)
    bad = b"\x00" + s[0][1:]
    sigs = s + [ident] + s[:1] + [bad]
    out, st, sst = engine.sum_sigs(b"".join(sigs), [0, 3, 4, 5, 6, 6])
    want = None
    for x in s:
        want = bls.g2_add(want, bls.g2_decompress(x))
    assert out[0].tobytes() == bls.g2_compress(want)
    assert st.tolist() == [eng.DS_OK, eng.DS_AGG_IDENTITY, eng.DS_OK, eng.DS_DECODE, eng.DS_AGG_IDENTITY]
    assert out[2].tobytes() == s[0]
    assert sst.tolist() == [eng.PS_NOT_VERIFIED] * 3 + [eng.PS_ERR_IDENTITY, eng.PS_NOT_VERIFIED, eng.PS_ERR_FLAGS]
    first, kst = engine.load_pubkeys(b"".join(H(v) for v in G["deposit"][0]["pubshares"].values()))
    assert kst.tolist() == [0] * 4
    ids = [first + i for i in range(4)]
    pk, pst = engine.sum_pubkeys(ids + [ids[0], 10 ** 9], [0, 4, 4, 6])
    want = None
    for v in G["deposit"][0]["pubshares"].values():
        want = bls.g1_add(want, bls.g1_decompress(H(v)))
    assert pk[0].tobytes() == bls.g1_compress(want)
    assert pst.tolist() == [eng.DS_OK, eng.DS_AGG_IDENTITY, eng.DS_DECODE]


def test_fast_aggregate_verify_many_sets(engine):
    """Sets from 1 to 3000 keys, each signed by the sum of its secrets over its
    own message; one set per size class gets a foreign key (invalid)."""
    rng = random.Random(11)
    R = bls.R
    sizes = [1, 2, 5, 33, 64, 65, 500, 3000]
    sks = [rng.randrange(1, R) for _ in range(sum(sizes) + 1)]
    pks = engine.sk_to_pk(b"".join(k.to_bytes(32, "big") for k in sks))
    first, st = engine.load_pubkeys(pks.tobytes())
    assert (st == 0).all()
    off, ids, msgs, sums = [0], [], [], []
    pos = 0
    for n in sizes:
        ids += [first + pos + j for j in range(n)]
        sums.append(sum(sks[pos:pos + n]) % R)
        pos += n
        off.append(len(ids))
        msgs.append(b"lock-%d" % n)
    sig = engine.sign(b"".join(s.to_bytes(32, "big") for s in sums), msgs, np.arange(len(sizes)))
    got = engine.fast_aggregate_verify(ids, off, msgs, sig.tobytes())
    assert got.tolist() == [eng.PS_VALID] * len(sizes)
    ids_bad = list(ids)
    for k in range(len(sizes)):
        ids_bad[off[k]] = first + len(sks) - 1  # the spare key
    got = engine.fast_aggregate_verify(ids_bad, off, msgs, sig.tobytes())
    assert got.tolist() == [eng.PS_INVALID] * len(sizes)
    # the 3000-key sum against the oracle's
    big, _ = engine.sum_pubkeys(ids[off[-2]:off[-1]], [0, sizes[-1]])
    want = None
    for row in pks[pos - sizes[-1]:pos]:
        want = bls.g1_add(want, bls.g1_decompress(row.tobytes()))
    assert big[0].tobytes() == bls.g1_compress(want)
