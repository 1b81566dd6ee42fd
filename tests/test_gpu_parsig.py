"""GPU parity of the batch-aware call sites: the
reference's signing KATs through signing.verify_batch, and the parsigex ->
parsigdb -> sigagg flow over tests/golden/parsig_sets.json with one GPU
submit for all peer sets and one GPU launch per aggregation batch.
Bar: identical set verdicts (error class) and bit-exact 96-byte aggregates."""
import json
import os

import pytest

from charon_amd import parsig, signing, tbls
from charon_amd.parsig import Duty, ParSignedData

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def engine():
    from charon_amd import engine as eng
    e = eng.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(HERE, "golden", "parsig_sets.json")) as f:
        return json.load(f)


def _spec(fx):
    return signing.Spec(forks=[(e, bytes.fromhex(v)) for e, v in fx["forks"]],
                        genesis_validators_root=bytes.fromhex(fx["genesis_validators_root"]))


def _sets(fx):
    out = []
    for s in fx["sets"]:
        pset = {it["pubkey"]: ParSignedData(it["domain"], it["epoch"], bytes.fromhex(it["message_root"]),
                                            bytes.fromhex(it["sig"]), it["share_idx"]) for it in s["items"]}
        out.append((Duty(s["slot"], s["duty_type"]), pset))
    return out


def _verifier(fx, engine):
    pubshares = {d["pubkey"]: {int(k): tbls.PublicKey(bytes.fromhex(v)) for k, v in d["pubshares"].items()}
                 for d in fx["dvs"]}
    return parsig.Eth2Verifier(_spec(fx), pubshares, engine)


def test_signing_verify_deposit_and_builder_kats(engine):
    from tests.test_oracle_kat import DEPOSIT_GOLDEN
    spec = signing.Spec()
    items = [signing.VerifyItem(signing.DOMAIN_DEPOSIT, 0, bytes.fromhex(root), bytes.fromhex(sig), bytes.fromhex(pk))
             for pk, sig, root in DEPOSIT_GOLDEN]
    # the same signature claimed for the next key's message root must fail
    items += [signing.VerifyItem(signing.DOMAIN_DEPOSIT, 0, bytes.fromhex(DEPOSIT_GOLDEN[(i + 1) % 4][2]),
                                 bytes.fromhex(sig), bytes.fromhex(pk)) for i, (pk, sig, _) in enumerate(DEPOSIT_GOLDEN)]
    # right message, wrong domain (attester domain instead of deposit)
    pk, sig, root = DEPOSIT_GOLDEN[0]
    items.append(signing.VerifyItem(signing.DOMAIN_BEACON_ATTESTER, 0, bytes.fromhex(root), bytes.fromhex(sig),
                                    bytes.fromhex(pk)))
    res = signing.verify_batch(spec, items, engine)
    assert res[:4] == [None] * 4
    assert all(str(r) == "invalid signature" for r in res[4:])


def test_parsigex_sets_verdicts(fx, engine):
    v = _verifier(fx, engine)
    verdicts = v.verify_sets(_sets(fx))
    for s, r in zip(fx["sets"], verdicts):
        if s["expect_error"] is None:
            assert r is None, (s["duty"], s["peer"], r)
        else:
            assert r is not None and s["expect_error"] in str(r), (s["fault"], r)


def test_parsigex_to_sigagg_aggregates_bit_exact(fx, engine):
    v = _verifier(fx, engine)
    ex = parsig.ParSigEx(v)
    db = parsig.MemDB(fx["threshold"])
    agg = parsig.Aggregator(fx["threshold"], engine)
    results = {}
    agg.subscribe(lambda duty, pk, signed: results.__setitem__((duty.slot, pk), signed))
    db.subscribe_threshold_batch(agg.aggregate_batch)
    ex.subscribe(db.store_external)
    verdicts = ex.handle_batch(_sets(fx))
    # which (duty, DV) pairs must reach threshold: duties with >= t clean peer sets
    clean = {}
    for s, r in zip(fx["sets"], verdicts):
        clean[s["duty"]] = clean.get(s["duty"], 0) + (r is None)
    expect = {}
    for a in fx["aggregates"]:
        d = fx["duties"][a["duty"]]
        if clean[a["duty"]] >= fx["threshold"]:
            expect[(d["slot"], a["pubkey"])] = a["agg"]
    assert expect, "fixture must aggregate something"
    assert set(results) == set(expect)
    for k, a in expect.items():
        assert results[k].signature.hex() == a
        assert results[k].share_idx == 0


def test_aggregate_batch_decode_error_and_bypass(fx, engine):
    """sigagg's convert-signature error for an undecodable partial, beside a
    clean DV in the same GPU launch."""
    sets = _sets(fx)
    # honest partials of DV 0 for duty 0 from peers 1, 3, 4 (peer 2 is faulty)
    dv = fx["dvs"][0]["pubkey"]
    duty = sets[0][0]
    parts = [sets[p][1][dv] for p in (0, 2, 3)]
    bad = list(parts)
    bad[1] = ParSignedData(bad[1].domain, bad[1].epoch, bad[1].message_root, b"\xff" * 96, bad[1].share_idx)
    out = parsig.Aggregator(3, engine).aggregate_batch([(duty, dv, bad), (duty, dv, parts)])
    assert isinstance(out[0], parsig.ParSigError) and str(out[0]).startswith("convert signature: uncompress sig")
    want = [a["agg"] for a in fx["aggregates"] if a["duty"] == 0 and a["pubkey"] == dv][0]
    assert out[1].signature.hex() == want


def test_validatorapi_batch_verify(fx, engine):
    spec = _spec(fx)
    sets = _sets(fx)
    share_of = {d["pubkey"]: tbls.PublicKey(bytes.fromhex(d["pubshares"]["1"])) for d in fx["dvs"]}
    clean = [i for i, s in enumerate(fx["sets"]) if s["peer"] == 1 and s["expect_error"] is None]
    items = [(pk, data) for pk, data in sets[clean[0]][1].items()]
    assert parsig.verify_partial_sigs(spec, share_of.__getitem__, items, engine) is None
    # peer 1's wrong-share set: the first failure aborts the submitter's batch
    bad = [i for i, s in enumerate(fx["sets"]) if s["peer"] == 1 and s["fault"] == "wrong_share"][0]
    items = [(pk, data) for pk, data in sets[bad][1].items()]
    assert str(parsig.verify_partial_sigs(spec, share_of.__getitem__, items, engine)) == "invalid signature"


def test_reference_signed_objects_verify_through_native_roots(engine):
    """MessageRoot + GetDataRoot computed by the native batch (include/tbls_ssz.h)
    from the typed objects, then verified on the GPU: the reference's
    attestation (validatorapi_test.go:230-289), deposit and registration
    signatures all verify; each object with one field changed does not."""
    from charon_amd import ssz
    from oracle import bls12_381 as bls
    from oracle import tbls_oracle as tb
    H = bytes.fromhex
    g = json.load(open(os.path.join(HERE, "golden", "ssz_vectors.json")))
    v = g["sign_and_verify_attestation"]
    spec = signing.Spec(forks=[(0, H(v["fork_version"]))], genesis_validators_root=H(v["genesis_validators_root"]))
    att = ssz.AttestationData(v["slot"], v["index"], H(v["beacon_block_root"]),
                              ssz.Checkpoint(v["source"]["epoch"], H(v["source"]["root"])),
                              ssz.Checkpoint(v["target"]["epoch"], H(v["target"]["root"])))
    bad_att = ssz.AttestationData(v["slot"] + 1, v["index"], att.beacon_block_root, att.source, att.target)
    att_pk = tbls.PublicKey(bls.g1_compress(tb.sk_to_pk(int(v["secret_key"], 16))))
    roots = signing.message_signing_roots(spec, signing.DOMAIN_BEACON_ATTESTER, [0, 0], [att, bad_att])
    assert roots[0].hex() == v["signing_root"]
    items = [(att_pk, roots[0], tbls.Signature(H(v["signature"]))), (att_pk, roots[1], tbls.Signature(H(v["signature"])))]
    deps = g["deposits"]
    dspec = signing.Spec(forks=[(0, H(deps[0]["fork_version"]))])
    msgs = [ssz.DepositMessage(H(d["pubkey"]), H(d["withdrawal_credentials"]), d["amount"]) for d in deps]
    msgs += [ssz.DepositMessage(m.pubkey, m.withdrawal_credentials, m.amount + 1) for m in msgs]
    droots = signing.message_signing_roots(dspec, signing.DOMAIN_DEPOSIT, [0] * len(msgs), msgs)
    for k, m in enumerate(msgs):
        d = deps[k % len(deps)]
        items.append((tbls.PublicKey(H(d["pubkey"])), droots[k], tbls.Signature(H(d["signature"]))))
    r = g["validator_registration"]
    reg = ssz.ValidatorRegistration(H(r["fee_recipient"]), r["gas_limit"], r["timestamp"], H(r["pubkey"]))
    bad_reg = ssz.ValidatorRegistration(reg.fee_recipient, reg.gas_limit + 1, reg.timestamp, reg.pubkey)
    rspec = signing.Spec(forks=[(0, H(r["fork_version"]))])
    rroots = signing.message_signing_roots(rspec, signing.DOMAIN_APPLICATION_BUILDER, [0, 0], [reg, bad_reg])
    for rr in rroots:
        items.append((tbls.PublicKey(H(r["signer_pubkey"])), rr, tbls.Signature(H(r["signature"]))))
    got = tbls.verify_batch(items, engine)
    n = len(deps)
    assert got == [True, False] + [True] * n + [False] * n + [True, False]
