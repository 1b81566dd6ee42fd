"""charon_amd.dkg host logic that needs no GPU (cluster/lock.go:142-149
version rules) and the DKG fixtures against the oracle (the deposit
aggregates are the reference golden file's signatures)."""
import json
import os

import pytest

from oracle import bls12_381 as bls
from oracle import tbls_oracle as tb

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "dkg_vectors.json")))
LOCKS = json.load(open(os.path.join(HERE, "golden", "cluster_locks.json")))


def test_empty_aggregate_rules_need_no_gpu():
    from charon_amd import dkg
    for v in ("v1.0.0", "v1.1.0"):
        assert dkg.lock_verify_signatures({"cluster_definition": {"version": v}, "signature_aggregate": ""}) is None
    for v in ("v1.2.0", "v1.3.0", "v1.4.0"):
        with pytest.raises(dkg.DKGError, match="empty lock aggregate signature"):
            dkg.lock_verify_signatures({"cluster_definition": {"version": v}, "signature_aggregate": None})


def test_lock_verify_needs_a_recomputed_hash():
    """The reference checks the aggregate over hashLock(l) (cluster/lock.go:166),
    not the JSON's lock_hash: without the caller's hash nothing is trusted."""
    from charon_amd import dkg
    lock = {"cluster_definition": {"version": "v1.4.0"}, "lock_hash": "0x" + bytes(32).hex(),
            "signature_aggregate": "0x" + (b"\x80" + bytes(95)).hex()}
    with pytest.raises(ValueError, match="recomputed hashLock"):
        dkg.lock_verify_signatures(lock)
    # the JSON hash is VerifyHashes' concern (lock.go:117-131), not VerifySignatures'
    with pytest.raises(dkg.DKGError, match="^invalid lock hash$"):
        dkg.lock_verify_hashes(lock, b"\x01" * 32)
    assert dkg.lock_verify_hashes(lock, bytes(32)) is None
    with pytest.raises(dkg.DKGError, match="^invalid lock hash$"):
        dkg.lock_verify_hashes({k: v for k, v in lock.items() if k != "lock_hash"}, bytes(32))


def test_lock_byte_fields_decode_both_encodings():
    from charon_amd import dkg
    versions = [l["cluster_definition"]["version"] for l in LOCKS]
    assert versions == ["v1.0.0", "v1.1.0", "v1.2.0", "v1.3.0", "v1.4.0"]
    for l in LOCKS:  # base64 (v1.0 / v1.1) and 0x-hex (v1.2+)
        for dv in l["distributed_validators"]:
            assert all(len(dkg._lock_bytes(s)) == 48 for s in dv["public_shares"])
        # the reference test locks carry 32 random bytes as their aggregate:
        # rejected before any key or pairing work
        assert len(dkg._lock_bytes(l["signature_aggregate"])) == 32
        with pytest.raises(dkg.DKGError, match="uncompress sig: invalid length"):
            dkg.lock_verify_signatures(l, bytes(32))


def test_fixture_deposit_aggregates_are_the_golden_signatures():
    from tests.test_oracle_kat import DEPOSIT_GOLDEN
    gold = {pk: sig for pk, sig, _ in DEPOSIT_GOLDEN}
    for dv in G["deposit"]:
        parts = [(int(i), bls.g2_decompress(bytes.fromhex(s))) for i, s in dv["partials"].items()]
        assert bls.g2_compress(tb.combine_signatures(parts)).hex() == dv["aggregate"] == gold[dv["pubkey"]]


def test_fixture_lock_sums():
    L = G["lock"]
    sig = None
    for p in L["partials"]:
        sig = bls.g2_add(sig, bls.g2_decompress(bytes.fromhex(p["sig"])))
    assert bls.g2_compress(sig).hex() == L["aggregate_signature"]
    pk = None
    dvs = {d["pubkey"]: d for d in G["deposit"]}
    for p in L["partials"]:
        pk = bls.g1_add(pk, bls.g1_decompress(bytes.fromhex(dvs[p["pubkey"]]["pubshares"][str(p["share_idx"])])))
    assert bls.g1_compress(pk).hex() == L["aggregate_pubkey"]
