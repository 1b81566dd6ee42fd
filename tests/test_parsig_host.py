"""CPU tests of the batch-aware call-site mirror (charon_amd.signing,
charon_amd.parsig): signing roots and domains against the reference's KATs,
the host-side error paths of parsigex / validatorapi / sigagg (no GPU call is
made for them), parsigdb's dedup and threshold matching, and the parsig
fixture's expectations re-derived with the CPU oracle."""
import json
import os

import pytest

from charon_amd import parsig, signing
from charon_amd.parsig import Duty, ParSignedData

HERE = os.path.dirname(os.path.abspath(__file__))

# deposit signing roots recomputed from
# eth2util/deposit/testdata/TestMarshalDepositData.golden (fork 00001020).
DEPOSIT_SIGNING_ROOTS = {
    "4f5f7044a71d625c59974e32e8d86aed0a2211d423675303124ce5ac70969a46":
        "f8b77cb0fd0443b749ae4a3aec566eced77fb691b3688caf1e80bcf325e14465",
    "33109737473d6ccb5f3c4f7eccaa4a7cd3dd63de3d9878a978243053904d39bf":
        "60225fd501dd87ec978cce9b51b06581d0ce1cc805d38dd02f2224e41827918e",
    "8cec1018fcfcb6ae295546901f1c55e2f2643834b89c9a00e4806d8c6b197169":
        "0a2e9d430fbcd018600b6ef3829b62990bb400e36844a91a28f2df046b27286a",
    "6b6860824055330be4cb0a378a1ffd342e4de77fef1d51621d44419c4b313ca9":
        "639b8c93ca8e3371df3015d8e66bc48bc6d83aef20df26ba01280af9ad10269d",
}


class NoEngine:
    """Stands in for the GPU engine where the host must decide alone."""
    uid = -1

    def __getattr__(self, name):
        raise AssertionError(f"GPU engine used ({name}) on a host-only path")


def load_fixture():
    with open(os.path.join(HERE, "golden", "parsig_sets.json")) as f:
        return json.load(f)


def fixture_spec(fx):
    return signing.Spec(forks=[(e, bytes.fromhex(v)) for e, v in fx["forks"]],
                        genesis_validators_root=bytes.fromhex(fx["genesis_validators_root"]))


def test_deposit_signing_roots_match_reference_golden():
    spec = signing.Spec()  # genesis fork 00001020
    for msg_root, expect in DEPOSIT_SIGNING_ROOTS.items():
        got = signing.get_data_root(spec, signing.DOMAIN_DEPOSIT, 12345, bytes.fromhex(msg_root))
        assert got.hex() == expect


def test_builder_domain_is_genesis_based():
    from tests.test_oracle_kat import teku_signing_root
    spec = signing.Spec(forks=[(0, bytes.fromhex("00001020")), (5, bytes.fromhex("02001020"))],
                        genesis_validators_root=bytes(range(32)))
    root = bytes.fromhex("2c231b16a80337212ab1decde301bdb4383e74c0bf2f3439cc82542bf0f90fdd")
    assert signing.get_data_root(spec, signing.DOMAIN_APPLICATION_BUILDER, 99, root) == teku_signing_root()


def test_fixture_signing_roots():
    fx = load_fixture()
    spec = fixture_spec(fx)
    for r in fx["signing_roots"]:
        got = signing.get_data_root(spec, r["domain"], r["epoch"], bytes.fromhex(r["object_root"]))
        assert got.hex() == r["signing_root"]


def test_unknown_domain():
    spec = signing.Spec(domain_types={})
    with pytest.raises(signing.SigningError, match="domain type not found"):
        signing.get_domain(spec, signing.DOMAIN_RANDAO, 0)


def test_zero_signature_rejected_on_host():
    r = signing.verify_batch(signing.Spec(), [signing.VerifyItem(signing.DOMAIN_RANDAO, 0, bytes(32), bytes(96),
                                                                 bytes(48))], engine=NoEngine())
    assert str(r[0]) == "no signature found"


def _pd(root=b"\x01" * 32, sig=b"\x02" * 96, idx=1, domain=signing.DOMAIN_BEACON_ATTESTER, payload=b""):
    return ParSignedData(domain, 3, root, sig, idx, payload)


def test_verifier_host_errors_drop_the_set():
    pubshares = {"dv1": {1: bytes(48), 2: bytes(48)}}
    v = parsig.Eth2Verifier(signing.Spec(), pubshares, engine=NoEngine())
    duty = Duty(10, parsig.DUTY_ATTESTER)
    assert "unknown pubkey" in str(v.verify_sets([(duty, {"dvX": _pd()})])[0])
    assert "invalid shareIdx" in str(v.verify_sets([(duty, {"dv1": _pd(idx=7)})])[0])
    zero = v.verify_sets([(duty, {"dv1": _pd(sig=bytes(96))})])[0]
    assert "invalid signature" in str(zero) and "no signature found" in str(zero)
    with pytest.raises(parsig.ParSigError, match="invalid shareIdx"):
        v.verify_set(duty, {"dv1": _pd(idx=9)})
    ex = parsig.ParSigEx(v)
    got = []
    ex.subscribe(lambda d, s: got.append(s))
    assert ex.handle(duty, {"dv1": _pd(idx=9)}) is not None and got == []


def test_validatorapi_first_failure_in_order():
    def share(pk):
        if pk == "bad":
            raise parsig.ParSigError("pubshare not found")
        return bytes(48)
    items = [("dv1", _pd(sig=bytes(96))), ("bad", _pd())]
    err = parsig.verify_partial_sigs(signing.Spec(), share, items, engine=NoEngine())
    assert str(err) == "no signature found"
    err = parsig.verify_partial_sigs(signing.Spec(), share, items[::-1], engine=NoEngine())
    assert str(err) == "pubshare not found"
    assert parsig.verify_partial_sigs(signing.Spec(), share, items, insecure_test=True) is None


def test_memdb_dedup_mismatch_and_exact_threshold():
    db = parsig.MemDB(threshold=3)
    fired, batches = [], []
    db.subscribe_threshold(lambda d, pk, ps: fired.append((pk, [p.share_idx for p in ps])))
    db.subscribe_threshold_batch(lambda items: batches.append(len(items)))
    duty = Duty(1, parsig.DUTY_ATTESTER)
    for i in (1, 2):
        assert db.store_external(duty, {"a": _pd(idx=i), "b": _pd(idx=i)}) == []
    assert db.store_external(duty, {"a": _pd(idx=2)}) == []  # exact duplicate ignored
    with pytest.raises(parsig.ParSigError, match="mismatching partial signed data"):
        db.store_external(duty, {"a": _pd(idx=2, payload=b"x")})
    reached = db.store_external(duty, {"a": _pd(idx=3), "b": _pd(idx=3)})
    assert [pk for _, pk, _ in reached] == ["a", "b"] and batches == [2]
    assert fired == [("a", [1, 2, 3]), ("b", [1, 2, 3])]
    assert db.store_external(duty, {"a": _pd(idx=4)}) == []  # fires at exactly t only
    db.trim(duty)
    assert db.entries == {}


def test_memdb_groups_by_message_root():
    db = parsig.MemDB(threshold=2)
    duty = Duty(1, parsig.DUTY_PROPOSER)
    assert db.store_external(duty, {"a": _pd(root=b"\x01" * 32, idx=1)}) == []
    assert db.store_external(duty, {"a": _pd(root=b"\x02" * 32, idx=2)}) == []
    reached = db.store_external(duty, {"a": _pd(root=b"\x02" * 32, idx=3)})
    assert [p.share_idx for p in reached[0][2]] == [2, 3]
    # DutySignature ignores message roots (memory.go:198-201)
    sig_duty = Duty(1, parsig.DUTY_SIGNATURE)
    db.store_external(sig_duty, {"a": _pd(root=b"\x01" * 32, idx=1)})
    assert db.store_external(sig_duty, {"a": _pd(root=b"\x02" * 32, idx=2)})


def test_memdb_internal_subscribers():
    db = parsig.MemDB(threshold=2)
    seen = []
    db.subscribe_internal(lambda d, s: seen.append(sorted(s)))
    db.store_internal(Duty(2, parsig.DUTY_RANDAO), {"a": _pd(), "b": _pd()})
    assert seen == [["a", "b"]]


def test_aggregator_host_errors():
    agg = parsig.Aggregator(threshold=3, engine=NoEngine())
    duty = Duty(1, parsig.DUTY_ATTESTER)
    out = agg.aggregate_batch([(duty, "a", [_pd(idx=1), _pd(idx=2)])])
    assert str(out[0]) == "require threshold signatures"
    with pytest.raises(parsig.ParSigError, match="invalid threshold config"):
        parsig.Aggregator(threshold=0, engine=NoEngine()).aggregate(duty, "a", [])


def test_fixture_expectations_match_oracle():
    """Pin parsig_sets.json's per-set verdicts with the CPU oracle."""
    from oracle import bls12_381 as bls
    from oracle import tbls_oracle as tb
    fx = load_fixture()
    spec = fixture_spec(fx)
    shares = {d["pubkey"]: {int(k): v for k, v in d["pubshares"].items()} for d in fx["dvs"]}
    for s in fx["sets"]:
        first = None
        for it in s["items"]:
            if it["pubkey"] not in shares:
                err = "unknown pubkey"
            elif it["share_idx"] not in shares[it["pubkey"]]:
                err = "invalid shareIdx"
            elif it["sig"] == "00" * 96:
                err = "no signature found"
            else:
                try:
                    sig = bls.g2_decompress(bytes.fromhex(it["sig"]))
                except bls.DecodeError:
                    err = "uncompress sig"
                else:
                    pk = bls.g1_decompress(bytes.fromhex(shares[it["pubkey"]][it["share_idx"]]))
                    msg = signing.get_data_root(spec, it["domain"], it["epoch"], bytes.fromhex(it["message_root"]))
                    err = None if tb.verify(pk, msg, sig) else "invalid signature"
            if err is not None and first is None:
                first = err
        assert first == s["expect_error"], (s["duty"], s["peer"], s["fault"])
