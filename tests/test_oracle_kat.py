"""Pin the CPU oracle to the known-answer vectors the reference's own tests hold.

Sources (reference, read-only; values copied here as data):
  * eth2util/deposit/deposit_test.go:41-46 (secret keys) and
    eth2util/deposit/testdata/TestMarshalDepositData.golden (pubkey, signature,
    deposit_message_root per key; goerli fork version 00001020).
  * eth2util/keystore/keystore_test.go:64 + testdata/keystore-scrypt.json.
  * eth2util/signing/signing_test.go:34-80 (Teku builder-registration vector).
"""
import hashlib

import pytest

from oracle import bls12_381 as bls
from oracle import tbls_oracle as tb

DEPOSIT_SKS = [
    "01477d4bfbbcebe1fef8d4d6f624ecbb6e3178558bb1b0d6286c816c66842a6d",
    "5b77c0f0ef7c4ddc123d55b8bd93daeefbd7116764a941c0061a496649e145b5",
    "1dabcbfc9258f0f28606bf9e3b1c9f06d15a6e4eb0fbc28a43835eaaed7623fc",
    "002ff4fd29d3deb6de9f5d115182a49c618c97acaa365ad66a0b240bd825c4ff",
]
# (pubkey, signature, deposit_message_root) from TestMarshalDepositData.golden
DEPOSIT_GOLDEN = [
    ("80d0436ccacd2b263f5e9e7ebaa14015fe5c80d3e57dc7c37bcbda783895e3491019d3ed694ecbb49c8c80a0480c0392",
     "8e383948b4909a20e16c17883148adf56234c19540995830a1908720cbdf4bed309568fefbb40bec4b7f8b4b3df9e19016afb25d76899ec6e1cc7259abe5de6e7b9b04723014ebef47852925c4dd3ff343caeeeb5b4ed499c9d5be2cda1f8b84",
     "4f5f7044a71d625c59974e32e8d86aed0a2211d423675303124ce5ac70969a46"),
    ("813f5d2697f76841a752ef8c1ac11d1bb76e07003799c5745f8a569214653810def3b60920b54fb0ab3cb6deb08c3972",
     "b5f95360b98cb6db3c06998b43b1dce29aea4f085950018d9dbd3c9894941f4804c449c771392ed3dde1091d346d71c316273c7213237dfa6b9ea79fbcfe79b055a5880d309f5db2dcf3e9a0fee6a4c843f3adb5835958b0561996218cd63acf",
     "33109737473d6ccb5f3c4f7eccaa4a7cd3dd63de3d9878a978243053904d39bf"),
    ("940a838cd88c10daa9c26fcdf8472dfe09657c4aa4030380c6cca5ddb573a8036dfb03e61137c4baacdc9d69061f1eb2",
     "b8e638af308c9e1a1dfac291c7b0218dc3c1dc9baa000dbee0539ed6805cd76afd06fd50797e8192cf917d51c712c31212670e521e0cf326fadbbd8f361fa7a1e0fc80bc77279c71ddd2505835ec3da74a742a5ca19a635c6889915ef3a2dd89",
     "8cec1018fcfcb6ae295546901f1c55e2f2643834b89c9a00e4806d8c6b197169"),
    ("b3d95c8790d63114ab1e813e8943f1bd59683927942df076ad724de8cc00974306c95d6614ef93505b5acd9719a6de78",
     "a4f5fac20a37a109200594ab9ee3bf983aab4aea6202fab637e7e79b9bbae37cef5815c746bdf01a57e659605346a9b80d4efe7e0884de144dcff28d07838a58819f03dd8fc2b48ea14e62222390fe3cb0284010f6acdcb1c4b5eb4c46a02560",
     "6b6860824055330be4cb0a378a1ffd342e4de77fef1d51621d44419c4b313ca9"),
]
KEYSTORE_SK = "10b16fc552aa607fa1399027f7b86ab789077e470b5653b338693dc2dde02468"
KEYSTORE_PK = "affcbf73c0609899141340513dc85f0ab2b6099e7beb700b7dbc000bcefc25b621405a6b9e29578f708bfd443332202c"
TEKU_SK = "345768c0245f1dc702df9e50e811002f61ebb2680b3d5931527ef59f96cbaf9b"
TEKU_SIG = ("b101da0fc08addcc5d010ee569f6bbbdca049a5cb27efad231565bff2e3af504ec2bb87b11ed22843e9c1094f1dfe51a0b2a5"
            "ad1808df18530a2f59f004032dbf6281ecf0fc3df86d032da5b9d32a3d282c05923de491381f8f28c2863a00180")


def _sha(b):
    return hashlib.sha256(b).digest()


def deposit_signing_root(msg_root_hex):
    # compute_domain(DOMAIN_DEPOSIT, fork 00001020, genesis_validators_root = 0)
    fork_data_root = _sha(bytes.fromhex("00001020") + bytes(28) + bytes(32))
    domain = bytes.fromhex("03000000") + fork_data_root[:28]
    return _sha(bytes.fromhex(msg_root_hex) + domain)


def teku_signing_root():
    # hash_tree_root(ValidatorRegistration{fee_recipient, gas_limit, timestamp, pubkey})
    pk = bytes.fromhex("86966350b672bd502bfbdb37a6ea8a7392e8fb7f5ebb5c5e2055f4ee168ebfab0fef63084f28c9f62c3ba71f825e527e")
    leaves = [bytes.fromhex("000000000000000000000000000000000000dead") + bytes(12),
              (30000000).to_bytes(8, "little") + bytes(24),
              (1646092800).to_bytes(8, "little") + bytes(24),
              _sha(pk + bytes(16))]
    root = _sha(_sha(leaves[0] + leaves[1]) + _sha(leaves[2] + leaves[3]))
    assert root.hex() == "2c231b16a80337212ab1decde301bdb4383e74c0bf2f3439cc82542bf0f90fdd"
    fork_data_root = _sha(bytes.fromhex("00001020") + bytes(28) + bytes(32))
    domain = bytes.fromhex("00000001") + fork_data_root[:28]
    return _sha(root + domain)


def test_generators_on_curve_and_in_subgroup():
    assert bls.g1_on_curve(bls.G1_GEN) and bls.g2_on_curve(bls.G2_GEN)
    assert bls.g1_in_subgroup(bls.G1_GEN) and bls.g2_in_subgroup(bls.G2_GEN)


@pytest.mark.parametrize("i", range(4))
def test_deposit_kat_pubkey(i):
    pk = tb.sk_to_pk(int(DEPOSIT_SKS[i], 16))
    assert bls.g1_compress(pk).hex() in {g[0] for g in DEPOSIT_GOLDEN}


@pytest.mark.parametrize("i", range(4))
def test_deposit_kat_signature_and_verify(i):
    pk_to_sk = {bls.g1_compress(tb.sk_to_pk(int(s, 16))).hex(): int(s, 16) for s in DEPOSIT_SKS}
    pk_hex, sig_hex, msg_root = DEPOSIT_GOLDEN[i]
    sk = pk_to_sk[pk_hex]
    root = deposit_signing_root(msg_root)
    sig = tb.sign(sk, root)
    assert bls.g2_compress(sig).hex() == sig_hex
    pk = bls.g1_decompress(bytes.fromhex(pk_hex))
    dec = bls.g2_decompress(bytes.fromhex(sig_hex))
    assert dec == sig
    assert tb.verify(pk, root, dec)
    assert not tb.verify(pk, root[:-1] + bytes([root[-1] ^ 1]), dec)


def test_keystore_kat():
    assert bls.g1_compress(tb.sk_to_pk(int(KEYSTORE_SK, 16))).hex() == KEYSTORE_PK


def test_teku_kat():
    sk = int(TEKU_SK, 16)
    root = teku_signing_root()
    sig = tb.sign(sk, root)
    assert bls.g2_compress(sig).hex() == TEKU_SIG
    assert tb.verify(tb.sk_to_pk(sk), root, bls.g2_decompress(bytes.fromhex(TEKU_SIG)))


def test_final_exp_matches_plain_exponent():
    f = bls.miller_loop(bls.G1_GEN, bls.G2_GEN)
    a = bls.final_exp(f)
    b = bls.final_exp_plain(f)
    assert a == bls.f12_mul(bls.f12_mul(b, b), b)


def test_pairing_bilinear():
    e1 = bls.pairing(bls.g1_mul(bls.G1_GEN, 7), bls.G2_GEN)
    e2 = bls.pairing(bls.G1_GEN, bls.g2_mul(bls.G2_GEN, 7))
    assert e1 == e2 and e1 != bls.F12_ONE


def test_iso_map_lands_on_e2():
    import random
    rng = random.Random(5)
    for _ in range(4):
        u = (rng.randrange(bls.P), rng.randrange(bls.P))
        q = bls.map_to_curve_g2(u)
        assert bls.g2_on_curve(q)


def test_decode_rejections():
    good = bytes.fromhex(DEPOSIT_GOLDEN[0][1])
    with pytest.raises(bls.DecodeError):
        bls.g2_decompress(bytes([good[0] & 0x7F]) + good[1:])  # compression flag cleared
    with pytest.raises(bls.DecodeError):
        bls.g2_decompress(bytes([0xC0]) + bytes(94) + b"\x01")  # infinity with x != 0
    assert bls.g2_decompress(bytes([0xC0]) + bytes(95)) is None  # identity
    with pytest.raises(bls.DecodeError):
        bls.g2_decompress(bytes([0x9F]) + b"\xff" * 95)  # x >= p


def test_identifier_zero_aggregate():
    # dkg/dkg_test.go:174-195: identifiers start at 0; lambda_0(0) = 1, others 0.
    sigs = [(j, tb.sign(11 + j, b"data")) for j in range(3)]
    assert tb.aggregate(sigs) == sigs[0][1]


def test_threshold_aggregate_equals_group_signature():
    secret = 0x1234567890ABCDEF
    tss, shares = tb.generate_tss(secret, 3, 4, [777, 999])
    msg = b"Hello Obol"
    partials = [(i, tb.sign(shares[i], msg)) for i in (1, 2, 3, 4)]
    agg, signers = tb.verify_and_aggregate(tss, partials, msg)
    assert signers == [1, 2, 3, 4]
    assert agg == tb.sign(secret, msg)
    # any 3-subset gives the same group element
    assert tb.aggregate([partials[0], partials[1], partials[3]]) == agg
