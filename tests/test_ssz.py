"""Signing roots in front of the hot path (include/tbls_ssz.h, host code of
libtbls_gpu.so): the oracle (oracle/ssz_oracle.py) against the reference's
own vectors, and the native batch against the oracle -- every kind, both
SHA-256 implementations, one and several threads, per-object domains.
Host-only: no GPU call is made."""
import json
import os
import random
import struct
import subprocess
import sys

import pytest

from oracle import ssz_oracle as so

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "ssz_vectors.json")))
H = bytes.fromhex


def native():
    from charon_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libtbls_gpu.so not built (run __graft_entry__.build())")
    from charon_amd import ssz
    return ssz


# ----------------------------------------------------------- oracle pinning
def test_oracle_reference_uint64_roots():
    for v in GOLD["slot_hash_root"]:
        assert so.u64(v["slot"]).hex() == v["root"]          # eth2util/hash_test.go:27-34
    for v in GOLD["epoch_root"]:
        assert so.u64(v["epoch"]).hex() == v["root"]         # eth2util/types_test.go:27-36


def test_oracle_reference_attestation_pipeline():
    """validatorapi_test.go:230-289: domain, AttestationData root, signing root,
    and the signature of sk = 1 over it verifies."""
    v = GOLD["sign_and_verify_attestation"]
    dom = so.compute_domain(H(v["domain_type"]), H(v["fork_version"]), H(v["genesis_validators_root"]))
    assert dom.hex() == v["domain"]
    root = so.attestation_data_root(v["slot"], v["index"], H(v["beacon_block_root"]), v["source"]["epoch"],
                                    H(v["source"]["root"]), v["target"]["epoch"], H(v["target"]["root"]))
    assert root.hex() == v["attestation_data_root"]
    assert so.signing_root(root, dom).hex() == v["signing_root"]
    from oracle import bls12_381 as bls
    from oracle import tbls_oracle as tb
    sk = int(v["secret_key"], 16)
    assert bls.g2_compress(tb.sign(sk, H(v["signing_root"]))).hex() == v["signature"]


def test_oracle_reference_deposits():
    """The deposit golden file: message and data roots; its signatures are
    checked over these roots in test_oracle_kat / the GPU test below."""
    for d in GOLD["deposits"]:
        args = (H(d["pubkey"]), H(d["withdrawal_credentials"]), d["amount"])
        assert so.deposit_message_root(*args).hex() == d["deposit_message_root"]
        assert so.deposit_data_root(*args, H(d["signature"])).hex() == d["deposit_data_root"]


def test_oracle_reference_registration():
    v = GOLD["validator_registration"]
    root = so.validator_registration_root(H(v["fee_recipient"]), v["gas_limit"], v["timestamp"], H(v["pubkey"]))
    assert root.hex() == v["root"]
    from oracle import bls12_381 as bls
    from oracle import tbls_oracle as tb
    assert bls.g1_compress(tb.sk_to_pk(int(v["signer_secret"], 16))).hex() == v["signer_pubkey"]


# ------------------------------------------------------------ native parity
KIND_NAMES = ["root", "uint64", "attestation_data", "voluntary_exit", "sync_agg_selection",
              "validator_registration", "deposit_message", "deposit_data", "fork_data", "signing_data",
              "checkpoint"]
SIZES = [32, 8, 128, 16, 16, 84, 88, 184, 36, 64, 40]


def random_objects(kind, n, rng):
    objs = []
    for _ in range(n):
        b = bytearray(rng.getrandbits(8) for _ in range(SIZES[kind]))
        if rng.random() < 0.2:  # edge integers: 0 and 2^64 - 1 at every uint64 slot of the layout
            b[0:8] = struct.pack("<Q", rng.choice([0, 2 ** 64 - 1]))
        objs.append(bytes(b))
    return objs


def test_native_sizes_and_bad_args():
    ssz = native()
    from charon_amd import _native
    lib = _native.load()
    for k, sz in enumerate(SIZES):
        assert ssz.size(k) == sz
    assert lib.tbg_ssz_size(99) == 0
    assert lib.tbg_ssz_roots(99, b"", 0, None, 0) == -1
    with pytest.raises(ssz.SSZError):
        ssz.signing_roots([bytes(16)], [bytes(32)], domain_idx=[1], kind=ssz.VOLUNTARY_EXIT)
    with pytest.raises(ssz.SSZError):
        ssz.hash_tree_roots([bytes(15)], kind=ssz.VOLUNTARY_EXIT)
    assert ssz.hash_tree_roots([], kind=ssz.ROOT) == []


@pytest.mark.parametrize("kind", range(len(SIZES)))
def test_native_roots_match_oracle(kind):
    ssz = native()
    rng = random.Random(1000 + kind)
    objs = random_objects(kind, 300, rng)
    got = ssz.hash_tree_roots(objs, kind=kind, threads=1)
    assert got == [so.root_of_serialized(KIND_NAMES[kind], o) for o in objs]


def test_native_reference_vectors():
    ssz = native()
    v = GOLD["sign_and_verify_attestation"]
    att = ssz.AttestationData(v["slot"], v["index"], H(v["beacon_block_root"]),
                              ssz.Checkpoint(v["source"]["epoch"], H(v["source"]["root"])),
                              ssz.Checkpoint(v["target"]["epoch"], H(v["target"]["root"])))
    dom = ssz.compute_domain(H(v["domain_type"]), H(v["fork_version"]), H(v["genesis_validators_root"]))
    assert dom.hex() == v["domain"]
    assert ssz.hash_tree_roots([att])[0].hex() == v["attestation_data_root"]
    assert ssz.signing_roots([att], [dom])[0].hex() == v["signing_root"]
    assert ssz.hash_tree_roots([ssz.Slot(2)])[0].hex() == GOLD["slot_hash_root"][0]["root"]
    assert ssz.hash_tree_roots([ssz.Epoch(2)])[0].hex() == GOLD["epoch_root"][0]["root"]
    deps = GOLD["deposits"]
    msgs = [ssz.DepositMessage(H(d["pubkey"]), H(d["withdrawal_credentials"]), d["amount"]) for d in deps]
    data = [ssz.DepositData(H(d["pubkey"]), H(d["withdrawal_credentials"]), d["amount"], H(d["signature"]))
            for d in deps]
    assert [r.hex() for r in ssz.hash_tree_roots(msgs)] == [d["deposit_message_root"] for d in deps]
    assert [r.hex() for r in ssz.hash_tree_roots(data)] == [d["deposit_data_root"] for d in deps]
    r = GOLD["validator_registration"]
    reg = ssz.ValidatorRegistration(H(r["fee_recipient"]), r["gas_limit"], r["timestamp"], H(r["pubkey"]))
    assert ssz.hash_tree_roots([reg])[0].hex() == r["root"]


def test_native_threads_and_domains():
    """A large batch split over threads, per-object domains, equals the
    single-threaded oracle."""
    ssz = native()
    rng = random.Random(7)
    objs = random_objects(ssz.ATTESTATION_DATA, 6000, rng)
    domains = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(5)]
    idx = [rng.randrange(5) for _ in objs]
    want = [so.signing_root(so.root_of_serialized("attestation_data", o), domains[i]) for o, i in zip(objs, idx)]
    for threads in (1, 3, 8):
        assert ssz.signing_roots(objs, domains, idx, kind=ssz.ATTESTATION_DATA, threads=threads) == want
    one = ssz.signing_roots(objs[:50], domains[2:3], kind=ssz.ATTESTATION_DATA)
    assert one == [so.signing_root(so.root_of_serialized("attestation_data", o), domains[2]) for o in objs[:50]]


def test_native_portable_sha_path():
    """The same parity with the SHA extensions disabled (TBG_SHA_PORTABLE=1 is
    read once at load, so it runs in a child process)."""
    native()
    code = ("import random;from charon_amd import ssz;from oracle import ssz_oracle as so;"
            "from tests.test_ssz import random_objects, KIND_NAMES\n"
            "rng=random.Random(3)\n"
            "for k in range(11):\n"
            "  objs=random_objects(k,64,rng)\n"
            "  assert ssz.hash_tree_roots(objs,kind=k)==[so.root_of_serialized(KIND_NAMES[k],o) for o in objs], k\n"
            "print('ok')")
    env = dict(os.environ, TBG_SHA_PORTABLE="1", PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr[-2000:]


def test_signing_module_uses_native_roots():
    """charon_amd.signing's per-item GetDataRoot equals the native batch."""
    ssz = native()
    from charon_amd import signing
    spec = signing.Spec(forks=[(0, H("00001020")), (10, H("01001020"))], genesis_validators_root=H("11" * 32))
    rng = random.Random(5)
    roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(40)]
    epochs = [rng.randrange(20) for _ in roots]
    got = signing.get_data_roots(spec, signing.DOMAIN_BEACON_ATTESTER, epochs, roots)
    assert got == [signing.get_data_root(spec, signing.DOMAIN_BEACON_ATTESTER, e, r) for e, r in zip(epochs, roots)]
