"""Writes tests/golden/dkg_vectors.json and tests/golden/cluster_locks.json,
the fixtures of the DKG / cluster-lock GPU tests (charon_amd.dkg).

dkg_vectors.json -- computed by the oracle (oracle/tbls_oracle.py):
  deposit: each deposit key of the reference's golden file
    (eth2util/deposit/testdata/TestMarshalDepositData.golden; secret keys
    from eth2util/deposit/deposit_test.go:40-46) split 3-of-4, every share
    partially signing the deposit signing root; the threshold aggregate must
    be the golden file's signature, bit for bit (checked here and on the GPU).
  lock: the same three DVs' shares sign one lock hash; the expected
    AggregateSignatures / AggregatePublicKeys are the oracle's point sums
    (dkg/dkg.go:466-476), and they verify (VerifyMultiSignature, :377).
cluster_locks.json -- the reference's cluster lock files
  (cluster/testdata/cluster_lock_v1_*.json), reduced to the fields
  Lock.VerifySignatures reads (cluster/lock.go:137-179).

Run from the repo root:  python tests/golden/make_dkg_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import tbls_oracle as tb  # noqa: E402
from tests.test_oracle_kat import DEPOSIT_GOLDEN, DEPOSIT_SKS, deposit_signing_root  # noqa: E402

REF_LOCKS = "/root/reference/cluster/testdata"


def hx(b):
    return bytes(b).hex()


def main():
    rng = random.Random(20261016)
    pk_to_sk = {bls.g1_compress(tb.sk_to_pk(int(s, 16))).hex(): int(s, 16) for s in DEPOSIT_SKS}
    dvs = []
    for pk_hex, sig_hex, msg_root in DEPOSIT_GOLDEN:
        sk = pk_to_sk[pk_hex]
        shares, _ = tb.split_secret(sk, 3, 4, [rng.randrange(1, bls.R) for _ in range(2)])
        root = deposit_signing_root(msg_root)
        partials = {i: tb.sign(s, root) for i, s in shares.items()}
        combined = tb.combine_signatures([(i, p) for i, p in partials.items()])
        assert bls.g2_compress(combined).hex() == sig_hex  # the golden deposit signature
        dvs.append({"pubkey": pk_hex, "signing_root": hx(root), "aggregate": sig_hex,
                    "pubshares": {str(i): hx(bls.g1_compress(tb.sk_to_pk(s))) for i, s in shares.items()},
                    "shares": shares, "partials": {str(i): hx(bls.g2_compress(p)) for i, p in partials.items()}})
    lock_hash = hashlib.sha256(b"cluster lock hash").digest()
    lock_partials, sum_sig, sum_pk = [], None, None
    for dv in dvs[:3]:
        for i, s in dv["shares"].items():
            sig = tb.sign(s, lock_hash)
            lock_partials.append({"pubkey": dv["pubkey"], "share_idx": i, "sig": hx(bls.g2_compress(sig))})
            sum_sig = sig if sum_sig is None else bls.g2_add(sum_sig, sig)
            pk = tb.sk_to_pk(s)
            sum_pk = pk if sum_pk is None else bls.g1_add(sum_pk, pk)
    assert tb.core_verify(sum_pk, lock_hash, sum_sig)
    for dv in dvs:
        del dv["shares"]
    out = {"deposit": dvs,
           "lock": {"hash": hx(lock_hash), "partials": lock_partials, "aggregate_signature": hx(bls.g2_compress(sum_sig)),
                    "aggregate_pubkey": hx(bls.g1_compress(sum_pk))}}
    json.dump(out, open(os.path.join(HERE, "dkg_vectors.json"), "w"), indent=1)
    if os.path.isdir(REF_LOCKS):
        locks = []
        for v in ["1_0_0", "1_1_0", "1_2_0", "1_3_0", "1_4_0"]:
            d = json.load(open(os.path.join(REF_LOCKS, f"cluster_lock_v{v}.json")))
            locks.append({"cluster_definition": {"version": d["cluster_definition"]["version"]},
                          "signature_aggregate": d["signature_aggregate"], "lock_hash": d.get("lock_hash"),
                          "distributed_validators": [{"public_shares": dv["public_shares"]}
                                                     for dv in d["distributed_validators"]]})
        json.dump(locks, open(os.path.join(HERE, "cluster_locks.json"), "w"), indent=1)
    print("wrote dkg_vectors.json" + (" and cluster_locks.json" if os.path.isdir(REF_LOCKS) else ""))


if __name__ == "__main__":
    main()
