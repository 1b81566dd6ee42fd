#!/usr/bin/env python3
"""Generate tests/golden/parsig_sets.json: peer partial-signature sets for the
batch-aware parsigex -> parsigdb -> sigagg path, signed
by the CPU oracle (oracle/tbls_oracle.py, pinned by tests/test_oracle_kat.py).

One 3-of-4 cluster of DVs.  Every peer (share index 1..4) sends one set per
duty, {DV group pubkey: partial}; each partial signs the eth2 signing root
  hash_tree_root(SigningData{object_root, compute_domain(type, fork, gvr)})
(consensus-specs; reference eth2util/signing/signing.go:73-85) under a fork
schedule with a fork at epoch 10.  Injected faults, each dropping its whole
set (parsigex.go:101-107): a partial signed over the pre-fork domain, a zero
signature, a share index outside the cluster, an unknown DV pubkey, a
partial signed by another share, random bytes.  Expected: the error class per
set, and per (duty, DV) the aggregate = Sign(group secret, signing root).

Run:  python tests/golden/make_parsig_golden.py
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

SEED = 0x9A51
T, N, N_DV = 3, 4, 4
FORKS = [(0, "00001020"), (10, "01001020")]
# (duty name, core.DutyType, domain name, domain type, epoch, slot)
DUTIES = [
    ("attester", 2, "DOMAIN_BEACON_ATTESTER", "01000000", 12, 12 * 32 + 5),
    ("randao", 7, "DOMAIN_RANDAO", "02000000", 3, 3 * 32 + 1),
    ("sync_message", 10, "DOMAIN_SYNC_COMMITTEE", "07000000", 11, 11 * 32 + 9),
    ("proposer", 1, "DOMAIN_BEACON_PROPOSER", "00000000", 10, 10 * 32),
]


def sha(b):
    return hashlib.sha256(b).digest()


def domain(dtype_hex, epoch, gvr):
    version = FORKS[0][1]
    for start, v in FORKS:
        if epoch >= start:
            version = v
    return bytes.fromhex(dtype_hex) + sha(bytes.fromhex(version) + bytes(28) + gvr)[:28]


def main():
    rng = random.Random(SEED)
    gvr = bytes(rng.getrandbits(8) for _ in range(32))
    dvs = []
    for _ in range(N_DV):
        secret = rng.randrange(1, bls.R)
        coeffs = [rng.randrange(1, bls.R) for _ in range(T - 1)]
        tss, shares = tb.generate_tss(secret, T, N, coeffs)
        dvs.append((secret, tss, shares))
    pubkeys = [bls.g1_compress(tss.public_key).hex() for _, tss, _ in dvs]

    faults = {  # (duty index, peer) -> fault injected into that peer's set
        (0, 2): "pre_fork_domain",   # duties 0 and 1 keep 3 clean sets: aggregated
        (1, 3): "zero_signature",
        (2, 4): "bad_share_idx",     # duties 2 and 3 keep 2: below threshold
        (2, 1): "wrong_share",
        (3, 4): "unknown_pubkey",
        (3, 2): "random_bytes",
    }
    expect_err = {"pre_fork_domain": "invalid signature", "zero_signature": "no signature found",
                  "bad_share_idx": "invalid shareIdx", "unknown_pubkey": "unknown pubkey",
                  "wrong_share": "invalid signature", "random_bytes": "uncompress sig"}
    sets, aggregates, roots = [], [], []
    for di, (name, dtype, dname, dtype_hex, epoch, slot) in enumerate(DUTIES):
        obj = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in dvs]
        sroots = [sha(o + domain(dtype_hex, epoch, gvr)) for o in obj]
        for k, (secret, _, _) in enumerate(dvs):
            aggregates.append({"duty": di, "pubkey": pubkeys[k],
                               "agg": bls.g2_compress(tb.sign(secret, sroots[k])).hex()})
            roots.append({"domain": dname, "epoch": epoch, "object_root": obj[k].hex(), "signing_root": sroots[k].hex()})
        for peer in range(1, N + 1):
            fault = faults.get((di, peer))
            victim = rng.randrange(N_DV)
            items = []
            for k, (_, _, shares) in enumerate(dvs):
                share_idx, pk, root, sig = peer, pubkeys[k], sroots[k], None
                if k == victim and fault == "pre_fork_domain":
                    root = sha(obj[k] + domain(dtype_hex, 0, gvr))
                elif k == victim and fault == "zero_signature":
                    sig = bytes(96)
                elif k == victim and fault == "bad_share_idx":
                    share_idx = N + 5
                elif k == victim and fault == "unknown_pubkey":
                    pk = bls.g1_compress(tb.sk_to_pk(rng.randrange(1, bls.R))).hex()
                elif k == victim and fault == "random_bytes":
                    sig = bytes([0x80 | rng.getrandbits(5)]) + bytes(rng.getrandbits(8) for _ in range(95))
                signer = shares[peer % N + 1] if (k == victim and fault == "wrong_share") else shares[peer]
                if sig is None:
                    sig = bls.g2_compress(tb.sign(signer, root))
                items.append({"pubkey": pk, "share_idx": share_idx, "domain": dname, "epoch": epoch,
                              "message_root": obj[k].hex(), "sig": sig.hex()})
            sets.append({"duty": di, "slot": slot, "duty_type": dtype, "peer": peer, "fault": fault,
                         "expect_error": expect_err.get(fault), "items": items})
    out = {"generator": "tests/golden/make_parsig_golden.py", "seed": hex(SEED), "threshold": T,
           "num_shares": N, "forks": FORKS, "genesis_validators_root": gvr.hex(),
           "dvs": [{"pubkey": pubkeys[k],
                    "pubshares": {str(i): bls.g1_compress(pk).hex() for i, pk in sorted(tss.pubshares.items())}}
                   for k, (_, tss, _) in enumerate(dvs)],
           "duties": [{"name": d[0], "duty_type": d[1], "domain": d[2], "epoch": d[4], "slot": d[5]} for d in DUTIES],
           "signing_roots": roots, "sets": sets, "aggregates": aggregates}
    with open(os.path.join(HERE, "parsig_sets.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("parsig_sets.json", len(sets), "sets,", len(aggregates), "aggregates")


if __name__ == "__main__":
    main()
