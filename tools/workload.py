"""Synthetic Charon workloads for the bench and the full-size GPU tests.

A batch is n_dv distributed validators (t-of-n threshold clusters), each
signing one 32-byte signing root: group secret -> Shamir shares (x = 1..n) ->
pubshares and partial signatures, all generated on the GPU with the engine's
test-vector entry points (tbg_sk_to_pk / tbg_sign; reference tbls.PartialSign,
tss.go:200-207).  Seeds are explicit so the CPU baseline and the GPU run use
the same inputs.  make_batch's optional injection replaces a fraction of
partials with a signature over a different message (a "wrong-message"
partial); make_mixed_batch (config 5) injects every kind of invalid partial
the reference rejects (INJECT_KINDS).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


@dataclass
class ClusterBatch:
    n_dv: int
    t: int
    n: int
    duty_first: np.ndarray   # uint32 [n_dv + 1]
    sigs: np.ndarray         # uint8 [n_dv * n, 96]
    identifiers: np.ndarray  # uint8 [n_dv * n]
    pubkey_ids: np.ndarray   # uint32 [n_dv * n]
    pubshares: np.ndarray    # uint8 [n_dv * n, 48]
    msg_data: np.ndarray     # uint8 concatenated messages
    msg_off: np.ndarray      # uint32 [n_dv + 1]
    duty_msg: np.ndarray     # uint32 [n_dv]
    threshold: np.ndarray    # uint32 [n_dv]
    group_sig: np.ndarray    # uint8 [n_dv, 96]
    injected: np.ndarray     # bool [n_dv * n]
    expect_ok: np.ndarray    # bool [n_dv]
    secrets: list            # group secrets (ints)
    shares: list             # per partial share scalars (ints)
    msgs: list               # per DV message bytes
    pk_first: int = 0        # resident id of pubshares[0] in the engine that loaded them
    inject_kind: np.ndarray = None  # int8 [n_dv * n]: index into INJECT_KINDS, -1 if not injected (mixed batches)


def _scalars(rng, count):
    out = []
    raw = rng.integers(0, 2 ** 63, size=(count, 5), dtype=np.int64)
    for row in raw.tolist():
        v = 0
        for w in row:
            v = (v << 63) | int(w)
        out.append(v % (R - 1) + 1)
    return out


INJECT_KINDS = ("wrong_msg", "wrong_share", "random_bytes", "non_subgroup", "off_curve", "bad_flags", "identity",
                "missing_pubshare")
NO_PUBKEY = 0xFFFFFFFF


def invalid_pool():
    """Committed encodings that need curve arithmetic to find (a point on E2
    outside G2, an x with no point on E2): tests/golden/invalid_g2.json,
    written by tests/golden/make_golden.py.  Data only."""
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "invalid_g2.json")
    with open(path) as f:
        d = json.load(f)
    return {k: [bytes.fromhex(h) for h in v] for k, v in d["pools"].items()}


def _shares(secret, coeffs, ids):
    out = []
    poly = [secret] + list(coeffs)
    for x in ids:
        acc = 0
        for c in reversed(poly):
            acc = (acc * x + c) % R
        out.append(acc)
    return out


def make_mixed_batch(engine, n_dv, seed, inject=0.01, kinds=INJECT_KINDS, pool=None, committee=64,
                     thresholds=((3, 4), (5, 7), (7, 10)), load=None):
    """BASELINE config 5: mixed duties (attestation 90 %, sync committee 8 %,
    randao 1 %, proposal 1 %), thresholds drawn from
    `thresholds`, attestations of one committee (and the sync-committee
    duties of the batch) sharing one signing root, and a fraction `inject`
    of the partials replaced by an invalid one, cycling through `kinds`.
    `load` loads pubshares (defaults to engine.load_pubkeys)."""
    rng = np.random.default_rng(seed)
    pool = pool if pool is not None else (invalid_pool() if {"non_subgroup", "off_curve"} & set(kinds) else {})
    tn = [thresholds[i] for i in rng.integers(0, len(thresholds), size=n_dv)]
    duty_kind = rng.choice(4, size=n_dv, p=[0.90, 0.08, 0.01, 0.01])  # att, sync, randao, proposal
    secrets = _scalars(rng, n_dv)
    # messages: one per attestation committee, one for the sync duties, one per randao / proposal duty
    msgs, duty_msg = [], np.zeros(n_dv, dtype=np.uint32)
    att_seen = 0
    sync_msg = None
    for d in range(n_dv):
        k = duty_kind[d]
        if k == 0:
            if att_seen % committee == 0:
                msgs.append(rng.bytes(32))
            att_seen += 1
            duty_msg[d] = len(msgs) - 1
        elif k == 1:
            if sync_msg is None:
                msgs.append(rng.bytes(32))
                sync_msg = len(msgs) - 1
            duty_msg[d] = sync_msg
        else:
            msgs.append(rng.bytes(32))
            duty_msg[d] = len(msgs) - 1
    duty_first = np.zeros(n_dv + 1, dtype=np.uint32)
    duty_first[1:] = np.cumsum([n for _, n in tn])
    n_p = int(duty_first[-1])
    ids = np.concatenate([np.arange(1, n + 1, dtype=np.uint8) for _, n in tn])
    shares = []
    for d, (t, n) in enumerate(tn):
        shares += _shares(secrets[d], _scalars(rng, t - 1), range(1, n + 1))
    item_msg = np.repeat(duty_msg, [n for _, n in tn]).astype(np.uint32)
    sk32 = b"".join(s.to_bytes(32, "big") for s in shares)
    wrong = [m[:-1] + bytes([m[-1] ^ 0x5A]) for m in msgs]
    injected = rng.random(n_p) < inject
    kind_of = np.full(n_p, -1, dtype=np.int32)
    pos = np.flatnonzero(injected)
    kind_of[pos] = np.arange(len(pos)) % len(kinds)
    # signer of each partial: its own share, another share of its DV (wrong_share), own share on a wrong message
    signer = np.arange(n_p)
    sign_msg = item_msg.copy()
    part_duty = np.repeat(np.arange(n_dv), [n for _, n in tn])
    for p in pos:
        kind = kinds[kind_of[p]]
        d = part_duty[p]
        if kind == "wrong_share":
            lo, hi = int(duty_first[d]), int(duty_first[d + 1])
            signer[p] = lo + (p - lo + 1) % (hi - lo)
        elif kind == "wrong_msg":
            sign_msg[p] = item_msg[p] + len(msgs)
    sk_signer = b"".join(shares[s].to_bytes(32, "big") for s in signer)
    sigs = engine.sign(sk_signer, msgs + wrong, sign_msg)
    pubshares = engine.sk_to_pk(sk32)
    first, st = (load or engine.load_pubkeys)(pubshares)
    assert (st == 0).all()
    pubkey_ids = (first + np.arange(n_p)).astype(np.uint32)
    cyc = {}
    for p in pos:
        kind = kinds[kind_of[p]]
        if kind == "random_bytes":
            sigs[p] = np.frombuffer(rng.bytes(96), dtype=np.uint8)
        elif kind in ("non_subgroup", "off_curve"):
            lst = pool[kind]
            sigs[p] = np.frombuffer(lst[cyc.get(kind, 0) % len(lst)], dtype=np.uint8)
            cyc[kind] = cyc.get(kind, 0) + 1
        elif kind == "bad_flags":
            sigs[p, 0] &= 0x7F
        elif kind == "identity":
            sigs[p] = 0
            sigs[p, 0] = 0xC0
        elif kind == "missing_pubshare":
            pubkey_ids[p] = NO_PUBKEY
    group_sig = engine.sign(b"".join(s.to_bytes(32, "big") for s in secrets), msgs, duty_msg)
    valid_per_dv = np.add.reduceat((~injected).astype(np.int64), duty_first[:-1].astype(np.int64))
    thr = np.array([t for t, _ in tn], dtype=np.uint32)
    msg_off = np.arange(len(msgs) + 1, dtype=np.uint32) * 32
    return ClusterBatch(
        n_dv=n_dv, t=0, n=0, duty_first=duty_first, sigs=sigs, identifiers=ids, pubkey_ids=pubkey_ids,
        pubshares=pubshares, msg_data=np.frombuffer(b"".join(msgs), dtype=np.uint8), msg_off=msg_off,
        duty_msg=duty_msg, threshold=thr, group_sig=group_sig, injected=injected, expect_ok=valid_per_dv >= thr,
        secrets=secrets, shares=shares, msgs=msgs, pk_first=int(first), inject_kind=kind_of.astype(np.int8))


def make_batch(engine, n_dv, t, n, seed, inject=0.0, load=None):
    rng = np.random.default_rng(seed)
    secrets = _scalars(rng, n_dv)
    coeffs = _scalars(rng, n_dv * (t - 1))
    shares = []
    for d in range(n_dv):
        poly = [secrets[d]] + coeffs[d * (t - 1):(d + 1) * (t - 1)]
        for x in range(1, n + 1):
            acc = 0
            for c in reversed(poly):
                acc = (acc * x + c) % R
            shares.append(acc)
    msgs = [rng.bytes(32) for _ in range(n_dv)]
    wrong = [m[:-1] + bytes([m[-1] ^ 0xFF]) for m in msgs]
    n_p = n_dv * n
    injected = rng.random(n_p) < inject
    item_msg = np.repeat(np.arange(n_dv, dtype=np.uint32), n)
    item_msg = np.where(injected, item_msg + n_dv, item_msg).astype(np.uint32)
    sk32 = b"".join(s.to_bytes(32, "big") for s in shares)
    sigs = engine.sign(sk32, msgs + wrong, item_msg)
    pubshares = engine.sk_to_pk(sk32)
    first, st = (load or engine.load_pubkeys)(pubshares)
    assert (st == 0).all()
    group_sig = engine.sign(b"".join(s.to_bytes(32, "big") for s in secrets), msgs, np.arange(n_dv))
    valid_per_dv = (~injected).reshape(n_dv, n).sum(axis=1)
    msg_off = np.arange(n_dv + 1, dtype=np.uint32) * 32
    return ClusterBatch(
        n_dv=n_dv, t=t, n=n,
        duty_first=(np.arange(n_dv + 1, dtype=np.uint32) * n),
        sigs=sigs, identifiers=np.tile(np.arange(1, n + 1, dtype=np.uint8), n_dv),
        pubkey_ids=(first + np.arange(n_p)).astype(np.uint32), pubshares=pubshares,
        msg_data=np.frombuffer(b"".join(msgs), dtype=np.uint8), msg_off=msg_off,
        duty_msg=np.arange(n_dv, dtype=np.uint32), threshold=np.full(n_dv, t, dtype=np.uint32),
        group_sig=group_sig, injected=injected, expect_ok=valid_per_dv >= t,
        secrets=secrets, shares=shares, msgs=msgs, pk_first=int(first))
