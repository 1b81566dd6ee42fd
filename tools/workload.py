"""Synthetic Charon workloads for the bench and the full-size GPU tests.

A batch is n_dv distributed validators (t-of-n threshold clusters), each
signing one 32-byte signing root: group secret -> Shamir shares (x = 1..n) ->
pubshares and partial signatures, all generated on the GPU with the engine's
test-vector entry points (tbg_sk_to_pk / tbg_sign; reference tbls.PartialSign,
tss.go:200-207).  Seeds are explicit so the CPU baseline and the GPU run use
the same inputs.  Optional injection replaces a fraction of partials with a
signature over a different message (a "wrong-message" partial).
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


def _scalars(rng, count):
    out = []
    raw = rng.integers(0, 2 ** 63, size=(count, 5), dtype=np.int64)
    for row in raw.tolist():
        v = 0
        for w in row:
            v = (v << 63) | int(w)
        out.append(v % (R - 1) + 1)
    return out


def make_batch(engine, n_dv, t, n, seed, inject=0.0, pk_offset=None):
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
    first, st = engine.load_pubkeys(pubshares)
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
        secrets=secrets, shares=shares, msgs=msgs)
