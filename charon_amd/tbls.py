"""Host-side mirror of Charon's ``tbls`` package (reference tbls/tss.go) on the
MI355X engine.

Same names, argument meaning and error behaviour as the Go API, so that a
parity test reads like ``tbls/tss_test.go``:

  verify(pk, msg, sig) -> bool                         tss.go:190-197
  aggregate(partial_sigs) -> Signature                 tss.go:142-149
  verify_and_aggregate(tss, partial_sigs, msg)         tss.go:153-187
  TSS(pubshares, num_shares, threshold, public_key)    tss.go:62-116

plus the batch entry points the batch-aware call sites use:

  verify_batch(items) -> list[bool | TblsError]
  verify_and_aggregate_batch(duties) -> list[(Signature, signers) | TblsError]
  aggregate_batch(duties) -> list[Signature | TblsError]

Keys and signatures are carried as their wire encodings (48-byte G1 /
96-byte G2, ZCash-compressed); decoding, hashing, pairing and Lagrange
recombination all run on the GPU.  Errors follow the Go strings:
"uncompress sig" (tblsconv.go:128), "verify signature" (tss.go:193),
"aggregate signatures" (tss.go:145), "insufficient signatures" (tss.go:155),
"insufficient valid signatures" (tss.go:177).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import engine as eng


class TblsError(Exception):
    """Mirror of the Go ``error`` values returned by tbls / tblsconv."""


@dataclass(frozen=True)
class PublicKey:
    """bls_sig.PublicKey (48-byte compressed G1)."""
    raw: bytes

    def __post_init__(self):
        if len(self.raw) != 48:
            raise TblsError("unmarshal pubkey: invalid length")


@dataclass(frozen=True)
class Signature:
    """bls_sig.Signature (96-byte compressed G2)."""
    raw: bytes

    def __post_init__(self):
        if len(self.raw) != 96:
            raise TblsError("uncompress sig: invalid length")


@dataclass(frozen=True)
class PartialSignature:
    """bls_sig.PartialSignature{Identifier byte; Signature G2}."""
    identifier: int
    signature: Signature

    def __post_init__(self):
        if not 0 <= self.identifier <= 255:
            raise TblsError("identifier must fit a byte")


@dataclass
class TSS:
    """tbls.TSS: pubshares by share index, n, t, group public key."""
    pubshares: dict
    num_shares: int
    threshold: int
    public_key: PublicKey | None = None

    def public_share(self, share_idx: int):
        return self.pubshares.get(share_idx)

    def public_shares(self):
        return self.pubshares


_DECODE_ERRORS = {
    eng.PS_ERR_FLAGS: "compressed flag must be set / invalid infinity encoding",
    eng.PS_ERR_FIELD: "invalid bytes - not in field",
    eng.PS_ERR_CURVE: "point is not on the curve",
    eng.PS_ERR_SUBGROUP: "point is not in correct subgroup",
}
_DUTY_ERRORS = {
    eng.DS_INSUFFICIENT: "insufficient signatures",
    eng.DS_INSUFFICIENT_VALID: "insufficient valid signatures",
    eng.DS_AGG_TOO_FEW: "aggregate signatures: insufficient partial signatures",
    eng.DS_AGG_DUPLICATE_ID: "aggregate signatures: duplicate identifier",
    eng.DS_AGG_IDENTITY: "aggregate signatures: identity signature",
    eng.DS_DECODE: "uncompress sig",
}


class _PubkeyCache:
    """Resident pubkey ids per engine (the startup pubshare upload of
    app/app.go:334-376 happens here, lazily).  Every distinct key is uploaded
    (decoded into the device table) once per engine; its table id and decode
    status are kept, so repeated lookups never grow the device table."""

    def __init__(self):
        self.ids = {}
        self.status = {}

    def _load(self, e: eng.Engine, keys):
        """Upload the keys not resident yet; returns (id cache, status cache)."""
        cache = self.ids.setdefault(e.uid, {})
        stat = self.status.setdefault(e.uid, {})
        missing = [k for k in dict.fromkeys(keys) if k not in cache]
        if missing:
            first, st = e.load_pubkeys(b"".join(missing))
            for i, (k, s) in enumerate(zip(missing, st.tolist())):
                cache[k] = first + i
                stat[k] = int(s)
        return cache, stat

    def ids_for(self, e: eng.Engine, keys):
        cache, _ = self._load(e, keys)
        return [cache[k] for k in keys]

    def statuses_for(self, e: eng.Engine, keys):
        _, stat = self._load(e, keys)
        return [stat[k] for k in keys]


_pk_cache = _PubkeyCache()

_PK_ERRORS = {
    1: "public key is the identity",
    eng.PS_ERR_FLAGS: "compressed flag must be set / invalid infinity encoding",
    eng.PS_ERR_FIELD: "invalid bytes - not in field",
    eng.PS_ERR_CURVE: "point is not on the curve",
    eng.PS_ERR_SUBGROUP: "point is not in correct subgroup",
}


def key_from_bytes_batch(raws, engine=None):
    """tblsconv.KeyFromBytes (tblsconv.go:30-37) for many 48-byte keys at once:
    decoded and validated on the GPU (flags, field, curve, subgroup; the
    identity is refused as a public key), and made resident.  Per key returns
    a PublicKey or TblsError("unmarshal pubkey: ...")."""
    raws = [bytes(r) for r in raws]
    if not raws:
        return []
    e = _engine(engine)
    for r in raws:
        if len(r) != 48:
            raise TblsError("unmarshal pubkey: invalid length")
    out = []
    for r, s in zip(raws, _pk_cache.statuses_for(e, raws)):  # only keys not resident yet are uploaded
        if s == 0:
            out.append(PublicKey(r))
        else:
            out.append(TblsError("unmarshal pubkey: " + _PK_ERRORS.get(s, str(s))))
    return out


def wire_pubshares(validators, engine=None):
    """Startup pubshare wiring of app/app.go:334-376 (wireCoreWorkflow):
    ``validators`` maps a DV public key to its list of 48-byte pubshares (share
    index = list position + 1).  Every pubshare of the cluster is decoded in
    ONE GPU batch and stays resident for the verifies that follow; the first
    bad pubshare, in the reference's loop order, aborts with its
    KeyFromBytes error (app.go:347-350).  Returns {dv: {share_idx: PublicKey}}."""
    flat = [(dv, i, bytes(b)) for dv, shares in validators.items() for i, b in enumerate(shares)]
    keys = key_from_bytes_batch([b for _, _, b in flat], engine)
    out = {dv: {} for dv in validators}
    for (dv, i, _), k in zip(flat, keys):
        if isinstance(k, TblsError):
            raise k
        out[dv][i + 1] = k
    return out


def _engine(e):
    return e if e is not None else eng.default_engine()


def _raw(x, cls):
    if isinstance(x, cls):
        return x.raw
    return bytes(x)


# --------------------------------------------------------------------- batch API
def verify_batch(items, engine=None):
    """items: iterable of (pk, msg, sig).  Returns a list with True/False per
    item, or a TblsError for items whose encodings do not decode."""
    items = list(items)
    if not items:
        return []
    e = _engine(engine)
    pks = [_raw(pk, PublicKey) if pk is not None else None for pk, _, _ in items]
    present = [p for p in pks if p is not None]
    ids_present = iter(_pk_cache.ids_for(e, present))
    pk_ids = [next(ids_present) if p is not None else eng.NO_PUBKEY for p in pks]
    msgs = [bytes(m) for _, m, _ in items]
    sigs = b"".join(_raw(s, Signature) for _, _, s in items)
    n = len(items)
    res = e.run(eng.OP_VERIFY, np.arange(n + 1), sigs, np.zeros(n, np.uint8), msgs=msgs, duty_msg=np.arange(n),
                pubkey_ids=pk_ids)
    out = []
    for st in res.partial_status.tolist():
        if st == eng.PS_VALID:
            out.append(True)
        elif st in (eng.PS_INVALID, eng.PS_ERR_IDENTITY, eng.PS_ERR_PUBKEY):
            out.append(False)
        else:
            out.append(TblsError("uncompress sig: " + _DECODE_ERRORS.get(st, str(st))))
    return out


def _duty_arrays(duties, with_msg):
    duty_first = [0]
    sigs, ids, msgs, thr, pk_keys = [], [], [], [], []
    for d in duties:
        partials = d["partials"]
        for p in partials:
            sigs.append(_raw(p.signature, Signature))
            ids.append(p.identifier)
            if with_msg:
                pk = d["tss"].public_share(int(p.identifier))
                pk_keys.append(_raw(pk, PublicKey) if pk is not None else None)
        duty_first.append(duty_first[-1] + len(partials))
        if with_msg:
            msgs.append(bytes(d["msg"]))
            thr.append(d["tss"].threshold)
    return duty_first, b"".join(sigs), ids, msgs, thr, pk_keys


def verify_and_aggregate_batch(duties, engine=None):
    """duties: iterable of dicts {tss, partials, msg}.  Per duty returns
    (Signature, signers) or a TblsError, like tbls.VerifyAndAggregate."""
    duties = list(duties)
    if not duties:
        return []
    e = _engine(engine)
    duty_first, sigs, ids, msgs, thr, pk_keys = _duty_arrays(duties, True)
    present = [k for k in pk_keys if k is not None]
    it = iter(_pk_cache.ids_for(e, present))
    pk_ids = [next(it) if k is not None else eng.NO_PUBKEY for k in pk_keys]
    res = e.run(eng.OP_VERIFY_AGGREGATE, duty_first, sigs, ids, msgs=msgs, duty_msg=np.arange(len(duties)),
                pubkey_ids=pk_ids, duty_threshold=thr)
    out = []
    for d, ds in enumerate(res.duty_status.tolist()):
        lo, hi = duty_first[d], duty_first[d + 1]
        ps = res.partial_status[lo:hi].tolist()
        if ds == eng.DS_OK:
            signers = [ids[lo + j] for j, s in enumerate(ps) if s == eng.PS_VALID]
            out.append((Signature(bytes(res.agg[d])), signers))
        else:
            out.append(TblsError(_DUTY_ERRORS.get(ds, f"aggregate signatures: status {ds}")))
    return out


def aggregate_batch(duties, engine=None):
    """duties: iterable of lists of PartialSignature.  Per duty returns the
    aggregate Signature or a TblsError, like tbls.Aggregate."""
    duties = [{"partials": list(p)} for p in duties]
    if not duties:
        return []
    e = _engine(engine)
    duty_first, sigs, ids, _, _, _ = _duty_arrays(duties, False)
    res = e.run(eng.OP_AGGREGATE, duty_first, sigs, ids)
    out = []
    for d, ds in enumerate(res.duty_status.tolist()):
        if ds == eng.DS_OK:
            out.append(Signature(bytes(res.agg[d])))
        else:
            out.append(TblsError(_DUTY_ERRORS.get(ds, f"aggregate signatures: status {ds}")))
    return out


# ------------------------------------------------------------ Go-API mirror
def verify(pk, msg: bytes, sig, engine=None) -> bool:
    """tbls.Verify: (bool, error).  Decode failures raise TblsError."""
    if pk is None:
        raise TblsError("verify signature: public key cannot be nil")
    r = verify_batch([(pk, msg, sig)], engine)[0]
    if isinstance(r, Exception):
        raise r
    return r


def aggregate(partial_sigs, engine=None) -> Signature:
    """tbls.Aggregate (CombineSignatures over all partials)."""
    r = aggregate_batch([partial_sigs], engine)[0]
    if isinstance(r, Exception):
        raise r
    return r


def verify_and_aggregate(tss: TSS, partial_sigs, msg: bytes, engine=None):
    """tbls.VerifyAndAggregate: returns (Signature, signers)."""
    partial_sigs = list(partial_sigs)
    if len(partial_sigs) < tss.threshold:
        raise TblsError("insufficient signatures")
    r = verify_and_aggregate_batch([{"tss": tss, "partials": partial_sigs, "msg": msg}], engine)[0]
    if isinstance(r, Exception):
        raise r
    return r
