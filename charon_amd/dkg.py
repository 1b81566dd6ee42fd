"""DKG and cluster-lock signature work on the GPU.

  agg_deposit_data_sigs    dkg/dkg.go:545-601   verify every peer's deposit-data
                           partial against its pubshare, threshold-aggregate per DV
  verify_deposit_aggregates dkg/dkg.go:408-421  the aggregate of each DV verifies
                           under the DV's own public key
  agg_lock_hash_sig        dkg/dkg.go:428-478   verify every lock-hash partial,
                           then AggregateSignatures / AggregatePublicKeys
                           (plain sums: the multi-signature of all shares)
  verify_multi_signature   dkg/dkg.go:377       VerifyMultiSignature
  lock_verify_hashes       cluster/lock.go:117-131  the JSON lock hash == hashLock(l)
  lock_verify_signatures   cluster/lock.go:137-179  the lock's aggregate
                           signature: FastAggregateVerify over every pubshare,
                           over the hash the caller recomputed (not the JSON's)

Each step is one GPU submit over the whole ceremony (every DV and peer at
once) instead of the reference's per-partial loop: the deposit data runs as a
TBG_OP_VERIFY_AGGREGATE batch with threshold = the partial count (all must
verify, as the reference aborts on the first bad one), the lock hash as one
TBG_OP_VERIFY batch over a single message, and the sums / FastAggregateVerify
through tbg_sum_pubkeys, tbg_sum_sigs and tbg_fast_aggregate_verify.

Errors mirror the reference's strings; where the reference iterates a Go map
(random order) the first error in the caller's order is raised.  Out of scope
(host work off the signature path): the definition's operator ECDSA
signatures (Definition.VerifySignatures) and hashLock's SSZ walk -- the
caller passes the lock hash it recomputed; the JSON's lock_hash is only
compared against it.
"""
from __future__ import annotations

import base64
from dataclasses import dataclass

import numpy as np

from . import engine as eng
from . import tbls


class DKGError(Exception):
    pass


@dataclass(frozen=True)
class DKGPartial:
    """core.ParSignedData of the DKG exchange: the peer's share index (1-based)
    and its 96-byte partial signature."""
    share_idx: int
    signature: bytes


def _pk_ids(e, keys):
    present = [k for k in keys if k is not None]
    it = iter(tbls._pk_cache.ids_for(e, present))
    return [next(it) if k is not None else eng.NO_PUBKEY for k in keys]


def _decode_error(st: int) -> str:
    return "signature from core: uncompress sig: " + tbls._DECODE_ERRORS.get(st, str(st))


def _is_decode_error(st: int) -> bool:
    return st < 0 and st not in (eng.PS_ERR_PUBKEY, eng.PS_ERR_IDENTITY)


def agg_deposit_data_sigs(data, shares, msgs, engine=None) -> dict:
    """data {dv_pk48: [DKGPartial]}, shares {dv_pk48: {share_idx: pubshare48}},
    msgs {dv_pk48: deposit signing root}.  Returns {dv_pk48: 96-byte aggregate}."""
    e = tbls._engine(engine)
    dvs = list(data)
    if not dvs:
        return {}
    duty_first, sigs, ids, keys, mlist, thr = [0], [], [], [], [], []
    for dv in dvs:
        ps = list(data[dv])
        pub = shares.get(dv)
        for p in ps:
            sigs.append(bytes(p.signature))
            ids.append(p.share_idx)
            k = pub.get(p.share_idx) if pub is not None else None
            keys.append(tbls._raw(k, tbls.PublicKey) if k is not None else None)
        duty_first.append(duty_first[-1] + len(ps))
        mlist.append(bytes(msgs.get(dv, b"")))
        thr.append(len(ps))
    res = e.run(eng.OP_VERIFY_AGGREGATE, duty_first, b"".join(sigs), ids, msgs=mlist, duty_msg=np.arange(len(dvs)),
                pubkey_ids=_pk_ids(e, keys), duty_threshold=thr)
    out = {}
    for d, dv in enumerate(dvs):
        for j in range(duty_first[d], duty_first[d + 1]):
            st = int(res.partial_status[j])
            if _is_decode_error(st):
                raise DKGError(_decode_error(st))
            if dv not in shares:
                raise DKGError("invalid pubkey in deposit data partial signature from peer")
            if ids[j] not in shares[dv]:
                raise DKGError("invalid pubshare")
            if st != eng.PS_VALID:
                raise DKGError("invalid deposit data partial signature from peer")
        ds = int(res.duty_status[d])
        if ds != eng.DS_OK:
            raise DKGError(tbls._DUTY_ERRORS.get(ds, f"aggregate signatures: status {ds}"))
        out[dv] = bytes(res.agg[d])
    return out


def verify_deposit_aggregates(aggs, msgs, engine=None) -> None:
    """dkg.go:408-421: every DV's aggregate verifies under the DV key."""
    items = [(tbls.PublicKey(bytes(dv)), bytes(msgs[dv]), tbls.Signature(bytes(sig))) for dv, sig in aggs.items()]
    for r in tbls.verify_batch(items, engine):
        if isinstance(r, Exception):
            raise DKGError(str(r))
        if not r:
            raise DKGError("invalid deposit data aggregated signature")


def agg_lock_hash_sig(data, shares, lock_hash: bytes, engine=None):
    """data {dv_pk48: [DKGPartial]}, shares {dv_pk48: {share_idx: pubshare48}}.
    Returns (aggregate signature 96 B, aggregate public key 48 B)."""
    e = tbls._engine(engine)
    flat = [(dv, p) for dv, ps in data.items() for p in ps]
    if not flat:
        raise DKGError("bls aggregate Signatures: no signatures")
    keys = []
    for dv, p in flat:
        k = shares.get(dv, {}).get(p.share_idx)
        keys.append(tbls._raw(k, tbls.PublicKey) if k is not None else None)
    n = len(flat)
    pk_ids = _pk_ids(e, keys)
    sigs = b"".join(bytes(p.signature) for _, p in flat)
    res = e.run(eng.OP_VERIFY, np.arange(n + 1), sigs, np.zeros(n, np.uint8), msgs=[bytes(lock_hash)],
                duty_msg=np.zeros(n, np.int64), pubkey_ids=pk_ids)
    for j, (dv, p) in enumerate(flat):
        st = int(res.partial_status[j])
        if _is_decode_error(st):
            raise DKGError(_decode_error(st))
        if dv not in shares:
            raise DKGError("invalid pubkey in lock hash partial signature from peer")
        if p.share_idx not in shares[dv]:
            raise DKGError("invalid pubshare")
        if st != eng.PS_VALID:
            raise DKGError("invalid lock hash partial signature from peer")
    agg_sig, sst, _ = e.sum_sigs(sigs, [0, n])
    if int(sst[0]) != eng.DS_OK:
        raise DKGError("bls aggregate Signatures: " + tbls._DUTY_ERRORS.get(int(sst[0]), str(int(sst[0]))))
    agg_pk, pst = e.sum_pubkeys(pk_ids, [0, n])
    if int(pst[0]) != eng.DS_OK:
        raise DKGError("bls aggregate Public Keys: status %d" % int(pst[0]))
    return bytes(agg_sig[0]), bytes(agg_pk[0])


def verify_multi_signature(agg_pk48: bytes, msg: bytes, agg_sig96: bytes, engine=None) -> bool:
    """VerifyMultiSignature (dkg.go:377): CoreVerify of the aggregates."""
    r = tbls.verify_batch([(tbls.PublicKey(bytes(agg_pk48)), bytes(msg), tbls.Signature(bytes(agg_sig96)))], engine)[0]
    if isinstance(r, Exception):
        raise DKGError(str(r))
    return r


def _lock_bytes(v) -> bytes:
    """Lock JSON byte fields: 0x-hex (v1.2+) or base64 (v1.0 / v1.1)."""
    if v is None:
        return b""
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    if v.startswith("0x"):
        return bytes.fromhex(v[2:])
    return base64.b64decode(v)


def lock_verify_hashes(lock: dict, lock_hash: bytes) -> None:
    """The lock-hash half of Lock.VerifyHashes (cluster/lock.go:117-131): the
    JSON's lock_hash must equal the caller's recomputed hashLock(l)
    ("invalid lock hash").  The definition-hash half and the SSZ walk that
    recomputes both hashes are host work outside the BLS path."""
    lock_hash = bytes(lock_hash)
    if len(lock_hash) != 32:
        raise ValueError("lock_hash must be the 32-byte hashLock(l)")
    if _lock_bytes(lock.get("lock_hash")) != lock_hash:
        raise DKGError("invalid lock hash")


def lock_verify_signatures(lock: dict, lock_hash: bytes | None = None, engine=None) -> None:
    """Lock.VerifySignatures' aggregate check (cluster/lock.go:137-177) over a
    lock in its JSON form: cluster_definition.version, signature_aggregate,
    distributed_validators[].public_shares.

    The reference verifies the aggregate over hashLock(l), the hash it
    recomputes from the lock's fields (lock.go:166), never over the lock_hash
    the JSON carries.  hashLock's SSZ walk of the definition and validators is
    host work outside this path, so the CALLER supplies the hash it recomputed
    as `lock_hash`; without it this raises (ValueError) instead of trusting
    the file.  Like VerifySignatures this never reads the JSON's lock_hash:
    comparing it with the recomputed hash is VerifyHashes' job
    (lock_verify_hashes).  The definition's operator signatures
    (Definition.VerifySignatures, lock.go:138-140) are ECDSA work outside the
    BLS path and are not checked here."""
    version = lock.get("cluster_definition", {}).get("version", "")
    sig = _lock_bytes(lock.get("signature_aggregate"))
    if not sig:
        if version in ("v1.0.0", "v1.1.0"):
            return  # earlier versions did not populate SignatureAggregate
        raise DKGError("empty lock aggregate signature")
    if len(sig) != 96:  # (the reference's (*[96]byte) conversion would panic)
        raise DKGError("uncompress sig: invalid length")
    if lock_hash is None:
        raise ValueError("lock_verify_signatures needs the caller's recomputed hashLock(l) (cluster/lock.go:166); "
                         "the lock_hash field of the JSON is not trusted")
    lock_hash = bytes(lock_hash)
    if len(lock_hash) != 32:
        raise ValueError("lock_hash must be the 32-byte hashLock(l)")
    e = tbls._engine(engine)
    _, st, sst = e.sum_sigs(sig, [0, 1])  # tblsconv.SigFromBytes: decode only
    if _is_decode_error(int(sst[0])):
        raise DKGError("uncompress sig: " + tbls._DECODE_ERRORS.get(int(sst[0]), str(int(sst[0]))))
    raws = [_lock_bytes(s) for dv in lock.get("distributed_validators", []) for s in dv.get("public_shares", [])]
    keys = tbls.key_from_bytes_batch(raws, e)
    for k in keys:
        if isinstance(k, Exception):
            raise DKGError(str(k))
    ids = tbls._pk_cache.ids_for(e, raws)
    out = e.fast_aggregate_verify(ids, [0, len(ids)], [lock_hash], sig)
    if int(out[0]) != eng.PS_VALID:
        raise DKGError("invalid lock signature aggregate")
