"""Host mirror of the Charon call sites around the threshold-BLS path
(SURVEY.md §8 a10-a13, f1-f2), made batch-aware over the GPU engine.

  Eth2Verifier               core/parsigex/parsigex.go:152-176 (NewEth2Verifier)
    .verify_set              parsigex.go:101-107: any failure drops the set
    .verify_sets             many peer sets, one GPU submit, per-set verdicts
  verify_partial_sigs        core/validatorapi/validatorapi.go:1052-1067 plus the
                             submitters' loops (e.g. :228-287): first failure
                             aborts the batch
  MemDB                      core/parsigdb/memory.go:31-221 (store, dedup,
                             getThresholdMatching, threshold subscribers)
  Aggregator                 core/sigagg/sigagg.go:40-103
    .aggregate_batch         every DV that reached threshold in one store call,
                             aggregated in one GPU launch

Data model: a partial is ``ParSignedData`` -- the eth2 signed object reduced to
what the verify / aggregate path reads (domain name, epoch, 32-byte message
root, 96-byte signature, share index); the rest of the SSZ object is opaque
payload carried along (the reference's JSON equality in parSignedDataEqual,
memory.go:224-237, is dataclass equality here).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace

from . import signing, tbls

# core.DutyType values (core/types.go:41-57)
DUTY_UNKNOWN, DUTY_PROPOSER, DUTY_ATTESTER, DUTY_SIGNATURE, DUTY_EXIT = 0, 1, 2, 3, 4
DUTY_BUILDER_PROPOSER, DUTY_BUILDER_REGISTRATION, DUTY_RANDAO = 5, 6, 7
DUTY_PREPARE_AGGREGATOR, DUTY_AGGREGATOR, DUTY_SYNC_MESSAGE = 8, 9, 10
DUTY_PREPARE_SYNC_CONTRIBUTION, DUTY_SYNC_CONTRIBUTION, DUTY_INFO_SYNC = 11, 12, 13


class ParSigError(Exception):
    """Mirror of the errors the parsigex / parsigdb / sigagg / validatorapi
    components return."""


@dataclass(frozen=True)
class Duty:
    slot: int
    type: int


@dataclass(frozen=True)
class ParSignedData:
    """core.ParSignedData over an Eth2SignedData (core/types.go, core/eth2signeddata.go)."""
    domain: str          # Eth2SignedData.DomainName()
    epoch: int           # Eth2SignedData.Epoch()
    message_root: bytes  # Eth2SignedData.MessageRoot()
    signature: bytes     # 96-byte partial signature
    share_idx: int
    payload: bytes = b""  # the rest of the signed object (opaque here)

    def set_signature(self, sig: bytes) -> "ParSignedData":
        """SignedData.SetSignature: same object, aggregate signature."""
        return replace(self, signature=bytes(sig), share_idx=0)


# ------------------------------------------------------------------ parsigex
class Eth2Verifier:
    """parsigex.NewEth2Verifier: pubshares_by_key maps a DV's group pubkey to
    {share_idx: tbls.PublicKey}."""

    def __init__(self, spec: signing.Spec, pubshares_by_key: dict, engine=None):
        self.spec = spec
        self.pubshares_by_key = pubshares_by_key
        self.engine = engine

    def _item(self, pubkey, data: ParSignedData):
        pubshares = self.pubshares_by_key.get(pubkey)
        if pubshares is None:
            return ParSigError("unknown pubkey, not part of cluster lock")
        pubshare = pubshares.get(data.share_idx)
        if pubshare is None:
            return ParSigError("invalid shareIdx")
        if not isinstance(data, ParSignedData):
            return ParSigError("invalid eth2 signed data")
        return signing.VerifyItem(data.domain, data.epoch, data.message_root, data.signature, pubshare)

    def verify_items(self, duties_pubkeys_datas):
        """Per (duty, pubkey, data): None or the error verifyFunc returns."""
        triples = list(duties_pubkeys_datas)
        out = [None] * len(triples)
        idx, items = [], []
        for i, (duty, pubkey, data) in enumerate(triples):
            it = self._item(pubkey, data)
            if isinstance(it, Exception):
                out[i] = it
            else:
                idx.append(i)
                items.append(it)
        if items:
            for i, r in zip(idx, signing.verify_batch(self.spec, items, self.engine)):
                if r is not None:
                    out[i] = ParSigError(f"invalid signature: {r} (duty={triples[i][0]})")
        return out

    def __call__(self, duty: Duty, pubkey, data: ParSignedData):
        """The per-item verifyFunc: raises on failure."""
        r = self.verify_items([(duty, pubkey, data)])[0]
        if r is not None:
            raise r

    def verify_sets(self, sets):
        """sets: [(duty, {pubkey: ParSignedData})].  One GPU submit for every
        partial of every set; per set returns None or the first failing
        item's error -- the whole set is dropped (parsigex.go:101-107)."""
        sets = list(sets)
        flat, owner = [], []
        for k, (duty, pset) in enumerate(sets):
            for pubkey, data in pset.items():
                flat.append((duty, pubkey, data))
                owner.append(k)
        res = self.verify_items(flat)
        out = [None] * len(sets)
        for k, r in zip(owner, res):
            if r is not None and out[k] is None:
                out[k] = r
        return out

    def verify_set(self, duty: Duty, pset: dict) -> None:
        r = self.verify_sets([(duty, pset)])[0]
        if r is not None:
            raise r


class ParSigEx:
    """The receive side of parsigex.Handle (parsigex.go:80-114), batch-aware:
    ``handle_batch`` verifies many received peer sets with one GPU submit and
    forwards only the sets that verify completely to the subscribers."""

    def __init__(self, verifier: Eth2Verifier):
        self.verifier = verifier
        self.subs = []

    def subscribe(self, fn):
        self.subs.append(fn)

    def handle_batch(self, sets):
        """Returns per set None (forwarded) or the error that dropped it."""
        sets = list(sets)
        verdicts = self.verifier.verify_sets(sets)
        for (duty, pset), err in zip(sets, verdicts):
            if err is None:
                for sub in self.subs:
                    sub(duty, dict(pset))
        return verdicts

    def handle(self, duty: Duty, pset: dict):
        return self.handle_batch([(duty, pset)])[0]


# --------------------------------------------------------------- validatorapi
def verify_partial_sigs(spec: signing.Spec, get_pubshare, parsigs, engine=None, insecure_test=False):
    """validatorapi.verifyPartialSig over a submitter's batch (e.g.
    SubmitAttestations, validatorapi.go:228-287): parsigs is a list of
    (group pubkey, ParSignedData); get_pubshare(pubkey) returns this node's
    public share or raises.  Returns None, or the first failure in input
    order (the submitter aborts before any subscriber runs)."""
    if insecure_test:
        return None
    items, errs = [], []
    for pubkey, data in parsigs:
        try:
            pubshare = get_pubshare(pubkey)
        except Exception as e:  # mirrors getVerifyShareFunc's error
            errs.append(e)
            items.append(None)
            continue
        if not isinstance(data, ParSignedData):
            errs.append(ParSigError("invalid eth2 signed data"))
            items.append(None)
            continue
        errs.append(None)
        items.append(signing.VerifyItem(data.domain, data.epoch, data.message_root, data.signature, pubshare))
    live = [i for i, it in enumerate(items) if it is not None]
    if live:
        for i, r in zip(live, signing.verify_batch(spec, [items[i] for i in live], engine)):
            errs[i] = r
    for e in errs:
        if e is not None:
            return e
    return None


# ------------------------------------------------------------------- parsigdb
def get_threshold_matching(duty_type: int, sigs, threshold: int):
    """memory.go:194-221: ``threshold`` partials with identical message root,
    or None.  Fires at exactly t, so later partials do not re-trigger."""
    if len(sigs) < threshold:
        return None
    if duty_type == DUTY_SIGNATURE:
        return list(sigs) if len(sigs) == threshold else None
    by_root = {}
    for s in sigs:
        by_root.setdefault(bytes(s.message_root), []).append(s)
    for group in by_root.values():
        if len(group) == threshold:
            return group
    return None


class MemDB:
    """parsigdb.MemDB (memory.go:31-190).  Threshold subscribers are called
    per DV as in the reference; batch subscribers are called once per store
    call with every (duty, pubkey, partials) that reached threshold, which is
    how the batch aggregator gets a whole peer set in one GPU launch."""

    def __init__(self, threshold: int):
        self.threshold = threshold
        self.entries = {}
        self.keys_by_duty = {}
        self.internal_subs = []
        self.thresh_subs = []
        self.thresh_batch_subs = []

    def subscribe_internal(self, fn):
        self.internal_subs.append(fn)

    def subscribe_threshold(self, fn):
        self.thresh_subs.append(fn)

    def subscribe_threshold_batch(self, fn):
        self.thresh_batch_subs.append(fn)

    def _store(self, key, value: ParSignedData):
        lst = self.entries.get(key, [])
        for s in lst:
            if s.share_idx == value.share_idx:
                if s != value:
                    raise ParSigError(f"mismatching partial signed data (share_idx={s.share_idx})")
                return None
        lst = lst + [value]
        self.entries[key] = lst
        self.keys_by_duty.setdefault(key[0], []).append(key)
        return list(lst)

    def store_external(self, duty: Duty, signed_set: dict):
        reached = []
        for pubkey, sig in signed_set.items():
            sigs = self._store((duty, pubkey), sig)
            if sigs is None:
                continue  # duplicate, ignored
            psigs = get_threshold_matching(duty.type, sigs, self.threshold)
            if psigs is None:
                continue
            reached.append((duty, pubkey, psigs))
            for sub in self.thresh_subs:
                sub(duty, pubkey, list(psigs))
        if reached:
            for sub in self.thresh_batch_subs:
                sub(list(reached))
        return reached

    def store_internal(self, duty: Duty, signed_set: dict):
        reached = self.store_external(duty, signed_set)
        for sub in self.internal_subs:
            sub(duty, dict(signed_set))
        return reached

    def trim(self, duty: Duty):
        """Deadliner expiry (memory.go:140-157)."""
        for key in self.keys_by_duty.pop(duty, []):
            self.entries.pop(key, None)


# --------------------------------------------------------------------- sigagg
class Aggregator:
    """sigagg.Aggregator: threshold partials -> aggregate signed data."""

    def __init__(self, threshold: int, engine=None):
        self.threshold = threshold
        self.engine = engine
        self.subs = []

    def subscribe(self, fn):
        self.subs.append(fn)

    def _check(self, parsigs):
        if len(parsigs) < self.threshold:
            return ParSigError("require threshold signatures")
        if self.threshold == 0:
            return ParSigError("invalid threshold config")
        return None

    def aggregate_batch(self, items):
        """items: [(duty, pubkey, [ParSignedData])].  One GPU launch decodes
        every partial, recombines each DV with Lagrange coefficients and
        encodes the aggregates.  Returns per item the aggregate
        ParSignedData (share_idx 0) or a ParSigError; subscribers are called
        for the successes."""
        items = list(items)
        out = [None] * len(items)
        live, duties = [], []
        for k, (duty, pubkey, parsigs) in enumerate(items):
            err = self._check(parsigs)
            if err is not None:
                out[k] = err
                continue
            live.append(k)
            duties.append([tbls.PartialSignature(p.share_idx, tbls.Signature(bytes(p.signature))) for p in parsigs])
        if duties:
            for k, r in zip(live, tbls.aggregate_batch(duties, self.engine)):
                if isinstance(r, Exception):
                    msg = str(r)
                    out[k] = ParSigError("convert signature: " + msg if msg.startswith("uncompress") else msg)
                else:
                    out[k] = items[k][2][0].set_signature(r.raw)
        for (duty, pubkey, _), r in zip(items, out):
            if not isinstance(r, Exception):
                for sub in self.subs:
                    sub(duty, pubkey, r)
        return out

    def aggregate(self, duty: Duty, pubkey, parsigs):
        r = self.aggregate_batch([(duty, pubkey, parsigs)])[0]
        if isinstance(r, Exception):
            raise r
        return r
