"""Host mirror of Charon's ``eth2util/signing`` verify path.

  get_domain(spec, name, epoch)              signing.go:52-70 (eth2Cl.Domain)
  get_data_root(spec, name, epoch, root)     signing.go:73-85
  verify(spec, name, epoch, root, sig, pk)   signing.go:120-151
  verify_batch(spec, items)                  the batched form the batch-aware
                                             call sites use: one GPU submit
  get_data_roots / message_signing_roots     the signing roots of a batch in
                                             one native call (include/tbls_ssz.h)

The signing root is SSZ ``hash_tree_root(SigningData{object_root, domain})``,
i.e. SHA-256 over the two 32-byte leaves, and the domain is
``domain_type || hash_tree_root(ForkData{version, genesis_validators_root})[:28]``
(consensus-specs ``compute_domain``).  Both are host work (a few SHA-256
compressions per item, batched in charon_amd/csrc/ssz_roots.cpp); everything after
-- G2 decode, hash_to_G2, the pairing check -- runs on the GPU through
``charon_amd.tbls``.

Error strings follow the reference: ``"no signature found"`` (signing.go:133),
``"convert signature: uncompress sig: ..."`` (signing.go:137-140, 157),
``"invalid signature"`` (signing.go:147), ``"domain type not found"``
(signing.go:59).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field

from . import tbls

# DomainName constants (signing.go:38-48) -> consensus-specs domain types.
DOMAIN_BEACON_PROPOSER = "DOMAIN_BEACON_PROPOSER"
DOMAIN_BEACON_ATTESTER = "DOMAIN_BEACON_ATTESTER"
DOMAIN_RANDAO = "DOMAIN_RANDAO"
DOMAIN_EXIT = "DOMAIN_VOLUNTARY_EXIT"
DOMAIN_APPLICATION_BUILDER = "DOMAIN_APPLICATION_BUILDER"
DOMAIN_SELECTION_PROOF = "DOMAIN_SELECTION_PROOF"
DOMAIN_AGGREGATE_AND_PROOF = "DOMAIN_AGGREGATE_AND_PROOF"
DOMAIN_SYNC_COMMITTEE = "DOMAIN_SYNC_COMMITTEE"
DOMAIN_SYNC_COMMITTEE_SELECTION_PROOF = "DOMAIN_SYNC_COMMITTEE_SELECTION_PROOF"
DOMAIN_CONTRIBUTION_AND_PROOF = "DOMAIN_CONTRIBUTION_AND_PROOF"
DOMAIN_DEPOSIT = "DOMAIN_DEPOSIT"

DOMAIN_TYPES = {
    DOMAIN_BEACON_PROPOSER: bytes.fromhex("00000000"),
    DOMAIN_BEACON_ATTESTER: bytes.fromhex("01000000"),
    DOMAIN_RANDAO: bytes.fromhex("02000000"),
    DOMAIN_DEPOSIT: bytes.fromhex("03000000"),
    DOMAIN_EXIT: bytes.fromhex("04000000"),
    DOMAIN_SELECTION_PROOF: bytes.fromhex("05000000"),
    DOMAIN_AGGREGATE_AND_PROOF: bytes.fromhex("06000000"),
    DOMAIN_SYNC_COMMITTEE: bytes.fromhex("07000000"),
    DOMAIN_SYNC_COMMITTEE_SELECTION_PROOF: bytes.fromhex("08000000"),
    DOMAIN_CONTRIBUTION_AND_PROOF: bytes.fromhex("09000000"),
    DOMAIN_APPLICATION_BUILDER: bytes.fromhex("00000001"),
}
# Domains computed over the genesis fork version and a zero validators root,
# independent of the epoch (consensus-specs deposit / builder-specs
# registration; reference eth2util/deposit/deposit.go:148, signing_test.go:34-80).
_GENESIS_DOMAINS = (DOMAIN_DEPOSIT, DOMAIN_APPLICATION_BUILDER)


class SigningError(Exception):
    """Mirror of the errors signing.Verify returns."""


def _sha(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def fork_data_root(version: bytes, genesis_validators_root: bytes) -> bytes:
    """hash_tree_root(ForkData{current_version (Bytes4), genesis_validators_root})."""
    assert len(version) == 4 and len(genesis_validators_root) == 32
    return _sha(version + bytes(28) + genesis_validators_root)


def compute_domain(domain_type: bytes, version: bytes, genesis_validators_root: bytes = bytes(32)) -> bytes:
    return bytes(domain_type) + fork_data_root(version, genesis_validators_root)[:28]


def signing_root(object_root: bytes, domain: bytes) -> bytes:
    """hash_tree_root(SigningData{object_root, domain}) (signing.go:80)."""
    if len(object_root) != 32 or len(domain) != 32:
        raise SigningError("marshal signing data")
    return _sha(bytes(object_root) + bytes(domain))


@dataclass
class Spec:
    """The slice of the beacon spec the verify path reads from eth2Cl
    (eth2Cl.Spec / eth2Cl.Domain): the fork schedule and the genesis
    validators root.  forks: [(activation_epoch, 4-byte version)], ascending;
    the first is the genesis fork."""
    forks: list = field(default_factory=lambda: [(0, bytes.fromhex("00001020"))])
    genesis_validators_root: bytes = bytes(32)
    domain_types: dict = field(default_factory=lambda: dict(DOMAIN_TYPES))

    def fork_version(self, epoch: int) -> bytes:
        version = self.forks[0][1]
        for start, v in self.forks:
            if epoch >= start:
                version = v
        return version

    def domain(self, name: str, epoch: int) -> bytes:
        dt = self.domain_types.get(name)
        if dt is None:
            raise SigningError("domain type not found")
        if name in _GENESIS_DOMAINS:
            return compute_domain(dt, self.forks[0][1], bytes(32))
        return compute_domain(dt, self.fork_version(epoch), self.genesis_validators_root)


def get_domain(spec: Spec, name: str, epoch: int) -> bytes:
    return spec.domain(name, epoch)


def get_data_root(spec: Spec, name: str, epoch: int, root: bytes) -> bytes:
    return signing_root(root, spec.domain(name, epoch))


def _domain_table(spec: Spec, names, epochs):
    """Distinct domains of (name, epoch) pairs and each pair's index."""
    table, domains, idx = {}, [], []
    for name, e in zip(names, epochs):
        d = spec.domain(name, e)
        if d not in table:
            table[d] = len(domains)
            domains.append(d)
        idx.append(table[d])
    return domains, idx


def get_data_roots(spec: Spec, name, epochs, object_roots) -> list:
    """GetDataRoot over a batch (one native call, include/tbls_ssz.h).  `name`
    is one domain name or one per item."""
    from . import ssz
    epochs = list(epochs)
    names = [name] * len(epochs) if isinstance(name, str) else list(name)
    roots = list(object_roots)
    if not roots:
        return []
    if any(len(r) != 32 for r in roots):
        raise SigningError("marshal signing data")
    domains, idx = _domain_table(spec, names, epochs)
    return ssz.signing_roots([bytes(r) for r in roots], domains, idx, kind=ssz.ROOT)


def message_signing_roots(spec: Spec, name, epochs, objects) -> list:
    """MessageRoot + GetDataRoot fused for typed duty objects of one kind
    (charon_amd.ssz): the 32-byte messages their signatures cover."""
    from . import ssz
    objects, epochs = list(objects), list(epochs)
    if not objects:
        return []
    names = [name] * len(epochs) if isinstance(name, str) else list(name)
    domains, idx = _domain_table(spec, names, epochs)
    return ssz.signing_roots(objects, domains, idx)


@dataclass(frozen=True)
class VerifyItem:
    """Arguments of one signing.Verify call."""
    domain: str
    epoch: int
    object_root: bytes  # 32-byte message root (Eth2SignedData.MessageRoot)
    signature: bytes    # 96-byte eth2 BLS signature
    pubkey: object      # tbls.PublicKey (or 48 bytes); None = unknown share


_ZERO_SIG = bytes(96)


def verify_batch(spec: Spec, items, engine=None):
    """signing.Verify over many items with one GPU submit.  Returns, per item,
    None (valid) or the SigningError the reference would return."""
    items = list(items)
    out = [None] * len(items)
    todo, gpu_items = [], []
    # signing roots of every well-formed item in one native batch
    ok = []
    for i, it in enumerate(items):
        try:
            spec.domain(it.domain, it.epoch)
            if len(it.object_root) != 32:
                raise SigningError("marshal signing data")
            ok.append(i)
        except SigningError as e:
            out[i] = e
    msgs = dict(zip(ok, get_data_roots(spec, [items[i].domain for i in ok], [items[i].epoch for i in ok],
                                       [items[i].object_root for i in ok])))
    for i, it in enumerate(items):
        if out[i] is not None:
            continue
        msg = msgs[i]
        sig = bytes(it.signature)
        if sig == _ZERO_SIG:
            out[i] = SigningError("no signature found")
            continue
        if len(sig) != 96:
            out[i] = SigningError("convert signature: uncompress sig: invalid length")
            continue
        pk = it.pubkey
        if pk is not None and not isinstance(pk, tbls.PublicKey):
            pk = tbls.PublicKey(bytes(pk))
        todo.append(i)
        gpu_items.append((pk, msg, tbls.Signature(sig)))
    if gpu_items:
        res = tbls.verify_batch(gpu_items, engine)
        for i, r in zip(todo, res):
            if isinstance(r, Exception):
                out[i] = SigningError("convert signature: " + str(r))
            elif not r:
                out[i] = SigningError("invalid signature")
    return out


def verify(spec: Spec, domain: str, epoch: int, object_root: bytes, signature: bytes, pubkey, engine=None) -> None:
    """signing.Verify: raises SigningError unless the signature is valid."""
    r = verify_batch(spec, [VerifyItem(domain, epoch, object_root, signature, pubkey)], engine)[0]
    if r is not None:
        raise r
