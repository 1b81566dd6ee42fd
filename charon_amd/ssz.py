"""Batched message roots and signing roots of the duty objects (host code of
libtbls_gpu.so, include/tbls_ssz.h) -- the step in front of every verify of
the hot path:

  MessageRoot   core/signeddata.go:455 (Attestation), :516 (VoluntaryExit),
                :598 (ValidatorRegistration), :713 (Randao), :774 (selection),
                :837 (sync selection), :962 (sync message)
  GetDomain     eth2util/signing/signing.go:52-70
  GetDataRoot   eth2util/signing/signing.go:73-85

Objects are typed here and handed to the native code in their SSZ
serialization, one contiguous buffer per batch; the hashing (SHA-256 with the
x86 SHA extensions where present, split over host threads) runs in
charon_amd/csrc/ssz_roots.cpp.
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass

import numpy as np

from . import _native

# enum tbg_ssz_kind (include/tbls_ssz.h)
ROOT, UINT64, ATTESTATION_DATA, VOLUNTARY_EXIT, SYNC_AGG_SELECTION, VALIDATOR_REGISTRATION, \
    DEPOSIT_MESSAGE, DEPOSIT_DATA, FORK_DATA, SIGNING_DATA, CHECKPOINT = range(11)


class SSZError(Exception):
    pass


def _u64(v: int) -> bytes:
    return struct.pack("<Q", int(v))


def _fixed(b, n: int, what: str) -> bytes:
    b = bytes(b)
    if len(b) != n:
        raise SSZError(f"{what}: want {n} bytes, got {len(b)}")
    return b


@dataclass(frozen=True)
class Checkpoint:
    epoch: int
    root: bytes = bytes(32)
    KIND = CHECKPOINT

    def ssz(self) -> bytes:
        return _u64(self.epoch) + _fixed(self.root, 32, "checkpoint root")


@dataclass(frozen=True)
class AttestationData:
    """phase0 AttestationData (Attestation.MessageRoot, signeddata.go:455-457)."""
    slot: int
    index: int
    beacon_block_root: bytes
    source: Checkpoint
    target: Checkpoint
    KIND = ATTESTATION_DATA

    def ssz(self) -> bytes:
        return _u64(self.slot) + _u64(self.index) + _fixed(self.beacon_block_root, 32, "beacon_block_root") + \
            self.source.ssz() + self.target.ssz()


@dataclass(frozen=True)
class VoluntaryExit:
    epoch: int
    validator_index: int
    KIND = VOLUNTARY_EXIT

    def ssz(self) -> bytes:
        return _u64(self.epoch) + _u64(self.validator_index)


@dataclass(frozen=True)
class SyncAggregatorSelectionData:
    slot: int
    subcommittee_index: int
    KIND = SYNC_AGG_SELECTION

    def ssz(self) -> bytes:
        return _u64(self.slot) + _u64(self.subcommittee_index)


@dataclass(frozen=True)
class ValidatorRegistration:
    fee_recipient: bytes
    gas_limit: int
    timestamp: int
    pubkey: bytes
    KIND = VALIDATOR_REGISTRATION

    def ssz(self) -> bytes:
        return _fixed(self.fee_recipient, 20, "fee_recipient") + _u64(self.gas_limit) + _u64(self.timestamp) + \
            _fixed(self.pubkey, 48, "pubkey")


@dataclass(frozen=True)
class DepositMessage:
    pubkey: bytes
    withdrawal_credentials: bytes
    amount: int
    KIND = DEPOSIT_MESSAGE

    def ssz(self) -> bytes:
        return _fixed(self.pubkey, 48, "pubkey") + _fixed(self.withdrawal_credentials, 32, "withdrawal_credentials") + \
            _u64(self.amount)


@dataclass(frozen=True)
class DepositData:
    pubkey: bytes
    withdrawal_credentials: bytes
    amount: int
    signature: bytes
    KIND = DEPOSIT_DATA

    def ssz(self) -> bytes:
        return DepositMessage(self.pubkey, self.withdrawal_credentials, self.amount).ssz() + \
            _fixed(self.signature, 96, "signature")


@dataclass(frozen=True)
class Epoch:
    """SignedRandao's root: SignedEpoch hashes only its epoch (eth2util/types.go:44-52)."""
    epoch: int
    KIND = UINT64

    def ssz(self) -> bytes:
        return _u64(self.epoch)


@dataclass(frozen=True)
class Slot:
    """BeaconCommitteeSelection's root: SlotHashRoot (eth2util/hash.go:26-41)."""
    slot: int
    KIND = UINT64

    def ssz(self) -> bytes:
        return _u64(self.slot)


@dataclass(frozen=True)
class Root:
    """SignedSyncMessage's root: the beacon block root itself (signeddata.go:962-964)."""
    root: bytes
    KIND = ROOT

    def ssz(self) -> bytes:
        return _fixed(self.root, 32, "root")


def size(kind: int) -> int:
    return int(_native.load().tbg_ssz_size(kind))


def _pack(kind, objs):
    """(kind, contiguous SSZ bytes, n) of a batch: typed objects of one kind,
    or already-serialized bytes with an explicit kind."""
    objs = list(objs)
    if kind is None:
        if not objs:
            raise SSZError("empty batch needs an explicit kind")
        kind = type(objs[0]).KIND
    sz = size(kind)
    if not sz:
        raise SSZError(f"unknown kind {kind}")
    parts = [o if isinstance(o, (bytes, bytearray)) else o.ssz() for o in objs]
    if any(len(p) != sz for p in parts):
        raise SSZError(f"kind {kind}: every object serializes to {sz} bytes")
    return kind, b"".join(parts), len(parts)


def _check(rc, what):
    if rc != 0:
        raise SSZError(f"{what}: rc={rc}")


def hash_tree_roots(objs, kind=None, threads: int = 0) -> list:
    """hash_tree_root of every object (the duty types' MessageRoot)."""
    kind, buf, n = _pack(kind, objs)
    out = ctypes.create_string_buffer(32 * max(n, 1))
    _check(_native.load().tbg_ssz_roots(kind, buf, n, out, threads), "tbg_ssz_roots")
    raw = out.raw
    return [raw[32 * i:32 * i + 32] for i in range(n)]


def compute_domain(domain_type: bytes, version: bytes, genesis_validators_root: bytes = bytes(32)) -> bytes:
    out = ctypes.create_string_buffer(32)
    _check(_native.load().tbg_compute_domain(_fixed(domain_type, 4, "domain type"), _fixed(version, 4, "version"),
                                             _fixed(genesis_validators_root, 32, "genesis_validators_root"), out),
           "tbg_compute_domain")
    return out.raw


def signing_roots(objs, domains, domain_idx=None, kind=None, threads: int = 0) -> list:
    """GetDataRoot(MessageRoot(obj)) for every object: domains is a list of
    32-byte domains, domain_idx (optional) the domain of each object."""
    kind, buf, n = _pack(kind, objs)
    domains = [_fixed(d, 32, "domain") for d in domains]
    if not domains:
        raise SSZError("no domain")
    idx = None
    if domain_idx is not None:
        idx = np.ascontiguousarray(np.asarray(domain_idx, dtype=np.uint32))
        if idx.shape != (n,):
            raise SSZError("one domain index per object")
    out = ctypes.create_string_buffer(32 * max(n, 1))
    rc = _native.load().tbg_signing_roots(kind, buf, n, b"".join(domains), len(domains),
                                          None if idx is None else idx.ctypes.data, out, threads)
    _check(rc, "tbg_signing_roots")
    raw = out.raw
    return [raw[32 * i:32 * i + 32] for i in range(n)]
