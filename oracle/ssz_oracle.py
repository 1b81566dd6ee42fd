"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the SSZ hash_tree_root and
signing-root computation in front of the hot path, the checker for
include/tbls_ssz.h (charon_amd/csrc/ssz_roots.cpp).  Only tests/ may import it.

Follows consensus-specs ssz/simple-serialize.md (merkleization), as used by
the reference through go-eth2-client / fastssz (third-party, not vendored in
/root/reference; the generated HashTreeRootWith methods implement exactly
this algorithm):

  core/signeddata.go:455-457     Attestation.MessageRoot      = HTR(AttestationData)
  core/signeddata.go:516-518     SignedVoluntaryExit           = HTR(VoluntaryExit)
  core/signeddata.go:598-600     VersionedSignedValidatorRegistration = HTR(ValidatorRegistration)
  core/signeddata.go:713-715     SignedRandao                  = HTR(SignedEpoch) = HTR(uint64 epoch)
  core/signeddata.go:774-776     BeaconCommitteeSelection      = SlotHashRoot(slot)
  core/signeddata.go:837-844     SyncCommitteeSelection        = HTR(SyncAggregatorSelectionData)
  core/signeddata.go:962-964     SignedSyncMessage             = BeaconBlockRoot
  eth2util/types.go:44-52        SignedEpoch.HashTreeRootWith  (epoch only)
  eth2util/hash.go:26-41         SlotHashRoot
  eth2util/deposit/deposit.go:50-66, :117, :148-160, :166-190  deposit message / data / domain
  eth2util/signing/signing.go:52-85  GetDomain / GetDataRoot (SigningData)

Parity is pinned by the reference's own vectors (tests/golden/ssz_vectors.json,
tests/golden/make_ssz_golden.py): hash_test.go:27-34, types_test.go:27-36,
validatorapi_test.go:230-276, the deposit golden file, signing_test.go:34-80.
"""
from __future__ import annotations

import hashlib
import struct


def sha256(b: bytes) -> bytes:
    return hashlib.sha256(b).digest()


def merkleize(chunks):
    """Root of the chunks padded with zero chunks to the next power of two."""
    chunks = [bytes(c) for c in chunks]
    assert chunks and all(len(c) == 32 for c in chunks)
    n = 1
    while n < len(chunks):
        n *= 2
    layer = chunks + [bytes(32)] * (n - len(chunks))
    while len(layer) > 1:
        layer = [sha256(layer[i] + layer[i + 1]) for i in range(0, len(layer), 2)]
    return layer[0]


def u64(v: int) -> bytes:
    """A uint64 as its own chunk (little-endian, zero padded)."""
    return struct.pack("<Q", v) + bytes(24)


def bytes_root(b: bytes) -> bytes:
    """hash_tree_root of a fixed byte vector: its 32-byte chunks merkleized."""
    b = bytes(b)
    if len(b) <= 32:
        return b + bytes(32 - len(b))
    padded = b + bytes(-len(b) % 32)
    return merkleize([padded[i:i + 32] for i in range(0, len(padded), 32)])


def checkpoint_root(epoch: int, root: bytes) -> bytes:
    return merkleize([u64(epoch), bytes_root(root)])


def attestation_data_root(slot, index, beacon_block_root, source_epoch, source_root, target_epoch, target_root):
    return merkleize([u64(slot), u64(index), bytes_root(beacon_block_root),
                      checkpoint_root(source_epoch, source_root), checkpoint_root(target_epoch, target_root)])


def voluntary_exit_root(epoch, validator_index):
    return merkleize([u64(epoch), u64(validator_index)])


def sync_agg_selection_root(slot, subcommittee_index):
    return merkleize([u64(slot), u64(subcommittee_index)])


def validator_registration_root(fee_recipient: bytes, gas_limit: int, timestamp: int, pubkey: bytes):
    assert len(fee_recipient) == 20 and len(pubkey) == 48
    return merkleize([bytes_root(fee_recipient), u64(gas_limit), u64(timestamp), bytes_root(pubkey)])


def deposit_message_root(pubkey: bytes, withdrawal_credentials: bytes, amount: int):
    return merkleize([bytes_root(pubkey), bytes_root(withdrawal_credentials), u64(amount)])


def deposit_data_root(pubkey: bytes, withdrawal_credentials: bytes, amount: int, signature: bytes):
    return merkleize([bytes_root(pubkey), bytes_root(withdrawal_credentials), u64(amount), bytes_root(signature)])


def fork_data_root(version: bytes, genesis_validators_root: bytes):
    return merkleize([bytes_root(version), bytes_root(genesis_validators_root)])


def compute_domain(domain_type: bytes, version: bytes, genesis_validators_root: bytes = bytes(32)):
    return bytes(domain_type) + fork_data_root(version, genesis_validators_root)[:28]


def signing_root(object_root: bytes, domain: bytes):
    return merkleize([bytes(object_root), bytes(domain)])


# SSZ serializations of the fixed-size containers (fields back to back,
# integers little-endian): the input format of include/tbls_ssz.h.
def ser_u64(v):
    return struct.pack("<Q", v)


def root_of_serialized(kind: str, b: bytes) -> bytes:
    """hash_tree_root from the serialized bytes, field by field."""
    q = lambda o: struct.unpack_from("<Q", b, o)[0]
    if kind == "root":
        return bytes(b[:32])
    if kind == "uint64":
        return u64(q(0))
    if kind == "attestation_data":
        return attestation_data_root(q(0), q(8), b[16:48], q(48), b[56:88], q(88), b[96:128])
    if kind == "voluntary_exit":
        return voluntary_exit_root(q(0), q(8))
    if kind == "sync_agg_selection":
        return sync_agg_selection_root(q(0), q(8))
    if kind == "validator_registration":
        return validator_registration_root(b[:20], q(20), q(28), b[36:84])
    if kind == "deposit_message":
        return deposit_message_root(b[:48], b[48:80], q(80))
    if kind == "deposit_data":
        return deposit_data_root(b[:48], b[48:80], q(80), b[88:184])
    if kind == "fork_data":
        return fork_data_root(b[:4], b[4:36])
    if kind == "signing_data":
        return signing_root(b[:32], b[32:64])
    if kind == "checkpoint":
        return checkpoint_root(q(0), b[8:40])
    raise ValueError(kind)
