/*
 * tbls_ssz.h -- batched signing roots on the host (libtbls_gpu.so, host code).
 *
 * The step in front of every tbls.Verify of the hot path: the duty object's
 * SSZ hash_tree_root (reference core/signeddata.go MessageRoot methods) and
 * the signing root over its domain (eth2util/signing/signing.go:52-85,
 * GetDomain / GetDataRoot).  One call hashes a whole batch of duties, split
 * over host threads; SHA-256 uses the x86 SHA extensions when the CPU has
 * them (TBG_SHA_PORTABLE=1 in the environment forces the portable code).
 *
 * Objects are passed in their SSZ serialization (all kinds here are
 * fixed-size containers: the serialization is the fields back to back,
 * integers little-endian), n objects of tbg_ssz_size(kind) bytes each.
 */
#ifndef TBLS_SSZ_H
#define TBLS_SSZ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum tbg_ssz_kind {
  /* 32 B: the object root itself -- SignedSyncMessage.MessageRoot returns
   * BeaconBlockRoot (core/signeddata.go:962-964) */
  TBG_SSZ_ROOT = 0,
  /* 8 B uint64: SignedRandao / SignedEpoch (core/signeddata.go:713-715,
   * eth2util/types.go:44-52), BeaconCommitteeSelection via SlotHashRoot
   * (core/signeddata.go:774-776, eth2util/hash.go:26-41) */
  TBG_SSZ_UINT64 = 1,
  /* 128 B AttestationData{slot, index, beacon_block_root, source{epoch, root},
   * target{epoch, root}}: Attestation.MessageRoot (core/signeddata.go:455-457) */
  TBG_SSZ_ATTESTATION_DATA = 2,
  /* 16 B VoluntaryExit{epoch, validator_index} (core/signeddata.go:516-518) */
  TBG_SSZ_VOLUNTARY_EXIT = 3,
  /* 16 B SyncAggregatorSelectionData{slot, subcommittee_index} (core/signeddata.go:837-844) */
  TBG_SSZ_SYNC_AGG_SELECTION = 4,
  /* 84 B ValidatorRegistration{fee_recipient[20], gas_limit, timestamp, pubkey[48]}
   * (core/signeddata.go:598-600) */
  TBG_SSZ_VALIDATOR_REGISTRATION = 5,
  /* 88 B DepositMessage{pubkey[48], withdrawal_credentials[32], amount}
   * (eth2util/deposit/deposit.go:50-66) */
  TBG_SSZ_DEPOSIT_MESSAGE = 6,
  /* 184 B DepositData{pubkey[48], withdrawal_credentials[32], amount, signature[96]}
   * (eth2util/deposit/deposit.go:117) */
  TBG_SSZ_DEPOSIT_DATA = 7,
  /* 36 B ForkData{current_version[4], genesis_validators_root[32]} */
  TBG_SSZ_FORK_DATA = 8,
  /* 64 B SigningData{object_root, domain} (eth2util/signing/signing.go:80) */
  TBG_SSZ_SIGNING_DATA = 9,
  /* 40 B Checkpoint{epoch, root} */
  TBG_SSZ_CHECKPOINT = 10,
  TBG_SSZ_KINDS = 11
};

/* Serialized size of one object of `kind`, 0 for an unknown kind. */
uint32_t tbg_ssz_size(uint32_t kind);

/* roots32[i] = hash_tree_root(object i).  n_threads = 0: the library picks
 * (at most 16).  TBG_OK or TBG_E_INVALID_ARG (-1). */
int tbg_ssz_roots(uint32_t kind, const uint8_t* ssz, uint32_t n, uint8_t* roots32, uint32_t n_threads);

/* compute_domain: domain_type[4] || hash_tree_root(ForkData{version, gvr})[:28]
 * (eth2util/signing/signing.go:52-70 through eth2Cl.Domain). */
int tbg_compute_domain(const uint8_t* type4, const uint8_t* version4, const uint8_t* gvr32, uint8_t* domain32);

/* MessageRoot + GetDataRoot fused: out32[i] = hash_tree_root(SigningData{
 * hash_tree_root(object i), domains32[domain_idx[i]]}) -- the 32-byte message
 * tbls.Verify signs over (signing.go:73-85).  domain_idx NULL: every object
 * uses domains32[0]; indices must be < n_domains. */
int tbg_signing_roots(uint32_t kind, const uint8_t* ssz, uint32_t n, const uint8_t* domains32, uint32_t n_domains,
                      const uint32_t* domain_idx, uint8_t* out32, uint32_t n_threads);

#ifdef __cplusplus
}
#endif

#endif /* TBLS_SSZ_H */
