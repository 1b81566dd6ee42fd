// HIP kernels of the threshold-BLS engine (one thread per item).
//
//   k_decode_pubkeys  48-byte G1 -> affine table          (tblsconv.KeyFromBytes, tblsconv.go:30-37)
//   k_decode_sigs     96-byte G2 -> affine + status       (tblsconv.SigFromCore, tblsconv.go:125-132)
//   k_hash_msgs       message -> H(m) affine              (hash_to_G2 inside SigEth2.Verify)
//   k_verify          e(pk, H(m)) e(-g1, sig) == 1         (tbls.Verify, tss.go:190-197)
//   k_lagrange        lambda_i(0) per participating partial (CombineSignatures)
//   k_aggregate       sum lambda_i sigma_i, compress      (tbls.Aggregate / VerifyAndAggregate)
#pragma once
#include <hip/hip_runtime.h>
#include "bls_pairing.h"
#include "bls_h2c.h"
#include "bls_tss.h"
#include "../../include/tbls_gpu.h"

namespace tbg {

// Device-side layout of one batch (all pointers into device memory).
struct DevBatch {
  uint32_t op, n_duties, n_partials, n_msgs;
  const uint8_t* msgs;
  const uint32_t* msg_off;
  const uint32_t* duty_msg;
  const uint32_t* duty_first;
  const uint32_t* duty_threshold;
  const uint32_t* partial_duty;
  const uint8_t* sigs;
  const uint8_t* identifiers;
  const uint32_t* pubkey_ids;
  // work buffers
  G2A* sig_aff;
  G2A* h_aff;
  int32_t* h_status;
  uint32_t* lam;       // [n_partials][8] scalar words
  // outputs
  int32_t* partial_status;
  int32_t* duty_status;
  uint8_t* agg;        // [n_duties][96]
};

__global__ void __launch_bounds__(64) k_decode_pubkeys(const uint8_t* pk48, uint32_t n, G1A* out, int32_t* status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t b[48];
  for (int j = 0; j < 48; ++j) b[j] = pk48[48ull * i + j];
  G1A a;
  int32_t st = g1_decompress(b, a);
  if (st != DEC_OK) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  out[i] = a;
  status[i] = st;
}

__global__ void __launch_bounds__(64) k_decode_sigs(DevBatch B) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials) return;
  uint8_t b[96];
  for (int j = 0; j < 96; ++j) b[j] = B.sigs[96ull * i + j];
  G2A a;
  int32_t st = g2_decompress(b, a);
  if (st == DEC_IDENTITY) st = TBG_PS_ERR_IDENTITY;
  if (st != DEC_OK) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  B.sig_aff[i] = a;
  B.partial_status[i] = (st == DEC_OK) ? TBG_PS_NOT_VERIFIED : st;
}

__global__ void __launch_bounds__(64) k_hash_msgs(DevBatch B) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B.n_msgs) return;
  uint32_t off = B.msg_off[m], len = B.msg_off[m + 1] - off;
  G2J h = hash_to_g2(B.msgs + off, len);
  G2A a;
  bool ok = jac_to_aff(h, a);
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  B.h_aff[m] = a;
  B.h_status[m] = ok ? 0 : 1;
}

__global__ void __launch_bounds__(64) k_verify(DevBatch B, const G1A* pk_aff, const int32_t* pk_status, uint32_t n_pk) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials) return;
  int32_t st = B.partial_status[i];
  if (st != TBG_PS_NOT_VERIFIED) return;  // decode error already recorded
  uint32_t pid = B.pubkey_ids[i];
  if (pid >= n_pk || pk_status[pid] != DEC_OK) {
    B.partial_status[i] = TBG_PS_ERR_PUBKEY;
    return;
  }
  uint32_t m = B.duty_msg[B.partial_duty[i]];
  if (B.h_status[m] != 0) {
    B.partial_status[i] = TBG_PS_INVALID;
    return;
  }
  bool ok = bls_verify_prepared(pk_aff[pid], B.h_aff[m], B.sig_aff[i]);
  B.partial_status[i] = ok ? TBG_PS_VALID : TBG_PS_INVALID;
}

// Participation of partial i in its duty's aggregate.
TBG_HD bool participates(uint32_t op, int32_t st) {
  return op == TBG_OP_VERIFY_AGGREGATE ? (st == TBG_PS_VALID) : (st == TBG_PS_NOT_VERIFIED);
}

__global__ void __launch_bounds__(64) k_lagrange(DevBatch B) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials) return;
  uint32_t* w = B.lam + 8ull * i;
  for (int j = 0; j < 8; ++j) w[j] = 0;
  if (!participates(B.op, B.partial_status[i])) return;
  uint32_t d = B.partial_duty[i];
  uint32_t first = B.duty_first[d], last = B.duty_first[d + 1];
  uint8_t ids[256];
  int k = 0, me = -1;
  for (uint32_t j = first; j < last; ++j) {
    if (!participates(B.op, B.partial_status[j])) continue;
    if (j == i) me = k;
    ids[k++] = B.identifiers[j];
  }
  uint32_t lw[8];
  if (!lagrange_at_zero_words(ids, k, me, lw)) return;  // duplicate ids: duty kernel reports it
  for (int j = 0; j < 8; ++j) w[j] = lw[j];
}

__global__ void __launch_bounds__(64) k_aggregate(DevBatch B) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= B.n_duties) return;
  uint8_t* out = B.agg + 96ull * d;
  for (int j = 0; j < 96; ++j) out[j] = 0;
  uint32_t first = B.duty_first[d], last = B.duty_first[d + 1];
  uint32_t n = last - first;
  if (B.op == TBG_OP_VERIFY) {
    B.duty_status[d] = TBG_DS_NOT_AGGREGATED;
    return;
  }
  int k = 0;
  bool decode_err = false, identity = false;
  for (uint32_t j = first; j < last; ++j) {
    int32_t st = B.partial_status[j];
    if (participates(B.op, st)) ++k;
    if (st == TBG_PS_ERR_IDENTITY) identity = true;
    else if (st < 0 && st != TBG_PS_ERR_PUBKEY) decode_err = true;
  }
  if (B.op == TBG_OP_VERIFY_AGGREGATE) {
    uint32_t t = B.duty_threshold[d];
    if (n < t) { B.duty_status[d] = TBG_DS_INSUFFICIENT; return; }
    if ((uint32_t)k < t) { B.duty_status[d] = TBG_DS_INSUFFICIENT_VALID; return; }
  } else {
    if (decode_err) { B.duty_status[d] = TBG_DS_DECODE; return; }
    if (identity) { B.duty_status[d] = TBG_DS_AGG_IDENTITY; return; }
  }
  if (k < 2) { B.duty_status[d] = TBG_DS_AGG_TOO_FEW; return; }
  // duplicate identifiers among participants
  for (uint32_t a = first; a < last; ++a) {
    if (!participates(B.op, B.partial_status[a])) continue;
    for (uint32_t b = a + 1; b < last; ++b) {
      if (participates(B.op, B.partial_status[b]) && B.identifiers[a] == B.identifiers[b]) {
        B.duty_status[d] = TBG_DS_AGG_DUPLICATE_ID;
        return;
      }
    }
  }
  // Straus: one shared doubling chain over the 255-bit scalars.
  G2J acc = jac_inf<Fp2>();
  for (int bit = 254; bit >= 0; --bit) {
    acc = jac_dbl(acc);
    for (uint32_t j = first; j < last; ++j) {
      if (!participates(B.op, B.partial_status[j])) continue;
      if ((B.lam[8ull * j + (bit >> 5)] >> (bit & 31)) & 1) acc = jac_add_aff(acc, B.sig_aff[j]);
    }
  }
  G2A a;
  if (!jac_to_aff(acc, a)) { B.duty_status[d] = TBG_DS_AGG_IDENTITY; return; }
  uint8_t enc[96];
  g2_compress(a, false, enc);
  for (int j = 0; j < 96; ++j) out[j] = enc[j];
  B.duty_status[d] = TBG_DS_OK;
}

}  // namespace tbg

namespace tbg {

// ---- test-vector / benchmark-input generation (tbls.Sign / PartialSign,
// reference tbls/tss.go:200-217; sk -> pk as bls_sig.SecretKey.GetPublicKey) ----
TBG_HD void sk_words_from_be32(const uint8_t* b, uint32_t (&w)[8]) {
  for (int i = 0; i < 8; ++i)
    w[i] = ((uint32_t)b[31 - 4 * i]) | ((uint32_t)b[30 - 4 * i] << 8) | ((uint32_t)b[29 - 4 * i] << 16) |
           ((uint32_t)b[28 - 4 * i] << 24);
}

__global__ void __launch_bounds__(64) k_sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* pk48) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  sk_words_from_be32(sk32 + 32ull * i, w);
  G1J g = {fp_from_const(G1_X), fp_from_const(G1_Y), fp_one()};
  G1J p = jac_mul_words(g, w, 256);
  G1A a;
  bool ok = jac_to_aff(p, a);
  uint8_t enc[48];
  g1_compress(a, !ok, enc);
  for (int j = 0; j < 48; ++j) pk48[48ull * i + j] = enc[j];
}

__global__ void __launch_bounds__(64) k_sign(const uint8_t* sk32, const uint32_t* item_msg, uint32_t n, const G2A* h_aff,
                                             const int32_t* h_status, uint8_t* sig96) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  sk_words_from_be32(sk32 + 32ull * i, w);
  uint32_t m = item_msg[i];
  G2A a;
  bool ok = false;
  if (h_status[m] == 0) {
    G2J p = jac_mul_words(jac_from_aff(h_aff[m]), w, 256);
    ok = jac_to_aff(p, a);
  }
  uint8_t enc[96];
  g2_compress(a, !ok, enc);
  for (int j = 0; j < 96; ++j) sig96[96ull * i + j] = enc[j];
}

}  // namespace tbg
