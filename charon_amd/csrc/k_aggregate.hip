// Threshold recombination (CombineSignatures, tss.go:142-149 / :181): Lagrange
// coefficients, G2 combination, affine conversion and 96-byte compression.
#include "tbls_launch.h"
#include "bls_tss.h"

namespace tbg {

__global__ void TBG_LAUNCH k_lagrange(DevBatch B) {
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
  if (!lagrange_encode(ids, k, me, lw)) return;  // duplicate ids: duty kernel reports it
  for (int j = 0; j < 8; ++j) w[j] = lw[j];
}

// Affine conversion, compression and status of a finished sum.
__device__ void agg_emit(const DevBatch& B, uint32_t d, const G2J& acc) {
  uint8_t* out = B.agg + 96ull * d;
  G2A a;
  if (!jac_to_aff(acc, a)) { B.duty_status[d] = TBG_DS_AGG_IDENTITY; return; }
  uint8_t enc[96];
  g2_compress(a, false, enc);
  for (int j = 0; j < 96; ++j) out[j] = enc[j];
  B.duty_status[d] = TBG_DS_OK;
}

// Duties whose participants' integer Lagrange coefficients share a
// denominator D > 1 (a partial missing from the middle of the id range,
// e.g. ids {1,2,4}: lambda_1 = 8/3) need a 255-bit [1/D] multiplication.
// Inline, one such duty makes its whole 64-lane wave pay that loop; they are
// listed here instead and finished by k_aggregate_finish in uniform waves.
__global__ void TBG_LAUNCH k_aggregate(DevBatch B) {
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
  uint8_t mask[256];
  for (uint32_t j = first; j < last; ++j) mask[j - first] = participates(B.op, B.partial_status[j]) ? 1 : 0;
  uint64_t D = 1;
  G2J acc = tss_combine(B.sig_aff + first, B.lam + 8ull * first, mask, (int)n, &D);
  if (D > 1) {
    B.agg_acc[d] = acc;
    B.agg_list[atomicAdd(&B.counters[CNT_AGG], 1u)] = d;
    return;
  }
  agg_emit(B, d, acc);
}

__global__ void TBG_LAUNCH k_aggregate_finish(DevBatch B) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B.counters[CNT_AGG]) return;
  uint32_t d = B.agg_list[k];
  uint32_t first = B.duty_first[d], last = B.duty_first[d + 1];
  uint32_t j = first;
  while (j < last && !participates(B.op, B.partial_status[j])) ++j;
  const uint32_t* w = B.lam + 8ull * j;  // listed duties have a participant (k >= 2)
  uint64_t D = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  agg_emit(B, d, tss_div_den(B.agg_acc[d], D));
}

void launch_lagrange(const DevBatch& B, hipStream_t st) {
  if (B.n_partials) TBG_KLAUNCH(k_lagrange, grid_for(B.n_partials), dim3(kBlock), st, B);
}
void launch_aggregate(const DevBatch& B, hipStream_t st) {
  if (B.n_duties) TBG_KLAUNCH(k_aggregate, grid_for(B.n_duties), dim3(kBlock), st, B);
}
void launch_aggregate_finish(const DevBatch& B, hipStream_t st) {
  if (B.n_duties) TBG_KLAUNCH(k_aggregate_finish, grid_for(B.n_duties), dim3(kBlock), st, B);
}

}  // namespace tbg
