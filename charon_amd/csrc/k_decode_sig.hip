// k_decode_sigs: the flags / field / Fp2 square-root half of the signature
// decode (tblsconv.SigFromCore, tblsconv.go:125-132; the subgroup half is
// k_decode.hip's k_subgroup_sigs or the batched test of k_sgb.hip).
//
// The square root is two Fp exponentiations, each one long chain of
// dependent Montgomery products whose carry chain (m_k, column to column)
// leaves the SIMD idle between instructions.  A lane takes TWO signatures,
// i and i + n/2, and runs their exponentiations interleaved
// (fp2_sqrt_x2 / fp_pow_const_x2): the other chain's multiply-adds fill
// those gaps.  This translation unit is compiled WITHOUT TBG_SCHED_FENCE
// (k_decode.hip keeps it for the lane-pair kernel), so the scheduler may
// interleave the two products.  TBG_DECODE_X2=0: one signature per lane.
#include "tbls_launch.h"
#include "bls_curve.h"

#ifndef TBG_DECODE_X2
#define TBG_DECODE_X2 1
#endif

namespace tbg {

// flags and field of one 96-byte compressed G2 point (the first half of
// g2_decompress_t): DEC_OK with x and rhs = x^3 + b, or the decode status
struct SigIn {
  int32_t st;
  uint32_t s_flag;
  Fp2 x, rhs;
};
__device__ __forceinline__ SigIn sig_parse(const uint8_t* src) {
  SigIn r;
  uint8_t b[96];
  for (int j = 0; j < 96; ++j) b[j] = src[j];
  const uint32_t c_flag = (b[0] >> 7) & 1, i_flag = (b[0] >> 6) & 1;
  r.s_flag = (b[0] >> 5) & 1;
  r.x = r.rhs = fp2_zero();
  if (!c_flag) {
    r.st = DEC_ERR_FLAGS;
    return r;
  }
  b[0] &= 0x1f;
  bool lt1, lt0;
  const Fp x1 = fp_limbs_from_be48(b, &lt1);
  const Fp x0 = fp_limbs_from_be48(b + 48, &lt0);
  if (i_flag) {
    uint32_t o = 0;
    for (int i = 0; i < NL; ++i) o |= x0.l[i] | x1.l[i];
    r.st = (r.s_flag == 0 && o == 0) ? DEC_IDENTITY : DEC_ERR_FLAGS;
    return r;
  }
  if (!lt0 || !lt1) {
    r.st = DEC_ERR_FIELD;
    return r;
  }
  r.x = {fp_to_mont(x0), fp_to_mont(x1)};
  r.rhs = fp2_reduce(fp2_add(fp2_mul(fp2_sqr(r.x), r.x), fp2_from_const(B2_M)));
  r.st = DEC_OK;
  return r;
}

// y from its root (sign by the s flag) and the partial's status / point
__device__ __forceinline__ void sig_store(const DevBatch& B, uint32_t i, const SigIn& s, bool root_ok, Fp2 y) {
  int32_t st = s.st;
  if (st == DEC_OK && !root_ok) st = DEC_ERR_NOT_ON_CURVE;
  if (st == DEC_IDENTITY) st = TBG_PS_ERR_IDENTITY;
  G2A a{fp2_zero(), fp2_zero()};
  if (st == DEC_OK) {
    if ((uint32_t)fp2_lex_largest(y) != s.s_flag) y = fp2_reduce(fp2_neg(y));
    a = {s.x, y};
  }
  B.sig_aff[i] = a;
  B.partial_status[i] = (st == DEC_OK) ? TBG_PS_NOT_VERIFIED : st;
}

__global__ void TBG_LAUNCH_N(TBG_DECODE_WAVES) k_decode_sigs(DevBatch B) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  // The chain's first kernel zeroes its work-list counters and level 0's
  // bucket sizes (a runtime memset kernel queued behind other streams' waves
  // held each chain for ~2 ms in the pipelined bench)
  if (t < CNT_WORDS) B.counters[t] = 0;
  if (B.rlc_batch && t <= MSM_BUCKETS) B.msm_off[t] = 0;
#if TBG_DECODE_X2
  const uint32_t half = (B.n_partials + 1) / 2;
  if (t >= half) return;
  const uint32_t i1 = t + half;
  const bool two = i1 < B.n_partials;
  const SigIn s0 = sig_parse(B.sigs + 96ull * t);
  SigIn s1;
  if (two) s1 = sig_parse(B.sigs + 96ull * i1);
  else {
    s1.st = DEC_ERR_FLAGS;
    s1.s_flag = 0;
    s1.x = s1.rhs = fp2_zero();
  }
  Fp2 y0, y1;
  const uint32_t f = fp2_sqrt_x2(s0.rhs, s1.rhs, y0, y1);
  bool ok0 = f & 1u, ok1 = (f >> 1) & 1u;
  // rhs in Fp (rhs.c1 == 0, only for crafted x): the reference root
  if (s0.st == DEC_OK && ((f >> 2) & 1u)) ok0 = fp2_sqrt(s0.rhs, y0);
  if (s1.st == DEC_OK && ((f >> 3) & 1u)) ok1 = fp2_sqrt(s1.rhs, y1);
  sig_store(B, t, s0, ok0, y0);
  if (two) sig_store(B, i1, s1, ok1, y1);
#else
  if (t >= B.n_partials) return;
  const SigIn s = sig_parse(B.sigs + 96ull * t);
  Fp2 y = fp2_zero();
  const bool ok = s.st == DEC_OK && fp2_sqrt(s.rhs, y);
  sig_store(B, t, s, ok, y);
#endif
}

void launch_decode_roots(const DevBatch& B, hipStream_t st) {
  // at least enough lanes to zero the counters (and level 0's bucket sizes)
  uint32_t lanes = TBG_DECODE_X2 ? (B.n_partials + 1) / 2 : B.n_partials;
  if (lanes < CNT_WORDS) lanes = CNT_WORDS;
  if (B.rlc_batch && lanes < MSM_BUCKETS + 1) lanes = MSM_BUCKETS + 1;
  TBG_KLAUNCH(k_decode_sigs, grid_for(lanes), dim3(kBlock), st, B);
}

}  // namespace tbg
