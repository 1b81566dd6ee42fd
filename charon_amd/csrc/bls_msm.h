// Level-0 bucket MSM: S = sum_i [r_i] s_i over every candidate of a device
// batch without a per-partial G2 scalar multiplication (k_msm.hip).
//
// r_i = a_0 + a_1 x + a_2 x^2 + a_3 x^3 with odd signed digits |a_k| < 2^16
// (bls_rlc.h), and [r_i] s_i = sum_k a_k psi^k(s_i) for s_i in G2.  So
//   S = sum_{i,k} a_ik psi^k(s_i) = sum_j (2j + 1) B_j,
//   B_j = sum of sign(a_ik) psi^k(s_i) over the (i, k) with |a_ik| = 2j + 1:
// 4 mixed additions per partial into 32768 buckets, then one 16-bit scalar
// multiplication per bucket and a tree sum -- Pippenger's bucket method with
// the digit as the bucket index.  The sum is a group element, so the order in
// which entries reach a bucket (atomics) changes its Jacobian form only.
#pragma once
#include "bls_rlc.h"

namespace tbg {

// Bucket of digit word u (a = 2u - (2^16 - 1)): j = (|a| - 1) / 2 and the sign.
TBG_HD uint32_t msm_bucket(uint32_t u, bool& neg) {
  neg = u < 0x8000u;
  return neg ? 0x7FFFu - u : u - 0x8000u;
}

// psi^k(s) for an affine point of G2 (k = 0..3): psi(x, y) = (conj(x) PSI_X,
// conj(y) PSI_Y) and psi^2(x, y) = (PSI2_X x, -y), as the RLC tables use them.
TBG_HD G2A msm_psi_k(const G2A& s, uint32_t k) {
  G2A p = s;
  if (k & 1) p = g2_psi_aff(p);
  if (k & 2) p = G2A{fp2_mul_fp(p.x, fp_from_const(PSI2_X)), fp2_reduce(fp2_neg(p.y))};
  return p;
}

TBG_HD uint32_t msm_entry(uint32_t i, uint32_t k, bool neg) { return (i << 3) | (k << 1) | (neg ? 1u : 0u); }

// Level 1's group MSM (k_gmsm.hip): window w of digit word u (bits 4w .. 4w +
// 3 as signed binary digits) is v = 2 nibble - 15, odd with |v| <= 15; its
// bucket w * 8 + (|v| - 1) / 2 (of GM_BUCKETS = 32) and sign.  a_k = sum_w
// 16^w v_w, so S = sum_w 16^w sum_b (2b + 1) B_(w, b).
TBG_HD uint32_t gm_bucket(uint32_t u, uint32_t w, bool& neg) {
  const uint32_t nib = (u >> (4 * w)) & 15u;
  neg = nib < 8u;
  return 8u * w + (neg ? 7u - nib : nib - 8u);
}

// Host reference of the group MSM (tests/hostcheck): sum_i [r_i] s_i with
// the 4-bit windows, buckets, running sums and the base-16 combination of
// k_gmsm.hip; lead < n takes r = 1 (the group's first candidate).
TBG_HD G2J gm_reference(const G2A* s, const uint64_t* r, uint32_t n, uint32_t lead) {
  G2J bk[32];
  for (uint32_t b = 0; b < 32; ++b) bk[b] = jac_inf<Fp2>();
  for (uint32_t i = 0; i < n; ++i) {
    if (i == lead) {
      bk[0] = jac_add_aff(bk[0], s[i]);
      continue;
    }
    uint32_t u[4];
    rlc_digits(r[i], u);
    for (uint32_t k = 0; k < 4; ++k) {
      const G2A pk = msm_psi_k(s[i], k);
      for (uint32_t w = 0; w < 4; ++w) {
        bool neg;
        const uint32_t b = gm_bucket(u[k], w, neg);
        G2A p = pk;
        if (neg) p.y = fp2_reduce(fp2_neg(p.y));
        bk[b] = jac_add_aff(bk[b], p);
      }
    }
  }
  G2J S = jac_inf<Fp2>();
  for (int w = 3; w >= 0; --w) {
    for (int d = 0; d < 4 && w < 3; ++d) S = jac_dbl(S);
    G2J run = jac_inf<Fp2>(), acc = jac_inf<Fp2>();
    for (int b = 7; b >= 1; --b) {
      run = jac_add(run, bk[8 * w + b]);
      acc = jac_add(acc, run);
    }
    run = jac_add(run, bk[8 * w]);
    S = jac_add(S, jac_add(jac_dbl(acc), run));
  }
  return S;
}

// Host reference of the whole method (tests/hostcheck): sum_i [r_i] s_i.
TBG_HD G2J msm_reference(const G2A* s, const uint64_t* r, uint32_t n, G2J* buckets /* [MSM_BUCKETS_HOST] */) {
  constexpr uint32_t NB = 32768;
  for (uint32_t j = 0; j < NB; ++j) buckets[j] = jac_inf<Fp2>();
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t u[4];
    rlc_digits(r[i], u);
    for (uint32_t k = 0; k < 4; ++k) {
      bool neg;
      const uint32_t j = msm_bucket(u[k], neg);
      G2A p = msm_psi_k(s[i], k);
      if (neg) p.y = fp2_reduce(fp2_neg(p.y));
      buckets[j] = jac_add_aff(buckets[j], p);
    }
  }
  G2J acc = jac_inf<Fp2>();
  for (uint32_t j = 0; j < NB; ++j) {
    if (jac_is_inf(buckets[j])) continue;
    acc = jac_add(acc, jac_mul_u64(buckets[j], 2ull * j + 1));
  }
  return acc;
}

}  // namespace tbg
