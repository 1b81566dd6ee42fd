// Threshold recombination (kryptology SigEth2.CombineSignatures, reached from
// reference tbls/tss.go:142-149 and :181): sigma = sum_i lambda_i(0) sigma_i,
// lambda_i(0) = prod_{j != i} x_j / (x_j - x_i) mod r, x_i = Identifier.
#pragma once
#include "bls_fr.h"
#include "bls_curve.h"

namespace tbg {

// lambda_i(0) as canonical scalar words; false when two identifiers collide.
// ids: identifiers of the k participating partials, i: index into ids.
TBG_NI bool lagrange_at_zero_words(const uint8_t* ids, int k, int i, uint32_t (&w)[8]) {
  Fr one = fr_from_u32(1);
  Fr num = one, den = one;
  Fr xi = fr_from_u32(ids[i]);
  for (int j = 0; j < k; ++j) {
    if (j == i) continue;
    Fr xj = fr_from_u32(ids[j]);
    num = fr_mul(num, xj);
    den = fr_mul(den, fr_sub(xj, xi));
  }
  if (fr_is_zero(den)) return false;
  fr_to_words(fr_mul(num, fr_inv(den)), w);
  return true;
}

// ---------------------------------------------------------------------------
// Integer form of the Lagrange coefficients.  lambda_i(0) = a_i / b_i with
// small integers; with D = lcm(b_i) and N_i = a_i D / b_i the aggregate is
// [D^-1 mod r] (sum_i N_i sigma_i): for identifiers 1..n the N_i are signed
// binomials and D = 1 (e.g. {1,2,3,4} -> (4, -6, 4, -1)), so the 255-bit MSM
// collapses to a few doublings and additions.  The group element is the same
// because every sigma_i has order r (decoded points are subgroup-checked).
TBG_HD uint64_t gcd_u64(uint64_t a, uint64_t b) {
  while (b) {
    uint64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

TBG_HD int bitlen_u64(uint64_t v) { return v ? 64 - __builtin_clzll(v) : 0; }

// Reduced fraction lambda_j(0) = (neg ? -a : a) / b of participant j, b > 0.
// Returns 1, 0 when the products would overflow 62 bits, -1 on duplicates.
TBG_HD int lagrange_frac(const uint8_t* ids, int k, int j, uint64_t& a, uint64_t& b, int& neg) {
  uint64_t num = 1, den = 1;
  int bits = 0;
  neg = 0;
  for (int m = 0; m < k; ++m) {
    if (m == j) continue;
    int64_t d = (int64_t)ids[m] - (int64_t)ids[j];
    if (d == 0) return -1;
    if (d < 0) { neg ^= 1; d = -d; }
    bits += bitlen_u64(ids[m]) + bitlen_u64((uint64_t)d);
    if (bits > 62) return 0;
    num *= ids[m];
    den *= (uint64_t)d;
  }
  if (num == 0) {
    a = 0;
    b = 1;
  } else {
    uint64_t g = gcd_u64(num, den);
    a = num / g;
    b = den / g;
  }
  return 1;
}

// Returns 1 on success (N, D set), 0 when the integers would overflow (use
// the mod-r path), -1 on duplicate identifiers.  The integer / mod-r choice
// is a property of the participant SET, never of i: every participant of a
// duty must get its coefficient in the same encoding, because tss_combine
// reads the mode of the first one for all of them.  So the overflow test runs
// over every j (pass 2), not only over i.
TBG_NI int lagrange_int(const uint8_t* ids, int k, int i, int64_t& N, uint64_t& D) {
  uint64_t lcm = 1;
  uint64_t a, b;
  int neg;
  for (int j = 0; j < k; ++j) {  // pass 1: D = lcm of the reduced denominators
    int r = lagrange_frac(ids, k, j, a, b, neg);
    if (r <= 0) return r;
    uint64_t q = b / gcd_u64(lcm, b);
    if (bitlen_u64(lcm) + bitlen_u64(q) > 62) return 0;
    lcm *= q;
  }
  int64_t ni = 0;
  for (int j = 0; j < k; ++j) {  // pass 2: every N_j = a_j D / b_j must fit
    lagrange_frac(ids, k, j, a, b, neg);
    uint64_t scale = lcm / b;
    if (bitlen_u64(a) + bitlen_u64(scale) > 62) return 0;
    if (j == i) ni = neg ? -(int64_t)(a * scale) : (int64_t)(a * scale);
  }
  N = ni;
  D = lcm;
  return 1;
}

TBG_HD Fr fr_from_u64(uint64_t v) {
  Fr a = fr_zero();
  a.l[0] = (uint32_t)(v & LMASK);
  a.l[1] = (uint32_t)((v >> 28) & LMASK);
  a.l[2] = (uint32_t)(v >> 56);
  return fr_mul(a, fr_from_limbs(R_R2_M));
}

// Encoding of a partial's coefficient in its 8-word lam slot:
//   mod-r mode:   words = lambda_i(0) (bit 255 clear)
//   integer mode: w[7] = 0x80000000 | sign, w[0..1] = |N_i|, w[2..3] = D
constexpr uint32_t LAM_INT_FLAG = 0x80000000u;

// Coefficient words of participant `me` among `ids[0..k)`; false on duplicates.
TBG_NI bool lagrange_encode(const uint8_t* ids, int k, int me, uint32_t (&w)[8]) {
  int64_t N;
  uint64_t D;
  int r = lagrange_int(ids, k, me, N, D);
  if (r < 0) return false;
  for (int j = 0; j < 8; ++j) w[j] = 0;
  if (r == 1) {
    uint64_t mag = (uint64_t)(N < 0 ? -N : N);
    w[0] = (uint32_t)mag;
    w[1] = (uint32_t)(mag >> 32);
    w[2] = (uint32_t)D;
    w[3] = (uint32_t)(D >> 32);
    w[7] = LAM_INT_FLAG | (N < 0 ? 1u : 0u);
    return true;
  }
  return lagrange_at_zero_words(ids, k, me, w);
}

// sum_j coeff_j * P_j over the participants (mask[j] != 0), coefficients as
// encoded by lagrange_encode.  pts / lam are indexed j = 0..count-1.
// defer_D != nullptr: an integer-mode sum with denominator D > 1 is returned
// before the [1/D] multiplication and *defer_D = D (else *defer_D = 1); the
// caller finishes it with tss_div_den.
//
// [k] P for a 255-bit k on G2 as a 4-way MSM of 64-bit digits: psi(P) = [x] P
// on G2 and x < 0, so [|x|^i] P = (-psi)^i (P) and with the base-|x| digits
// k = d0 + d1 |x| + d2 |x|^2 + d3 |x|^3 (0 <= d_i < |x|; r < |x|^4)
//   [k] P = [d0] P + [d1] (-psi(P)) + [d2] psi^2(P) + [d3] (-psi^3(P)).
// 64 doublings instead of 255; the GPU spreads the four terms over a lane quad
// (k_aggregate_finish).  P must have order r (decoded points are subgroup-checked).
TBG_HD void base_x_digits(const uint32_t (&w)[8], uint64_t (&d)[4]) {
  uint32_t q[8];
  for (int j = 0; j < 8; ++j) q[j] = w[j];
  for (int i = 0; i < 3; ++i) {  // q, d_i = divmod(q, |x|), restoring division MSB first
    uint64_t rem = 0;
    for (int b = 255; b >= 0; --b) {
      const uint32_t bit = (q[b >> 5] >> (b & 31)) & 1u;
      const uint64_t top = rem >> 63;
      rem = (rem << 1) | bit;  // the true value is < 2|x| < 2^65: subtract mod 2^64
      const bool ge = top || rem >= X_ABS;
      if (ge) rem -= X_ABS;
      q[b >> 5] = (q[b >> 5] & ~(1u << (b & 31))) | ((ge ? 1u : 0u) << (b & 31));
    }
    d[i] = rem;
  }
  d[3] = (uint64_t)q[0] | ((uint64_t)q[1] << 32);  // q < |x| after three divisions
}
// The four MSM bases: (-psi)^i (P).
TBG_HD G2J base_x_point(const G2J& p, int i) {
  G2J q = p;
  for (int j = 0; j < i; ++j) q = g2_psi(q);
  return (i & 1) ? jac_neg(q) : q;
}
TBG_HD G2J g2_mul_base_x(const G2J& p, const uint64_t (&d)[4]) {
  G2J q[4];
  for (int i = 0; i < 4; ++i) q[i] = base_x_point(p, i);
  G2J acc = jac_inf<Fp2>();
  for (int b = 63; b >= 0; --b) {  // Straus: one doubling chain for the four digits
    acc = jac_dbl(acc);
    for (int i = 0; i < 4; ++i)
      if ((d[i] >> b) & 1) acc = jac_add(acc, q[i]);
  }
  return acc;
}
TBG_HD void inv_den_digits(uint64_t D, uint64_t (&d)[4]) {
  uint32_t dw[8];
  fr_to_words(fr_inv(fr_from_u64(D)), dw);
  base_x_digits(dw, d);
}
TBG_HD G2J tss_div_den(const G2J& acc, uint64_t D) {
  uint64_t d[4];
  inv_den_digits(D, d);
  return g2_mul_base_x(acc, d);
}
TBG_NI G2J tss_combine(const G2A* pts, const uint32_t* lam, const uint8_t* mask, int count,
                       uint64_t* defer_D = nullptr) {
  if (defer_D) *defer_D = 1;
  int first = -1;
  for (int j = 0; j < count; ++j)
    if (mask[j]) { first = j; break; }
  if (first < 0) return jac_inf<Fp2>();
  G2J acc = jac_inf<Fp2>();
  if (lam[8 * first + 7] & LAM_INT_FLAG) {
    int nbits = 0;
    for (int j = 0; j < count; ++j) {
      if (!mask[j]) continue;
      uint64_t mag = (uint64_t)lam[8 * j] | ((uint64_t)lam[8 * j + 1] << 32);
      nbits = nbits > bitlen_u64(mag) ? nbits : bitlen_u64(mag);
    }
    for (int bit = nbits - 1; bit >= 0; --bit) {
      acc = jac_dbl(acc);
      for (int j = 0; j < count; ++j) {
        if (!mask[j]) continue;
        uint64_t mag = (uint64_t)lam[8 * j] | ((uint64_t)lam[8 * j + 1] << 32);
        if ((mag >> bit) & 1) {
          G2A p = pts[j];
          if (lam[8 * j + 7] & 1) p.y = fp2_reduce(fp2_neg(p.y));
          acc = jac_add_aff(acc, p);
        }
      }
    }
    uint64_t D = (uint64_t)lam[8 * first + 2] | ((uint64_t)lam[8 * first + 3] << 32);
    if (D > 1) {
      if (defer_D) *defer_D = D;
      else acc = tss_div_den(acc, D);
    }
    return acc;
  }
  for (int bit = 254; bit >= 0; --bit) {
    acc = jac_dbl(acc);
    for (int j = 0; j < count; ++j)
      if (mask[j] && ((lam[8 * j + (bit >> 5)] >> (bit & 31)) & 1)) acc = jac_add_aff(acc, pts[j]);
  }
  return acc;
}

}  // namespace tbg
