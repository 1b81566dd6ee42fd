// Random-linear-combination scalars and their application (k_rlc.hip).
//
// r_i is 64 secret random bits u, split into four 16-bit words u_k and read
// as SIGNED binary digits (bit j of u_k set -> +1, clear -> -1):
//   a_k = sum_j e_kj 2^j = 2 u_k - (2^16 - 1)   (odd, |a_k| < 2^16)
//   r_i = a_0 + a_1 x + a_2 x^2 + a_3 x^3      (x = -0xd201000000010000).
// Distinct u give distinct r_i mod r (digit differences are < 2^17 < |x| and
// 2^17 |x|^3 < r), so the usual RLC bound (a false accept <= 1/2^64) holds.
// For a signature s that passed the subgroup check psi(s) = [x] s, and on G1
// [x^2] = -phi (phi(x, y) = (beta x, y)), so
//   [r] s  = sum_k a_k psi^k(s)  = T(s, psi(s))   + psi^2 T'(s, psi(s))
//   [r] pk = a_0 pk + a_1 [x]pk - a_2 phi(pk) - a_3 phi([x]pk)
//          = T(pk, [x]pk) - phi T'(pk, [x]pk)
// with psi^2(x, y) = (PSI2_X x, -y) and -phi(x, y) = (beta x, -y).  Every
// digit is non-zero, so each of the 16 bit positions adds exactly one entry
// of {+-(q0 + q1), +-(q0 - q1)} per pair: 15 doublings + 31 additions in
// uniform control flow.  (Unsigned 0/1 digits made the additions of the
// four points lane-divergent: a wave executed all 64 of them, masked.)
#pragma once
#include "bls_h2c.h"

namespace tbg {

// 64 bits of SHA-256's compression function keyed by the 32-byte batch seed:
// one block seed || i || 0x80 || 0... built as words in registers (the
// byte-stream sha256_block kept the block and its schedule in scratch).
TBG_HD void rlc_block(const uint32_t (&seed)[8], uint32_t i, uint32_t tag, uint32_t (&h)[8]) {
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = seed[k];
  w[8] = i;
  w[9] = tag;
#pragma unroll
  for (int k = 10; k < 16; ++k) w[k] = 0;
  sha256_iv(h);
  sha256_compress(h, w);
}
TBG_HD uint64_t rlc_scalar(const uint32_t (&seed)[8], uint32_t i) {
  uint32_t h[8];
  rlc_block(seed, i, 0x80000000u, h);
  uint64_t r = ((uint64_t)h[0] << 32) | h[1];
  return r ? r : 1;
}

// The batched subgroup test's coefficients of partial i (k_sgb.hip): 18
// signed digits c_k in [-6, 6] -- uniform mod 13 -- from the same keyed
// compression function on a separate message (a tag byte after i), four
// base-13 digits per 32-bit word (13^4 = 28561: bias < 2^-17 per digit).
// (The byte-stream sha256_block call here, not rlc_block's unrolled register
// form: that took k_sgb_sort from 66 to 256 VGPRs -- one wave per SIMD for
// its four-wave workgroups, which then waited for four free SIMDs on a CU
// behind the other launches' kernels: -1.3 % on the driver shape.)
TBG_HD void sgb_digits(const uint32_t (&seed)[8], uint32_t i, int32_t (&c)[18]) {
  uint8_t blk[64];
  for (int k = 0; k < 8; ++k) {
    blk[4 * k] = (uint8_t)(seed[k] >> 24);
    blk[4 * k + 1] = (uint8_t)(seed[k] >> 16);
    blk[4 * k + 2] = (uint8_t)(seed[k] >> 8);
    blk[4 * k + 3] = (uint8_t)seed[k];
  }
  for (int k = 32; k < 64; ++k) blk[k] = 0;
  blk[32] = (uint8_t)(i >> 24);
  blk[33] = (uint8_t)(i >> 16);
  blk[34] = (uint8_t)(i >> 8);
  blk[35] = (uint8_t)i;
  blk[36] = 0x53;  // 'S': not rlc_scalar's message
  blk[37] = 0x80;
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  sha256_block(h, blk);
  for (int k = 0; k < 18; ++k) {
    uint32_t w = h[k >> 2] % 28561u;
    for (int j = 0; j < (k & 3); ++j) w /= 13u;
    c[k] = (int32_t)(w % 13u) - 6;
  }
}

TBG_HD void rlc_digits(uint64_t r, uint32_t (&u)[4]) {
  for (int k = 0; k < 4; ++k) u[k] = (uint32_t)((r >> (16 * k)) & 0xFFFF);
}

TBG_HD G2A g2_psi_aff(const G2A& a) {
  return {fp2_mul(fp2_conj(a.x), fp2_from_const(PSI_X)), fp2_mul(fp2_conj(a.y), fp2_from_const(PSI_Y))};
}

TBG_HD Fp rlc_mul_c(const Fp& a, const Fp& c) { return fp_mul(a, c); }
TBG_HD Fp2 rlc_mul_c(const Fp2& a, const Fp& c) { return fp2_mul_fp(a, c); }

// Table entry e0 q0 + e1 q1 (e = +-1 from bits b0, b1) out of A+ = q0 + q1
// and A- = q0 - q1; `endo` maps it through (x, y) -> (c x, -y).  The sign is
// applied by negating the selected y (cheaper than keeping -y resident).
template <class F>
TBG_HD Aff<F> rlc_entry(const Aff<F>& ap, const Aff<F>& am, uint32_t b0, uint32_t b1, bool endo, const Fp& c) {
  const bool same = b0 == b1;
  const bool negy = (b0 != 0) == endo;  // -(..) for b0 = 0, and endo negates y once more
  Aff<F> e;
  e.x = same ? ap.x : am.x;
  const F y = same ? ap.y : am.y;
  const F ny = f_reduce(f_neg(y));
  e.y = negy ? ny : y;
  if (endo) e.x = rlc_mul_c(e.x, c);
  return e;
}

// A+ = q0 + q1 and A- = q0 - q1 in affine form given inv = 1 / (x1 - x0)
// (q0 != +-q1: both are non-identity points of prime order r and
// q1 = [x] q0 or psi(q0) = [x] q0 with x != +-1 mod r).
template <class F>
TBG_HD void rlc_pair_from_inv(const Aff<F>& q0, const Aff<F>& q1, const F& inv, Aff<F>& ap, Aff<F>& am) {
  const F lp = f_mul(f_reduce(f_sub(q1.y, q0.y)), inv);
  // decoded coordinates may be up to 16p (a negated root): reduce the sums
  const F lm = f_mul(f_reduce(f_neg(f_reduce(f_add(q1.y, q0.y)))), inv);
  const F xs = f_reduce(f_add(q0.x, q1.x));
  ap.x = f_reduce(f_sub(f_sqr(lp), xs));
  ap.y = f_reduce(f_sub(f_mul(lp, f_reduce(f_sub(q0.x, ap.x))), q0.y));
  am.x = f_reduce(f_sub(f_sqr(lm), xs));
  am.y = f_reduce(f_sub(f_mul(lm, f_reduce(f_sub(q0.x, am.x))), q0.y));
}

// sum_j 2^j (e0j q0 + e1j q1 + endo(e2j q0 + e3j q1)) from the pair table
// A+-, digits u (see top).
template <class F>
TBG_HD Jac<F> rlc_mul_table(const Aff<F>& ap, const Aff<F>& am, const Fp& c, const uint32_t (&u)[4]) {
  Jac<F> acc = jac_from_aff(rlc_entry(ap, am, (u[0] >> 15) & 1, (u[1] >> 15) & 1, false, c));
  acc = jac_add_aff_in(acc, rlc_entry(ap, am, (u[2] >> 15) & 1, (u[3] >> 15) & 1, true, c));
#pragma unroll 1
  for (int bit = 14; bit >= 0; --bit) {
    acc = jac_dbl_in(acc);
    acc = jac_add_aff_in(acc, rlc_entry(ap, am, (u[0] >> bit) & 1, (u[1] >> bit) & 1, false, c));
    acc = jac_add_aff_in(acc, rlc_entry(ap, am, (u[2] >> bit) & 1, (u[3] >> bit) & 1, true, c));
  }
  return acc;
}

// Per-key window table (k_pubkey_tables): the eight points e0 q0 + e1 q1,
// e0 in {1, 3}, e1 in {-3, -1, 1, 3} (q0 = pk, q1 = [x]pk), at index
// 4 (e0 == 3) + (e1 + 3) / 2.  Two bits of each of two digits (bit set ->
// +1, clear -> -1, as above) select one entry +-e0 q0 +- e1 q1 (the sign of
// e0 moved to y), so [r] pk takes 14 doublings + 16 additions instead of
// the pair table's 15 + 32 -- for a table resident per key (896 bytes).
constexpr uint32_t PK_TAB_W2 = 8;
template <class F>
TBG_HD Jac<F> rlc_key_table_w2_entry(const Aff<F>& q0, const Aff<F>& q1, int k) {
  const int e0 = k >= 4 ? 3 : 1, e1 = 2 * (k & 3) - 3;
  const Jac<F> a = jac_from_aff(q0), b = jac_from_aff(q1);
  Jac<F> p0 = e0 == 3 ? jac_add(jac_dbl(a), a) : a;
  Jac<F> p1 = (e1 == 3 || e1 == -3) ? jac_add(jac_dbl(b), b) : b;
  if (e1 < 0) p1 = jac_neg(p1);
  return jac_add(p0, p1);
}
// the window of bits 2i + 1, 2i of a digit: 2 (+-1) + (+-1)
TBG_HD int rlc_win2(uint32_t u, int i) {
  return 2 * (2 * (int)((u >> (2 * i + 1)) & 1u) - 1) + (2 * (int)((u >> (2 * i)) & 1u) - 1);
}
template <class F>
TBG_HD Aff<F> rlc_entry_w2(const Aff<F>* tab, int v0, int v1, bool endo, const Fp& c) {
  const bool neg = v0 < 0;
  if (neg) {
    v0 = -v0;
    v1 = -v1;
  }
  Aff<F> e = tab[(v0 == 3 ? 4 : 0) + (v1 + 3) / 2];
  if (neg != endo) e.y = f_reduce(f_neg(e.y));  // endo maps (x, y) -> (c x, -y)
  if (endo) e.x = rlc_mul_c(e.x, c);
  return e;
}
template <class F>
TBG_HD Jac<F> rlc_mul_key_w2(const Aff<F>* tab, const Fp& c, const uint32_t (&u)[4]) {
  Jac<F> acc = jac_from_aff(rlc_entry_w2(tab, rlc_win2(u[0], 7), rlc_win2(u[1], 7), false, c));
  acc = jac_add_aff_in(acc, rlc_entry_w2(tab, rlc_win2(u[2], 7), rlc_win2(u[3], 7), true, c));
#pragma unroll 1
  for (int i = 6; i >= 0; --i) {
    acc = jac_dbl_in(jac_dbl_in(acc));
    acc = jac_add_aff_in(acc, rlc_entry_w2(tab, rlc_win2(u[0], i), rlc_win2(u[1], i), false, c));
    acc = jac_add_aff_in(acc, rlc_entry_w2(tab, rlc_win2(u[2], i), rlc_win2(u[3], i), true, c));
  }
  return acc;
}

// [r] pk from the key's resident table (PK_TAB entries, tbls_launch.h)
#if defined(TBG_PK_W2)
TBG_HD G1J rlc_mul_key(const G1A* tab, const uint32_t (&u)[4]) {
#if TBG_PK_W2
  return rlc_mul_key_w2(tab, fp_from_const(G1_BETA), u);
#else
  return rlc_mul_table(tab[0], tab[1], fp_from_const(G1_BETA), u);
#endif
}
#endif

// [r] s for s in G2 (affine): pairs (s, psi(s)) and psi^2 of the same table.
TBG_HD G2J rlc_mul_g2(const G2A& s, const uint32_t (&u)[4]) {
  const G2A ps = g2_psi_aff(s);
  G2A ap, am;
  rlc_pair_from_inv(s, ps, fp2_inv(fp2_reduce(fp2_sub(ps.x, s.x))), ap, am);
  return rlc_mul_table(ap, am, fp_from_const(PSI2_X), u);
}

// [r] pk on G1: pairs (pk, [x]pk) and -phi of the same table.
TBG_HD G1J rlc_mul_g1(const G1A& pk, const G1A& xpk, const uint32_t (&u)[4]) {
  G1A ap, am;
  rlc_pair_from_inv(pk, xpk, fp_inv(fp_reduce(fp_sub(xpk.x, pk.x))), ap, am);
  return rlc_mul_table(ap, am, fp_from_const(G1_BETA), u);
}

// Both products of one partial (k_rlc_partial) with ONE field inversion for
// the two tables (Montgomery's trick on dx1 and the norm n2 of dx2):
// t = 1 / (dx1 n2), 1/dx1 = t n2, 1/dx2 = conj(dx2) t dx1.
TBG_HD void rlc_mul_both(const G2A& s, const G1A& pk, const G1A& xpk, const uint32_t (&u)[4], G2J& S, G1J& P) {
  const G2A ps = g2_psi_aff(s);
  const Fp2 dx2 = fp2_reduce(fp2_sub(ps.x, s.x));
  const Fp dx1 = fp_reduce(fp_sub(xpk.x, pk.x));
  const Fp n2 = fp_mul2(dx2.c0, dx2.c0, dx2.c1, dx2.c1);
  const Fp t = fp_inv(fp_mul(n2, dx1));
  const Fp in2 = fp_mul(t, dx1);
  {
    G2A ap, am;
    rlc_pair_from_inv(s, ps, Fp2{fp_mul(dx2.c0, in2), fp_mul(fp_neg(dx2.c1), in2)}, ap, am);
    S = rlc_mul_table(ap, am, fp_from_const(PSI2_X), u);
  }
  {
    G1A ap, am;
    rlc_pair_from_inv(pk, xpk, fp_mul(t, n2), ap, am);
    P = rlc_mul_table(ap, am, fp_from_const(G1_BETA), u);
  }
}

// ---------------------------------------------------------------------------
// Inversion-free form (the split kernels k_rlc_g1 / k_rlc_g2_pair): the pair
// table A+- = q0 +- q1 stays Jacobian (one mixed addition each) and the 31
// table additions are full Jacobian additions.  Against the affine table this
// trades the field inversion (~480 Fp products, which the two lanes of a
// pair would both run) for 31 x (4M + 1S) extra products that the pair
// splits -- and it keeps no inversion on the lane at all.
template <class F>
TBG_HD Jac<F> rlc_entry_j(const Jac<F>& ap, const Jac<F>& am, uint32_t b0, uint32_t b1, bool endo, const Fp& c) {
  const bool same = b0 == b1;
  const bool negy = (b0 != 0) == endo;
  Jac<F> e;
  e.X = same ? ap.X : am.X;
  e.Z = same ? ap.Z : am.Z;
  const F y = same ? ap.Y : am.Y;
  const F ny = f_reduce(f_neg(y));
  e.Y = negy ? ny : y;
  if (endo) e.X = rlc_mul_c(e.X, c);  // (x, y) -> (c x, -y): X scales like x
  return e;
}

template <class F>
TBG_HD void rlc_pair_jac(const Aff<F>& q0, const Aff<F>& q1, Jac<F>& ap, Jac<F>& am) {
  const Jac<F> j0 = jac_from_aff(q0);
  ap = jac_add_aff_in(j0, q1);
  am = jac_add_aff_in(j0, Aff<F>{q1.x, f_reduce(f_neg(q1.y))});
}

template <class F>
TBG_HD Jac<F> rlc_mul_table_j(const Jac<F>& ap, const Jac<F>& am, const Fp& c, const uint32_t (&u)[4]) {
  Jac<F> acc = rlc_entry_j(ap, am, (u[0] >> 15) & 1, (u[1] >> 15) & 1, false, c);
  acc = jac_add_in<F, true>(acc, rlc_entry_j(ap, am, (u[2] >> 15) & 1, (u[3] >> 15) & 1, true, c));
#pragma unroll 1
  for (int bit = 14; bit >= 0; --bit) {
    acc = jac_dbl_in(acc);
    acc = jac_add_in<F, true>(acc, rlc_entry_j(ap, am, (u[0] >> bit) & 1, (u[1] >> bit) & 1, false, c));
    acc = jac_add_in<F, true>(acc, rlc_entry_j(ap, am, (u[2] >> bit) & 1, (u[3] >> bit) & 1, true, c));
  }
  return acc;
}

// [r] pk on G1, inversion-free: pairs (pk, [x]pk) and -phi of the same table.
TBG_HD G1J rlc_mul_g1_j(const G1A& pk, const G1A& xpk, const uint32_t (&u)[4]) {
  G1J ap, am;
  rlc_pair_jac(pk, xpk, ap, am);
  return rlc_mul_table_j(ap, am, fp_from_const(G1_BETA), u);
}

}  // namespace tbg
