// Extension tower for BLS12-381 on gfx950:
//   Fp2  = Fp[u]  / (u^2 + 1)
//   Fp6  = Fp2[v] / (v^3 - xi),  xi = 1 + u
//   Fp12 = Fp6[w] / (w^2 - v)
//
// Bound conventions (multiples of p per Fp component; see bls_field.h):
//   fp2_mul / fp2_sqr      inputs < 16p, output < 2p
//   fp6_mul / fp6_sqr      inputs <  8p, output < 2p
//   fp12_mul / fp12_sqr    inputs <  4p, output < 2p
//   *_add / *_sub / *_neg  lazy (no reduction), the caller tracks growth
//   *_reduce               -> < 2p
#pragma once
#include "bls_field.h"

namespace tbg {

struct Fp2 { Fp c0, c1; };
struct Fp6 { Fp2 c0, c1, c2; };
struct Fp12 { Fp6 c0, c1; };

// ----------------------------------------------------------------- Fp2
TBG_HD Fp2 fp2_from_const(const Fp2Const& c) { return {fp_from_const(c.c0), fp_from_const(c.c1)}; }
TBG_HD Fp2 fp2_zero() { return {fp_zero(), fp_zero()}; }
TBG_HD Fp2 fp2_one() { return {fp_one(), fp_zero()}; }
TBG_HD Fp2 fp2_add(const Fp2& a, const Fp2& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
TBG_HD Fp2 fp2_dbl(const Fp2& a) { return fp2_add(a, a); }
TBG_HD Fp2 fp2_sub(const Fp2& a, const Fp2& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
TBG_HD Fp2 fp2_neg(const Fp2& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
TBG_HD Fp2 fp2_conj(const Fp2& a) { return {a.c0, fp_neg(a.c1)}; }
TBG_HD Fp2 fp2_reduce(const Fp2& a) { return {fp_reduce(a.c0), fp_reduce(a.c1)}; }
TBG_HD Fp2 fp2_canon(const Fp2& a) { return {fp_canon(a.c0), fp_canon(a.c1)}; }
TBG_HD Fp2 fp2_select(bool c, const Fp2& a, const Fp2& b) { return {fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)}; }
TBG_HD Fp2 fp2_mul_small(const Fp2& a, uint32_t k) { return {fp_mul_small(a.c0, k), fp_mul_small(a.c1, k)}; }
// lazy limbs (bls_field.h): results for reductions and first operands only
TBG_HD Fp2 fp2_add_l(const Fp2& a, const Fp2& b) { return {fp_add_l(a.c0, b.c0), fp_add_l(a.c1, b.c1)}; }
TBG_HD Fp2 fp2_sub_l(const Fp2& a, const Fp2& b) { return {fp_sub_l(a.c0, b.c0), fp_sub_l(a.c1, b.c1)}; }

// Fp2 product: two REDC(a b + c d) (fp_mul2).  (A Karatsuba form with lazy
// reduction -- 5 x 196 mul-adds instead of 6 x 196 -- measured no faster on
// MI355X, round 1: the extra 64-bit column arithmetic and register pressure
// eat the saved products; removed.)
TBG_HD Fp2 fp2_mul(const Fp2& a, const Fp2& b) {
  Fp nb1 = fp_neg(b.c1);
  return {fp_mul2(a.c0, b.c0, a.c1, nb1), fp_mul2(a.c0, b.c1, a.c1, b.c0)};
}

TBG_HD Fp2 fp2_sqr(const Fp2& a) {
  Fp s = fp_add_l(a.c0, a.c1);
  Fp d = fp_sub_l(a.c0, a.c1);
  Fp a0d = fp_add_l(a.c0, a.c0);
  return {fp_mul(s, d), fp_mul(a0d, a.c1)};
}

TBG_HD Fp2 fp2_mul_fp(const Fp2& a, const Fp& s) { return {fp_mul(a.c0, s), fp_mul(a.c1, s)}; }

// (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u   [lazy: c0 < a0 + 16p, c1 < a0 + a1;
// lazy limbs too: every use reduces it, adds it to something that is
// reduced or normalised, or subtracts from it]
TBG_HD Fp2 fp2_mul_xi(const Fp2& a) { return {fp_sub_l(a.c0, a.c1), fp_add_l(a.c0, a.c1)}; }

TBG_HD bool fp2_is_zero(const Fp2& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
TBG_HD bool fp2_eq(const Fp2& a, const Fp2& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }

TBG_HD Fp2 fp2_inv(const Fp2& a) {
  Fp n = fp_mul2(a.c0, a.c0, a.c1, a.c1);
  Fp t = fp_inv(n);
  return {fp_mul(a.c0, t), fp_mul(fp_neg(a.c1), t)};
}

// Where the inline square roots keep their input across the exponentiations:
// in registers (RegKeep), or a kernel's memory slot (k_hash.hip,
// k_decode.hip: a struct whose put / get store and load with compiler
// barriers) so that the 28 words are not live across them.
struct RegKeep {
  Fp2 v;
  TBG_HD void put(const Fp2& a) { v = a; }
  TBG_HD Fp2 get() const { return v; }
};

#if defined(__HIP__)
// ... the memory form: the compiler barriers stop the load from reusing the
// registers of the store
struct SlotKeep {
  Fp2* p;
  __device__ void put(const Fp2& a) const {
    *p = a;
    __asm__ __volatile__("" ::: "memory");
  }
  __device__ Fp2 get() const {
    __asm__ __volatile__("" ::: "memory");
    return *p;
  }
};
#endif

// Square root in Fp2 via two Fp exponentiations (norm method).
// Returns false when a is not a square.  The root returned is unspecified
// up to sign; callers fix the sign.  _in: inline (window width WIN, a kept
// by `keep` across the exponentiations); fp2_sqrt: out of line.
// a in Fp (a1 == 0) takes the first exponentiation only: s = a0^((p+1)/4)
// has s^2 = a0 chi(a0), so the root is (s, 0) for a residue and (0, s) for a
// non-residue ((s u)^2 = -s^2 = a0).
template <int WIN = 3, class Keep = RegKeep>
TBG_HD bool fp2_sqrt_in(const Fp2& a_in, Fp2& out, Keep keep = Keep{}) {
  Fp2 a = fp2_reduce(a_in);
  const bool real = fp_is_zero(a.c1);
  keep.put(a);
  const Fp norm = fp_select(real, a.c0, fp_mul2(a.c0, a.c0, a.c1, a.c1));
  const Fp gamma = fp_pow_const_in<EXP_SQRT_BITS, EXP_SQRT_WORDS, WIN>(norm);
  a = keep.get();
  const Fp g2 = fp_sqr(gamma);
  if (real) {
    if (fp_eq(g2, a.c0)) out = {gamma, fp_zero()};
    else if (fp_eq(g2, fp_reduce(fp_neg(a.c0)))) out = {fp_zero(), gamma};
    else return false;
    return true;
  }
  if (!fp_eq(g2, fp_mul2(a.c0, a.c0, a.c1, a.c1))) return false;
  const Fp inv2 = fp_from_const(INV2_M);
  const Fp delta = fp_mul(fp_add(a.c0, gamma), inv2);  // non-zero because a1 != 0
  const Fp t = fp_pow_const_in<EXP_PM3D4_BITS, EXP_PM3D4_WORDS, WIN>(delta);  // delta^((p-3)/4)
  a = keep.get();
  const Fp x0 = fp_mul(delta, t);
  const Fp x0sq = fp_sqr(x0);
  Fp2 r;
  if (fp_eq(x0sq, delta)) {
    // delta is a residue: x0 = sqrt(delta), x1 = a1 / (2 x0) = a1 t / 2
    r.c0 = x0;
    r.c1 = fp_mul(fp_mul(a.c1, t), inv2);
  } else {
    // non-residue: x0 = a1 t / 2, x1 = -delta t
    r.c0 = fp_mul(fp_mul(a.c1, t), inv2);
    r.c1 = fp_neg(x0);
  }
  if (!fp2_eq(fp2_sqr(r), a)) return false;
  out = r;
  return true;
}
TBG_NI bool fp2_sqrt(const Fp2& a_in, Fp2& out) { return fp2_sqrt_in<3>(a_in, out); }

// Legendre-style square test in Fp2: a is a square iff norm(a) is a square in Fp.
TBG_NI bool fp2_is_square(const Fp2& a) {
  Fp norm = fp_mul2(a.c0, a.c0, a.c1, a.c1);
  if (fp_is_zero(norm)) return true;
  Fp l = fp_pow_const<EXP_LEGENDRE_BITS, EXP_LEGENDRE_WORDS>(norm);
  return fp_eq(l, fp_one());
}

// RFC 9380 sgn0 for Fp2 (on canonical values)
TBG_HD uint32_t fp2_sgn0(const Fp2& a) {
  Fp c0 = fp_from_mont(a.c0), c1 = fp_from_mont(a.c1);
  uint32_t s0 = c0.l[0] & 1;
  uint32_t z0 = 1;
  for (int i = 0; i < NL; ++i) z0 &= (c0.l[i] == 0);
  uint32_t s1 = c1.l[0] & 1;
  return s0 | (z0 & s1);
}

// ZCash: lexicographically largest, c1 first then c0 (Montgomery input)
TBG_HD bool fp2_lex_largest(const Fp2& a) {
  Fp c0 = fp_from_mont(a.c0), c1 = fp_from_mont(a.c1);
  uint32_t z1 = 0;
  for (int i = 0; i < NL; ++i) z1 |= c1.l[i];
  if (z1 != 0) return fp_lex_largest_canon(c1);
  return fp_lex_largest_canon(c0);
}

// ----------------------------------------------------------------- Fp6
TBG_HD Fp6 fp6_zero() { return {fp2_zero(), fp2_zero(), fp2_zero()}; }
TBG_HD Fp6 fp6_one() { return {fp2_one(), fp2_zero(), fp2_zero()}; }
TBG_HD Fp6 fp6_add(const Fp6& a, const Fp6& b) { return {fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
TBG_HD Fp6 fp6_sub(const Fp6& a, const Fp6& b) { return {fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
TBG_HD Fp6 fp6_neg(const Fp6& a) { return {fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
TBG_HD Fp6 fp6_reduce(const Fp6& a) { return {fp2_reduce(a.c0), fp2_reduce(a.c1), fp2_reduce(a.c2)}; }
// (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2  (lazy)
TBG_HD Fp6 fp6_mul_v(const Fp6& a) { return {fp2_mul_xi(a.c2), a.c0, a.c1}; }

// Karatsuba (6 Fp2 products). Inputs < 8p, output < 2p.
TBG_NI Fp6 fp6_mul(const Fp6& a, const Fp6& b) {
  Fp2 t0 = fp2_mul(a.c0, b.c0);
  Fp2 t1 = fp2_mul(a.c1, b.c1);
  Fp2 t2 = fp2_mul(a.c2, b.c2);
  Fp2 s12 = fp2_mul(fp2_add_l(a.c1, a.c2), fp2_add(b.c1, b.c2));
  Fp2 s01 = fp2_mul(fp2_add_l(a.c0, a.c1), fp2_add(b.c0, b.c1));
  Fp2 s02 = fp2_mul(fp2_add_l(a.c0, a.c2), fp2_add(b.c0, b.c2));
  Fp2 u = fp2_reduce(fp2_sub_l(s12, fp2_add(t1, t2)));         // < 2p
  Fp2 c0 = fp2_reduce(fp2_add_l(fp2_mul_xi(u), t0));             // t0 + xi(s12 - t1 - t2)
  Fp2 c1 = fp2_reduce(fp2_add_l(fp2_sub_l(s01, fp2_add(t0, t1)), fp2_mul_xi(t2)));
  Fp2 c2 = fp2_reduce(fp2_add_l(fp2_sub_l(s02, fp2_add(t0, t2)), t1));
  return {c0, c1, c2};
}

TBG_HD Fp6 fp6_sqr(const Fp6& a) { return fp6_mul(a, a); }

// a * (b0 + b1 v): 5 Fp2 products.  Inputs < 8p, output < 2p.
TBG_HD Fp6 fp6_mul_by_01(const Fp6& a, const Fp2& b0, const Fp2& b1) {
  Fp2 t0 = fp2_mul(a.c0, b0);
  Fp2 t1 = fp2_mul(a.c1, b1);
  Fp2 s01 = fp2_mul(fp2_add_l(a.c0, a.c1), fp2_add(b0, b1));
  Fp2 a2b1 = fp2_mul(a.c2, b1);
  Fp2 a2b0 = fp2_mul(a.c2, b0);
  Fp2 c0 = fp2_reduce(fp2_add_l(fp2_mul_xi(a2b1), t0));
  Fp2 c1 = fp2_reduce(fp2_sub_l(s01, fp2_add(t0, t1)));
  Fp2 c2 = fp2_reduce(fp2_add_l(t1, a2b0));
  return {c0, c1, c2};
}

// a * (b1 v): 3 Fp2 products.
TBG_HD Fp6 fp6_mul_by_1(const Fp6& a, const Fp2& b1) {
  Fp2 t0 = fp2_mul(a.c2, b1);
  Fp2 t1 = fp2_mul(a.c0, b1);
  Fp2 t2 = fp2_mul(a.c1, b1);
  return {fp2_reduce(fp2_mul_xi(t0)), t1, t2};
}

TBG_NI Fp6 fp6_inv(const Fp6& a) {
  Fp2 c0 = fp2_reduce(fp2_sub(fp2_sqr(a.c0), fp2_reduce(fp2_mul_xi(fp2_mul(a.c1, a.c2)))));
  Fp2 c1 = fp2_reduce(fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1)));
  Fp2 c2 = fp2_reduce(fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2)));
  Fp2 t = fp2_reduce(fp2_add(fp2_mul(a.c0, c0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, c1), fp2_mul(a.c1, c2)))));
  Fp2 ti = fp2_inv(t);
  return {fp2_mul(c0, ti), fp2_mul(c1, ti), fp2_mul(c2, ti)};
}

// ----------------------------------------------------------------- Fp12
TBG_HD Fp12 fp12_one() { return {fp6_one(), fp6_zero()}; }
TBG_HD Fp12 fp12_conj(const Fp12& a) { return {a.c0, fp6_reduce(fp6_neg(a.c1))}; }

// Inputs < 4p, output < 2p.
TBG_NI Fp12 fp12_mul(const Fp12& a, const Fp12& b) {
  Fp6 t0 = fp6_mul(a.c0, b.c0);
  Fp6 t1 = fp6_mul(a.c1, b.c1);
  Fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1));
  Fp6 c1 = fp6_reduce(fp6_sub(s, fp6_add(t0, t1)));
  Fp6 c0 = fp6_reduce(fp6_add(t0, fp6_mul_v(t1)));
  return {c0, c1};
}

// Complex squaring: 2 Fp6 products.
TBG_NI Fp12 fp12_sqr(const Fp12& a) {
  Fp6 t = fp6_mul(a.c0, a.c1);                                   // < 2p
  Fp6 va1 = fp6_reduce(fp6_mul_v(a.c1));
  Fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, va1));      // (a0+a1)(a0+v a1)
  Fp6 tvt = fp6_reduce(fp6_add(t, fp6_mul_v(t)));
  Fp6 c0 = fp6_reduce(fp6_sub(s, tvt));
  Fp6 c1 = fp6_reduce(fp6_add(t, t));
  return {c0, c1};
}

// Squaring in the cyclotomic subgroup (Granger-Scott): three Fp4 squarings,
// 6 Fp2 products instead of 12.  Valid only after the easy part of the final
// exponentiation.  Fp4 pairs: (c0.c0, c1.c1), (c1.c0, c0.c2), (c0.c1, c1.c2).
TBG_HD void fp4_sqr(const Fp2& a, const Fp2& b, Fp2& t0, Fp2& t1) {
  // (a + b y)^2 with y^2 = xi: t0 = a^2 + xi b^2, t1 = 2ab
  Fp2 ab = fp2_mul(a, b);
  Fp2 s = fp2_mul(fp2_add(a, b), fp2_add(a, fp2_mul_xi(b)));   // a^2 + xi b^2 + ab (1 + xi)
  Fp2 u = fp2_reduce(fp2_add(ab, fp2_mul_xi(ab)));
  t0 = fp2_reduce(fp2_sub(s, u));
  t1 = fp2_add(ab, ab);
}

TBG_NI Fp12 fp12_cyc_sqr(const Fp12& f) {
  const Fp2 &z0 = f.c0.c0, &z4 = f.c0.c1, &z3 = f.c0.c2, &z2 = f.c1.c0, &z1 = f.c1.c1, &z5 = f.c1.c2;
  Fp2 t0, t1, t2, t3, t4, t5;
  fp4_sqr(z0, z1, t0, t1);
  fp4_sqr(z2, z3, t2, t3);
  fp4_sqr(z4, z5, t4, t5);
  Fp12 r;
  // c0.c0 = 3 t0 - 2 z0 ; c1.c1 = 3 t1 + 2 z1
  Fp2 a = fp2_sub(t0, z0);
  r.c0.c0 = fp2_reduce(fp2_add(fp2_add(a, a), t0));
  Fp2 b = fp2_add(t1, z1);
  r.c1.c1 = fp2_reduce(fp2_add(fp2_add(b, b), t1));
  // c1.c0 = 3 xi t5 + 2 z2 ; c0.c2 = 3 t4 - 2 z3
  Fp2 x5 = fp2_reduce(fp2_mul_xi(t5));
  Fp2 c = fp2_add(x5, z2);
  r.c1.c0 = fp2_reduce(fp2_add(fp2_add(c, c), x5));
  Fp2 d = fp2_sub(t4, z3);
  r.c0.c2 = fp2_reduce(fp2_add(fp2_add(d, d), t4));
  // c0.c1 = 3 t2 - 2 z4 ; c1.c2 = 3 t3 + 2 z5
  Fp2 e = fp2_sub(t2, z4);
  r.c0.c1 = fp2_reduce(fp2_add(fp2_add(e, e), t2));
  Fp2 g = fp2_add(t3, z5);
  r.c1.c2 = fp2_reduce(fp2_add(fp2_add(g, g), t3));
  return r;
}

// f * (l0 + l1 v + l4 v w): the Miller-loop line (positions 0, 1, 4).
TBG_NI Fp12 fp12_mul_by_014(const Fp12& a, const Fp2& l0, const Fp2& l1, const Fp2& l4) {
  Fp6 t0 = fp6_mul_by_01(a.c0, l0, l1);
  Fp6 t1 = fp6_mul_by_1(a.c1, l4);
  Fp6 s = fp6_mul_by_01(fp6_add(a.c0, a.c1), l0, fp2_add(l1, l4));
  Fp6 c1 = fp6_reduce(fp6_sub(s, fp6_add(t0, t1)));
  Fp6 c0 = fp6_reduce(fp6_add(t0, fp6_mul_v(t1)));
  return {c0, c1};
}

TBG_NI Fp12 fp12_inv(const Fp12& a) {
  Fp6 t = fp6_reduce(fp6_sub(fp6_mul(a.c0, a.c0), fp6_reduce(fp6_mul_v(fp6_mul(a.c1, a.c1)))));
  Fp6 ti = fp6_inv(t);
  return {fp6_mul(a.c0, ti), fp6_reduce(fp6_neg(fp6_mul(a.c1, ti)))};
}

// f^p: conj every Fp2 coefficient and multiply by gamma_k = xi^(k(p-1)/6),
// with f = sum a_k w^k, a_0 = c0.c0, a_1 = c1.c0, a_2 = c0.c1, a_3 = c1.c1,
// a_4 = c0.c2, a_5 = c1.c2.
TBG_NI Fp12 fp12_frob(const Fp12& a) {
  Fp12 r;
  r.c0.c0 = fp2_reduce(fp2_conj(a.c0.c0));
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), fp2_from_const(FROB_G2));
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), fp2_from_const(FROB_G4));
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), fp2_from_const(FROB_G1));
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), fp2_from_const(FROB_G3));
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), fp2_from_const(FROB_G5));
  return r;
}

TBG_HD bool fp12_is_one(const Fp12& a) {
  bool ok = fp_eq(a.c0.c0.c0, fp_one()) && fp_is_zero(a.c0.c0.c1);
  ok = ok && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2);
  ok = ok && fp2_is_zero(a.c1.c0) && fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
  return ok;
}

}  // namespace tbg
