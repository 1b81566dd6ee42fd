// Latency-first Fp12 arithmetic: ONE Fp12 value spread over the lanes of one
// wave, for the single final exponentiation that ends every level-0 launch
// (k_l0_final).  The trio layout of bls_quad.h (three lanes, each owning an
// Fp4 coefficient A_q) is the throughput form -- many independent Fp12
// values, one per trio -- but a lone value on a trio runs its ~330 dependent
// cyclotomic squarings at ~7 Fp products of latency each (5.7 ms per launch,
// VERDICT r02).  Here every Fp2 product of a step gets its own lane PAIR
// (one REDC(a b + c d) per lane, the lane-pair split of bls_pair.h):
//
//   cyclotomic squaring (Granger-Scott over the trio's Fp4 coefficients):
//     12 lanes, one Fp product each: ab and (a + b)(a + xi b) of every A_q;
//   product C = A B (the trio's Karatsuba-3 over Fp4):
//     36 lanes: the three Fp2 products of each of P_q = A_q B_q and
//     Q_q = (A_{q+1} + A_{q+2})(B_{q+1} + B_{q+2});
//   then lanes 0..2 combine exactly as the trio's lane q does (quad_combine /
//   quad_cyc_lane), so the algebra is the one tests/hostcheck already checks
//   against the tower.
//
// State lives in LDS as 12 Fp (A_q = (a.c0, a.c1, b.c0, b.c1) at 4q, the
// trio's HBM order), products in a scratch array; phases are separated by
// barriers of the one-wave workgroup.  A step's latency is one REDC(ab + cd)
// plus the combination, ~4x below the trio's.  The per-phase lane functions
// are plain functions: the host emulates a wave by running the lanes of a
// phase in turn (tests/hostcheck).
#pragma once
#include "bls_quad.h"

namespace tbg {

constexpr int WIDE_FP = 12;   // Fp per wide Fp12 value
constexpr int WIDE_PROD = 36; // scratch Fp of a product step
static const int WIDE_SW12[3] = {0, 2, 1};

TBG_HD Fp2 wide_fp2(const Fp* A, int i) { return {A[i], A[i + 1]}; }
TBG_HD Fp4 wide_fp4(const Fp* A, int q) { return {wide_fp2(A, 4 * q), wide_fp2(A, 4 * q + 2)}; }
TBG_HD void wide_put4(Fp* A, int q, const Fp4& v) {
  A[4 * q] = v.a.c0;
  A[4 * q + 1] = v.a.c1;
  A[4 * q + 2] = v.b.c0;
  A[4 * q + 3] = v.b.c1;
}
// component c of the Fp2 product x y (the lane-pair split: REDC(x0 y0 - x1 y1)
// or REDC(x0 y1 + x1 y0)); inputs < 16p
TBG_HD Fp wide_mul_c(int c, const Fp2& x, const Fp2& y) {
  return c == 0 ? fp_mul2(x.c0, y.c0, x.c1, fp_neg(y.c1)) : fp_mul2(x.c0, y.c1, x.c1, y.c0);
}

// Per-lane choices are per-limb selects (fp_select), never ternaries on
// structs: those compile to selects of addresses and put their operands in
// scratch memory.
TBG_HD Fp2 wide_sel2(bool k, const Fp2& x, const Fp2& y) { return {fp_select(k, x.c0, y.c0), fp_select(k, x.c1, y.c1)}; }
// component j (0, 1) of xi u from u's two components (lazy: < u + 16p)
TBG_HD Fp wide_xi_c(int j, const Fp& u0, const Fp& u1) { return fp_select(j == 0, fp_sub(u0, u1), fp_add(u0, u1)); }

// ---- cyclotomic squaring: products (lanes 0..11), then combination (lanes
// 0..11, one output component each: lane 4 q + k writes component k of A_q)
TBG_HD void wide_cyc_products(int lane, const Fp* A, Fp* R) {
  if (lane >= 12) return;
  const int q = lane >> 2, k = (lane >> 1) & 1, c = lane & 1;
  const Fp2 a = wide_fp2(A, 4 * q), b = wide_fp2(A, 4 * q + 2);
  // fp4_sqr's two products: ab, (a + b)(a + xi b)
  const Fp2 x = wide_sel2(k == 0, a, fp2_add(a, b));
  const Fp2 y = wide_sel2(k == 0, b, fp2_add(a, fp2_mul_xi(b)));
  R[lane] = wide_mul_c(c, x, y);
}
// quad_cyc_lane(q, A_q, T_x), T_x = fp4_sqr(A_x) = {s - (ab + xi ab), 2 ab},
// component k:  s1 = q == 1 ? xi T.b : T.a,  s2 = q == 1 ? T.a : T.b,
//   a = 3 s1 -+ 2 A.a (q == 1: +),  b = 3 s2 +- 2 A.b (q == 1: -)
TBG_HD void wide_cyc_combine(int lane, Fp* A, const Fp* R) {
  if (lane >= 12) return;
  const int q = lane >> 2, k = lane & 3, x = WIDE_SW12[q], j = k & 1;
  const Fp ab0 = R[4 * x], ab1 = R[4 * x + 1];
  const Fp abj = fp_select(j == 0, ab0, ab1);
  const Fp sj = R[4 * x + 2 + j];
  const Fp Taj = fp_reduce(fp_sub(sj, fp_reduce(fp_add(abj, wide_xi_c(j, ab0, ab1)))));  // T.a component j
  const Fp Tb0 = fp_reduce(fp_add(ab0, ab0)), Tb1 = fp_reduce(fp_add(ab1, ab1));
  const Fp Tbj = fp_select(j == 0, Tb0, Tb1);
  const Fp xTbj = fp_reduce(wide_xi_c(j, Tb0, Tb1));
  // s: a components (k < 2) take s1, b components s2
  const Fp sv = k < 2 ? fp_select(q == 1, xTbj, Taj) : fp_select(q == 1, Taj, Tbj);
  const Fp own = A[4 * q + k];
  const bool plus = (k < 2) == (q == 1);  // a: + on q == 1; b: + on q != 1
  const Fp s3 = fp_mul_small(sv, 3), a2 = fp_add(own, own);
  A[4 * q + k] = fp_reduce(fp_select(plus, fp_add(s3, a2), fp_sub(s3, a2)));
}

// ---- product C = X Y: products (lanes 0..35), then combination (lanes
// 0..11, one output component each)
TBG_HD void wide_mul_products(int lane, const Fp* X, const Fp* Y, Fp* R) {
  if (lane >= WIDE_PROD) return;
  const int m = lane / 6, k = (lane % 6) >> 1, c = lane & 1;
  Fp4 x, y;
  if (m < 3) {
    x = wide_fp4(X, m);
    y = wide_fp4(Y, m);
  } else {  // Q_q: the two other coefficients summed
    const int q = m - 3, n1 = (q + 1) % 3, n2 = (q + 2) % 3;
    x = fp4_add(wide_fp4(X, n1), wide_fp4(X, n2));
    y = fp4_add(wide_fp4(Y, n1), wide_fp4(Y, n2));
  }
  // fp4_mul's three Fp2 products: a a', b b', (a + b)(a' + b')
  const Fp2 u = wide_sel2(k == 0, x.a, wide_sel2(k == 1, x.b, fp2_add(x.a, x.b)));
  const Fp2 v = wide_sel2(k == 0, y.a, wide_sel2(k == 1, y.b, fp2_add(y.a, y.b)));
  R[lane] = wide_mul_c(c, u, v);
}
TBG_HD Fp4 wide_fp4_from_products(const Fp* R, int m) {
  const Fp2 t0 = wide_fp2(R, 6 * m), t1 = wide_fp2(R, 6 * m + 2), s = wide_fp2(R, 6 * m + 4);
  return {fp2_reduce(fp2_add(t0, fp2_mul_xi(t1))), fp2_reduce(fp2_sub(s, fp2_add(t0, t1)))};
}
// component i (0..3: a.c0, a.c1, b.c0, b.c1) of product m = fp4 from R
TBG_HD Fp wide_pc(const Fp* R, int m, int i) {
  const int j = i & 1;
  const Fp t0 = R[6 * m + j], t1 = R[6 * m + 2 + j];
  const Fp a = fp_add(t0, wide_xi_c(j, R[6 * m + 2], R[6 * m + 3]));
  const Fp b = fp_sub(R[6 * m + 4 + j], fp_add(t0, t1));
  return fp_reduce(fp_select(i < 2, a, b));
}
// quad_combine(q, P, Pn, Pp, Qx), component k:
//   T = Qx - (f1 + f2), f1 = q == 1 ? Pp : Pn, f2 = q == 0 ? Pp : P
//   q = 0: (xi T.b + P.a, T.a + P.b);  q = 1: (T.a + xi Pn.b, T.b + Pn.a);  q = 2: T + Pp
TBG_HD void wide_mul_combine(int lane, Fp* C, const Fp* R) {
  if (lane >= 12) return;
  const int q = lane >> 2, k = lane & 3, j = k & 1;
  const int mP = q, mn = (q + 1) % 3, mp = (q + 2) % 3, mQ = 3 + WIDE_SW12[q];
  const int m1 = q == 1 ? mp : mn, m2 = q == 0 ? mp : mP;
  auto Tc = [&](int i) { return fp_reduce(fp_sub(wide_pc(R, mQ, i), fp_add(wide_pc(R, m1, i), wide_pc(R, m2, i)))); };
  Fp v;
  if (k < 2) {
    // the xi term: of T.b (q = 0) or Pn.b (q = 1); q = 2 has none
    const Fp u0 = q == 0 ? Tc(2) : wide_pc(R, mn, 2), u1 = q == 0 ? Tc(3) : wide_pc(R, mn, 3);
    const Fp xu = fp_reduce(wide_xi_c(j, u0, u1));
    const Fp t = Tc(k);
    const Fp w = q == 2 ? wide_pc(R, mp, k) : wide_pc(R, mP, k);
    v = fp_select(q == 0, fp_add(xu, w), fp_select(q == 1, fp_add(t, xu), fp_add(t, w)));
  } else {
    // q = 0: T.a_j + P.b_j;  q = 1: T.b_j + Pn.a_j;  q = 2: T.b_j + Pp.b_j
    const Fp t = Tc(q == 0 ? j : k);
    const Fp w = wide_pc(R, q == 0 ? mP : (q == 1 ? mn : mp), q == 1 ? j : k);
    v = fp_add(t, w);
  }
  C[4 * q + k] = fp_reduce(v);
}

// ---- the cheap per-coefficient maps (lanes 0..2) and the inversion (lane 0)
TBG_HD void wide_conj(int lane, Fp* C, const Fp* X) {
  if (lane < 3) wide_put4(C, lane, quad_conj_lane(lane, wide_fp4(X, lane)));
}
TBG_HD void wide_frob(int lane, Fp* C, const Fp* X) {
  if (lane < 3) wide_put4(C, lane, quad_frob_lane(lane, wide_fp4(X, lane)));
}
TBG_HD void wide_copy(int lane, Fp* C, const Fp* X) {
  if (lane < WIDE_FP) C[lane] = X[lane];
}
TBG_HD void wide_one(int lane, Fp* C) {
  if (lane < WIDE_FP) C[lane] = lane == 0 ? fp_one() : fp_zero();
}
// 1 / X through the tower (one lane: the single fp_inv dominates either way)
TBG_HD void wide_inv(int lane, Fp* C, const Fp* X) {
  if (lane != 0) return;
  const Fp12 r = fp12_inv(quad_to_fp12(wide_fp4(X, 0), wide_fp4(X, 1), wide_fp4(X, 2)));
  for (int q = 0; q < 3; ++q) wide_put4(C, q, quad_from_fp12(q, r));
}
TBG_HD bool wide_is_one(const Fp* X) {
  const Fp12 r = quad_to_fp12(wide_fp4(X, 0), wide_fp4(X, 1), wide_fp4(X, 2));
  return fp12_is_one(r);
}

// ---- the final exponentiation f^(3 (p^12 - 1) / r), as quad_final_exp:
// the same sequence of products, cyclotomic squarings, conjugations and
// Frobenius maps, each phase run by `Exec` (a barrier-separated lane phase on
// the device, a loop over 64 lanes on the host).  Slots: 6 wide values.
struct WideSlots {
  Fp v[6][WIDE_FP];
  Fp r[WIDE_PROD];
};

template <class Exec>
TBG_HD void wide_mul_to(Exec& ex, WideSlots& S, int dst, int x, int y) {
  ex([&](int l) { wide_mul_products(l, S.v[x], S.v[y], S.r); });
  ex([&](int l) { wide_mul_combine(l, S.v[dst], S.r); });
}
template <class Exec>
TBG_HD void wide_cyc_sqr(Exec& ex, WideSlots& S, int x) {
  ex([&](int l) { wide_cyc_products(l, S.v[x], S.r); });
  ex([&](int l) { wide_cyc_combine(l, S.v[x], S.r); });
}
// dst = conj(src^|x|) = src^x (cyclotomic); dst != src
template <class Exec>
TBG_HD void wide_pow_x(Exec& ex, WideSlots& S, int dst, int src) {
  ex([&](int l) { wide_copy(l, S.v[dst], S.v[src]); });
  for (int i = 62; i >= 0; --i) {
    wide_cyc_sqr(ex, S, dst);
    if ((X_ABS >> i) & 1) wide_mul_to(ex, S, dst, dst, src);
  }
  ex([&](int l) { wide_conj(l, S.v[dst], S.v[dst]); });
}
// S.v[0] <- FE(S.v[0]); uses slots 1..5
template <class Exec>
TBG_HD void wide_final_exp(Exec& ex, WideSlots& S) {
  enum { F = 0, T = 1, A = 2, B = 3, C = 4, U = 5 };
  ex([&](int l) { wide_inv(l, S.v[U], S.v[F]); });
  ex([&](int l) { wide_conj(l, S.v[T], S.v[F]); });
  wide_mul_to(ex, S, T, T, U);                                   // t = conj(f) / f
  ex([&](int l) { wide_frob(l, S.v[U], S.v[T]); });
  ex([&](int l) { wide_frob(l, S.v[U], S.v[U]); });
  wide_mul_to(ex, S, T, U, T);                                   // t = frob^2(t) t
  wide_pow_x(ex, S, A, T);
  ex([&](int l) { wide_conj(l, S.v[U], S.v[T]); });
  wide_mul_to(ex, S, A, A, U);                                   // a = t^x conj(t)
  wide_pow_x(ex, S, B, A);
  ex([&](int l) { wide_conj(l, S.v[U], S.v[A]); });
  wide_mul_to(ex, S, A, B, U);                                   // a = a^x conj(a)
  wide_pow_x(ex, S, B, A);
  ex([&](int l) { wide_frob(l, S.v[U], S.v[A]); });
  wide_mul_to(ex, S, B, B, U);                                   // b = a^x frob(a)
  wide_pow_x(ex, S, C, B);
  wide_pow_x(ex, S, A, C);                                       // (b^x)^x
  ex([&](int l) { wide_frob(l, S.v[U], S.v[B]); });
  ex([&](int l) { wide_frob(l, S.v[U], S.v[U]); });
  wide_mul_to(ex, S, C, A, U);                                   // c = b^(x^2) frob^2(b)
  ex([&](int l) { wide_conj(l, S.v[U], S.v[B]); });
  wide_mul_to(ex, S, C, C, U);                                   // c = c conj(b)
  ex([&](int l) { wide_copy(l, S.v[U], S.v[T]); });
  wide_cyc_sqr(ex, S, U);
  wide_mul_to(ex, S, U, U, T);                                   // t3 = cyc(t) t
  wide_mul_to(ex, S, F, C, U);                                   // FE = c t3
}

// host: a wave is its 64 lanes run in turn, phase by phase
struct WideHostExec {
  template <class Fn>
  void operator()(Fn&& fn) {
    for (int l = 0; l < 64; ++l) fn(l);
  }
};

}  // namespace tbg
