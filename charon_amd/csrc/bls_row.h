// Row Fp: ONE field element per 16-lane DPP row, limb j on lane j (j < 14;
// lanes 14 and 15 hold 0) -- the latency form of the field, for the single
// final exponentiation that ends every level-0 launch (k_l0_final).
//
// Why: a Montgomery product on one lane is a ~490-instruction dependent
// chain (1.19 us on gfx950, profiles/r03/fp_acc.txt).  On a row each lane
// runs the operand-scanning (CIOS) loop for its own limb column: per limb
// a_i of a, broadcast over the row, t_j += a_i b_j, then m = t_0 NINV (t_0
// broadcast from lane 0), t_j += m p_j and a one-lane shift down -- 14
// steps of a few instructions each.  Limbs are SIGNED redundant 32-bit
// values (value = sum_j l_j 2^(28 j), |l_j| <= 2^29): sums and differences
// are lane-local, carries move one lane per round (three rounds normalise),
// and no subtraction needs a multiple of p added first.
//
// The same source runs on the device (RowV holds this lane's value; the
// exchanges are ds_swizzle broadcasts and DPP row shifts) and on the host
// (RowV holds the whole row; the exchanges index the array), so
// tests/hostcheck runs the row algorithms themselves against the oracle.
#pragma once
#include "bls_quad.h"

namespace tbg {

#if defined(__HIP_DEVICE_COMPILE__)
constexpr int ROW_N = 1;  // this lane's value
#else
constexpr int ROW_N = 16;  // the whole row
#endif

template <class T>
struct RowV {
  T v[ROW_N];
};
using R32 = RowV<int32_t>;
using R64 = RowV<int64_t>;

template <class T, class F>
TBG_HD RowV<T> rmap(F&& f) {
  RowV<T> r;
#pragma unroll
  for (int k = 0; k < ROW_N; ++k) r.v[k] = f(k);
  return r;
}
// this lane's position in its row
TBG_HD R32 r_lane() {
#if defined(__HIP_DEVICE_COMPILE__)
  return {{(int32_t)(threadIdx.x & 15u)}};
#else
  return rmap<int32_t>([](int k) { return (int32_t)k; });
#endif
}
// per-lane table entry (limb j of a constant; 0 on lanes 14, 15)
TBG_HD R32 r_limbs(const uint32_t (&c)[NL]) {
  const R32 j = r_lane();
  return rmap<int32_t>([&](int k) { return j.v[k] < NL ? (int32_t)c[j.v[k]] : 0; });
}
TBG_HD R32 r_splat(int32_t x) { return rmap<int32_t>([&](int) { return x; }); }
TBG_HD R64 r_wide(const R32& a) { return rmap<int64_t>([&](int k) { return (int64_t)a.v[k]; }); }
TBG_HD R32 r_lo(const R64& a) { return rmap<int32_t>([&](int k) { return (int32_t)(uint32_t)a.v[k]; }); }
TBG_HD R32 operator+(const R32& a, const R32& b) { return rmap<int32_t>([&](int k) { return a.v[k] + b.v[k]; }); }
TBG_HD R32 operator-(const R32& a, const R32& b) { return rmap<int32_t>([&](int k) { return a.v[k] - b.v[k]; }); }
TBG_HD R32 operator-(const R32& a) { return rmap<int32_t>([&](int k) { return -a.v[k]; }); }
TBG_HD R32 r_mul_small(const R32& a, int32_t s) { return rmap<int32_t>([&](int k) { return a.v[k] * s; }); }
TBG_HD R64 operator+(const R64& a, const R64& b) { return rmap<int64_t>([&](int k) { return a.v[k] + b.v[k]; }); }
// acc + a b (signed 32 x 32 -> 64)
TBG_HD R64 r_mad(const R64& acc, const R32& a, const R32& b) {
  return rmap<int64_t>([&](int k) { return acc.v[k] + (int64_t)a.v[k] * (int64_t)b.v[k]; });
}
TBG_HD R32 r_sel(bool c, const R32& a, const R32& b) { return c ? a : b; }  // row-uniform choices only
TBG_HD R32 r_sel_lane(const R32& c, const R32& a, const R32& b) {
  return rmap<int32_t>([&](int k) { return c.v[k] ? a.v[k] : b.v[k]; });
}

// ---- row exchanges
// lane S's value on every lane of the row (ds_swizzle bitmask mode within
// 32-lane groups: and 0x10 keeps the row, or S picks the lane)
template <int S>
TBG_HD R32 r_bcast(const R32& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return {{__builtin_amdgcn_ds_swizzle(a.v[0], 0x10 | (S << 5))}};
#else
  return r_splat(a.v[S]);
#endif
}
// lane j reads lane j + 1 (lane 15 reads 0): DPP row_shl:1
TBG_HD R32 r_down(const R32& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return {{__builtin_amdgcn_update_dpp(0, a.v[0], 0x101, 0xf, 0xf, true)}};
#else
  return rmap<int32_t>([&](int k) { return k < 15 ? a.v[k + 1] : 0; });
#endif
}
// lane j reads lane j - 1 (lane 0 reads 0): DPP row_shr:1
TBG_HD R32 r_up(const R32& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return {{__builtin_amdgcn_update_dpp(0, a.v[0], 0x111, 0xf, 0xf, true)}};
#else
  return rmap<int32_t>([&](int k) { return k > 0 ? a.v[k - 1] : 0; });
#endif
}
TBG_HD R64 r_down64(const R64& a) {
  const R32 lo = rmap<int32_t>([&](int k) { return (int32_t)(uint32_t)a.v[k]; });
  const R32 hi = rmap<int32_t>([&](int k) { return (int32_t)(uint32_t)((uint64_t)a.v[k] >> 32); });
  const R32 dl = r_down(lo), dh = r_down(hi);
  return rmap<int64_t>([&](int k) { return (int64_t)(((uint64_t)(uint32_t)dh.v[k] << 32) | (uint32_t)dl.v[k]); });
}
TBG_HD R64 r_up64(const R64& a) {
  const R32 lo = rmap<int32_t>([&](int k) { return (int32_t)(uint32_t)a.v[k]; });
  const R32 hi = rmap<int32_t>([&](int k) { return (int32_t)(uint32_t)((uint64_t)a.v[k] >> 32); });
  const R32 ul = r_up(lo), uh = r_up(hi);
  return rmap<int64_t>([&](int k) { return (int64_t)(((uint64_t)(uint32_t)uh.v[k] << 32) | (uint32_t)ul.v[k]); });
}

// ---- carries: three rounds of "keep 28 bits, pass the rest one lane up"
// (arithmetic shifts: signed limbs).  Lane 13 keeps its whole value (the
// top limb carries the excess); lanes 14, 15 stay 0.  A round of 64-bit
// columns below 2^63 leaves |limb| < 2^28 + 2^36, the next < 2^28 + 2^9,
// the third <= 2^28 in magnitude.
TBG_HD R32 r_carry32(const R32& a) {
  const R32 j = r_lane();
  const R32 c = rmap<int32_t>([&](int k) { return j.v[k] < NL - 1 ? (a.v[k] >> 28) : 0; });
  const R32 l = rmap<int32_t>([&](int k) { return j.v[k] < NL - 1 ? (a.v[k] & (int32_t)LMASK) : a.v[k]; });
  return l + r_up(c);
}
TBG_HD R32 r_norm64(const R64& t) {
  const R32 j = r_lane();
  const R64 c = rmap<int64_t>([&](int k) { return j.v[k] < NL - 1 ? (t.v[k] >> 28) : 0; });
  const R64 l = rmap<int64_t>([&](int k) { return j.v[k] < NL - 1 ? (t.v[k] & (int64_t)LMASK) : t.v[k]; });
  const R64 s = l + r_up64(c);  // |s| < 2^28 + 2^36 (lane 13: the top, < 2^62)
  const R64 c2 = rmap<int64_t>([&](int k) { return j.v[k] < NL - 1 ? (s.v[k] >> 28) : 0; });
  const R64 l2 = rmap<int64_t>([&](int k) { return j.v[k] < NL - 1 ? (s.v[k] & (int64_t)LMASK) : s.v[k]; });
  const R64 s2 = l2 + r_up64(c2);
  return r_carry32(r_lo(s2));
}
TBG_HD R32 r_norm(const R32& a) { return r_carry32(r_carry32(a)); }

// ---- REDC(sum_k a_k b_k) over the row (K <= 2; |limbs| <= 2^29: the
// 64-bit lane columns stay below 14 (2 * 2^58 + 2^56) < 2^63).  The value
// is (sum a_k b_k + m p) / 2^392: for |a_k b_k| < 2^11 p^2 it lies in
// (-p, 2p) -- signed, as every row value may be.
template <int K>
TBG_HD R32 row_mul_sum(const R32 (&a)[K], const R32 (&b)[K]) {
  const R32 pj = r_limbs(P_L);
  const R32 j = r_lane();
  R64 t = rmap<int64_t>([](int) { return (int64_t)0; });
  auto step = [&](const R32 (&ai)[K]) {
#pragma unroll
    for (int n = 0; n < K; ++n) t = r_mad(t, ai[n], b[n]);
    const R32 t0 = r_bcast<0>(r_lo(t));
    const R32 m = rmap<int32_t>([&](int k) { return (int32_t)(((uint32_t)t0.v[k] * NINV) & LMASK); });
    t = r_mad(t, m, pj);
    // t / 2^28: lane j takes lane j + 1's column, lane 0 adds its own carry
    const R64 sh = r_down64(t);
    t = rmap<int64_t>([&](int k) { return sh.v[k] + (j.v[k] == 0 ? (t.v[k] >> 28) : 0); });
  };
#define TBG_ROW_STEP(I)                                      \
  {                                                          \
    R32 ai[K];                                               \
    _Pragma("unroll") for (int n = 0; n < K; ++n) ai[n] = r_bcast<I>(a[n]); \
    step(ai);                                                \
  }
  TBG_ROW_STEP(0) TBG_ROW_STEP(1) TBG_ROW_STEP(2) TBG_ROW_STEP(3) TBG_ROW_STEP(4) TBG_ROW_STEP(5)
  TBG_ROW_STEP(6) TBG_ROW_STEP(7) TBG_ROW_STEP(8) TBG_ROW_STEP(9) TBG_ROW_STEP(10) TBG_ROW_STEP(11)
  TBG_ROW_STEP(12) TBG_ROW_STEP(13)
#undef TBG_ROW_STEP
  return r_norm64(t);
}
TBG_HD R32 row_mul(const R32& a, const R32& b) {
  const R32 A[1] = {a}, B[1] = {b};
  return row_mul_sum<1>(A, B);
}
TBG_HD R32 row_mul2(const R32& a, const R32& b, const R32& c, const R32& d) {
  const R32 A[2] = {a, c}, B[2] = {b, d};
  return row_mul_sum<2>(A, B);
}

// x - q p with q from the top limbs (as fp_reduce): a normalised row value of
// magnitude < 2^389 comes back in (-p, 2p)
TBG_HD R32 row_reduce(const R32& a) {
  const R32 x13 = r_bcast<13>(a), x12 = r_bcast<12>(a), x11 = r_bcast<11>(a);
  const R32 pj = r_limbs(P_L);
  const R64 t = rmap<int64_t>([&](int k) {
    // a >> 330 from the top limbs (signed; limbs 11, 12 within +-2^28)
    const double top = (double)x13.v[k] * 17179869184.0 + (double)x12.v[k] * 64.0 + (double)(x11.v[k] >> 22);
    const double qd = top * INV_PT;
    const int64_t q = (int64_t)(qd < 0.0 ? qd - 1.0 : qd);  // floor, |q| < 2^31
    return (int64_t)a.v[k] - q * (int64_t)pj.v[k];
  });
  return r_norm64(t);
}

// ---- a row value from / to the plain limb form (the quad layout's Fp)
TBG_HD R32 row_from_limbs(const uint32_t* l) {
  const R32 j = r_lane();
  return rmap<int32_t>([&](int k) { return j.v[k] < NL ? (int32_t)l[j.v[k]] : 0; });
}

// A signed row value (|value| < 8p, |limbs| < 2^31) as a plain Fp in [0, 2p)
// -- one lane's sequential carry pass (the rare gathers: inversion, test)
TBG_HD Fp fp_from_signed(const int32_t* l) {
  Fp r;
  int64_t carry = 0;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    // + 16p (SUB16P_L: every limb but the top >= 2^28 - 1, value 16p)
    const int64_t v = (int64_t)l[j] + (int64_t)SUB16P_L[j] + carry;
    if (j < NL - 1) {
      r.l[j] = (uint32_t)(v & (int64_t)LMASK);
      carry = v >> 28;
    } else {
      r.l[j] = (uint32_t)v;
    }
  }
  return fp_reduce(r);
}

// ---------------------------------------------------------------------------
// Fp12 on rows: the 12 Fp of the trio's quad order (A_q = (a.c0, a.c1, b.c0,
// b.c1) at 4 q, as bls_wide.h) on 12 rows, products on up to 36 rows.  Row
// values live in LDS as 16 words (lane j reads word j: conflict-free); the
// phases are the wide value's (bls_wide.h) with a ROW per lane there, and
// every row of a wave runs the same instructions (row roles by selects, not
// branches: rows of one wave would otherwise serialise).
constexpr int RW_FP = 12, RW_PROD = 36;
using RowMem = int32_t (*)[16];
using RowCMem = const int32_t (*)[16];

TBG_HD R32 row_ld(const int32_t* s) {
#if defined(__HIP_DEVICE_COMPILE__)
  return {{s[threadIdx.x & 15u]}};
#else
  return rmap<int32_t>([&](int k) { return s[k]; });
#endif
}
TBG_HD void row_st(int32_t* s, const R32& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  s[threadIdx.x & 15u] = a.v[0];
#else
  for (int k = 0; k < 16; ++k) s[k] = a.v[k];
#endif
}
TBG_HD R32 rsel(bool c, const R32& a, const R32& b) {
  return rmap<int32_t>([&](int k) { return c ? a.v[k] : b.v[k]; });
}
// component j of xi u = (u0 - u1) + (u0 + u1) i
TBG_HD R32 row_xi(int j, const R32& u0, const R32& u1) { return rsel(j == 0, u0 - u1, u0 + u1); }
// component c of the Fp2 product x y: REDC(x0 y0 - x1 y1) or REDC(x0 y1 + x1 y0)
TBG_HD R32 row_fp2_mul_c(int c, const R32& x0, const R32& x1, const R32& y0, const R32& y1) {
  return row_mul2(x0, rsel(c == 0, y0, y1), x1, rsel(c == 0, -y1, y0));
}

// ---- cyclotomic squaring (wide_cyc_products / wide_cyc_combine)
TBG_HD void row_cyc_products(int r, RowCMem A, RowMem R) {
  if (r >= 12) return;
  const int q = r >> 2, k = (r >> 1) & 1, c = r & 1;
  const R32 a0 = row_ld(A[4 * q]), a1 = row_ld(A[4 * q + 1]), b0 = row_ld(A[4 * q + 2]), b1 = row_ld(A[4 * q + 3]);
  // fp4_sqr's two products: ab, (a + b)(a + xi b)
  const R32 x0 = rsel(k == 0, a0, a0 + b0), x1 = rsel(k == 0, a1, a1 + b1);
  const R32 y0 = rsel(k == 0, b0, r_norm(a0 + b0 - b1)), y1 = rsel(k == 0, b1, r_norm(a1 + b0 + b1));
  row_st(R[r], row_fp2_mul_c(c, x0, x1, y0, y1));
}
TBG_HD void row_cyc_combine(int r, RowMem A, RowCMem R) {
  if (r >= 12) return;
  const int q = r >> 2, k = r & 3, x = q == 0 ? 0 : 3 - q, j = k & 1;
  const R32 ab0 = row_ld(R[4 * x]), ab1 = row_ld(R[4 * x + 1]);
  const R32 abj = rsel(j == 0, ab0, ab1), sj = row_ld(R[4 * x + 2 + j]);
  const R32 Taj = sj - abj - row_xi(j, ab0, ab1);             // T.a component j
  const R32 Tbj = r_mul_small(abj, 2);                         // T.b = 2 ab
  const R32 xTbj = r_mul_small(row_xi(j, ab0, ab1), 2);        // xi T.b
  const R32 sv = r_norm(rsel(k < 2, rsel(q == 1, xTbj, Taj), rsel(q == 1, Taj, Tbj)));
  const R32 own = row_ld(A[4 * q + k]);
  const bool plus = (k < 2) == (q == 1);
  const R32 s3 = r_mul_small(sv, 3), a2 = r_mul_small(own, 2);
  row_st(A[4 * q + k], row_reduce(rsel(plus, s3 + a2, s3 - a2)));
}

// ---- product C = X Y (wide_mul_products / wide_mul_combine), the
// combination in two phases: the six Fp4 products' components, then C
struct RowSlots {
  int32_t v[6][RW_FP][16];
  int32_t r[RW_PROD][16];
  int32_t pc[24][16];
};
TBG_HD void row_mul_products(int r, RowCMem X, RowCMem Y, RowMem R) {
  if (r >= RW_PROD) return;
  const int m = r / 6, k = (r % 6) >> 1, c = r & 1;
  const int q = m < 3 ? m : m - 3, i1 = m < 3 ? m : (q + 1) % 3, i2 = (q + 2) % 3;
  const bool two = m >= 3;
  R32 x[4], y[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const R32 z = r_splat(0);
    x[t] = row_ld(X[4 * i1 + t]) + rsel(two, row_ld(X[4 * i2 + t]), z);
    y[t] = row_ld(Y[4 * i1 + t]) + rsel(two, row_ld(Y[4 * i2 + t]), z);
  }
  // fp4_mul's three Fp2 products: a a', b b', (a + b)(a' + b')
  const R32 u0 = r_norm(rsel(k == 0, x[0], rsel(k == 1, x[2], x[0] + x[2])));
  const R32 u1 = r_norm(rsel(k == 0, x[1], rsel(k == 1, x[3], x[1] + x[3])));
  const R32 v0 = r_norm(rsel(k == 0, y[0], rsel(k == 1, y[2], y[0] + y[2])));
  const R32 v1 = r_norm(rsel(k == 0, y[1], rsel(k == 1, y[3], y[1] + y[3])));
  row_st(R[r], row_fp2_mul_c(c, u0, u1, v0, v1));
}
// component i (a.c0, a.c1, b.c0, b.c1) of Fp4 product m from R: t0 + xi t1, s - t0 - t1
TBG_HD void row_mul_pc(int r, RowCMem R, RowMem PC) {
  if (r >= 24) return;
  const int m = r >> 2, i = r & 3, j = i & 1;
  const R32 t0 = row_ld(R[6 * m + j]), t1 = row_ld(R[6 * m + 2 + j]), sj = row_ld(R[6 * m + 4 + j]);
  const R32 xt1 = row_xi(j, row_ld(R[6 * m + 2]), row_ld(R[6 * m + 3]));
  row_st(PC[r], r_norm(rsel(i < 2, t0 + xt1, sj - t0 - t1)));
}
// quad_combine(q, P, Pn, Pp, Qx), component k (see wide_mul_combine)
TBG_HD void row_mul_combine(int r, RowMem C, RowCMem PC) {
  if (r >= 12) return;
  const int q = r >> 2, k = r & 3, j = k & 1;
  const int mP = q, mn = (q + 1) % 3, mp = (q + 2) % 3, mQ = 3 + (q == 0 ? 0 : 3 - q);
  const int m1 = q == 1 ? mp : mn, m2 = q == 0 ? mp : mP;
  auto pc = [&](int m, int i) { return row_ld(PC[4 * m + i]); };
  auto Tc = [&](int i) { return r_norm(pc(mQ, i) - pc(m1, i) - pc(m2, i)); };
  // k < 2: the xi term -- of T.b (q = 0) or Pn.b (q = 1); q = 2 has none
  const R32 u0 = rsel(q == 0, Tc(2), pc(mn, 2)), u1 = rsel(q == 0, Tc(3), pc(mn, 3));
  const R32 xu = row_xi(j, u0, u1);
  const R32 lo_t = Tc(k < 2 ? k : j);
  const R32 lo_w = rsel(q == 2, pc(mp, k < 2 ? k : j), pc(mP, k < 2 ? k : j));
  const R32 lo = rsel(q == 0, xu + lo_w, rsel(q == 1, lo_t + xu, lo_t + lo_w));
  // k >= 2: q = 0: T.a_j + P.b_j;  q = 1: T.b_j + Pn.a_j;  q = 2: T.b_j + Pp.b_j
  const R32 hi_t = Tc(q == 0 ? j : (k < 2 ? k + 2 : k));
  const R32 hi_w = pc(q == 0 ? mP : (q == 1 ? mn : mp), q == 1 ? j : (k < 2 ? k + 2 : k));
  row_st(C[4 * q + k], row_reduce(rsel(k < 2, lo, hi_t + hi_w)));
}

// ---- the cheap maps (conj, Frobenius) and the gathered inversion
TBG_HD void row_conj(int r, RowMem C, RowCMem X) {
  if (r >= 12) return;
  const int q = r >> 2, k = r & 3;
  const bool neg = q == 1 ? k < 2 : k >= 2;
  const R32 x = row_ld(X[r]);
  row_st(C[r], rsel(neg, -x, x));
}
// (C != X: row r reads its partner component's row)
TBG_HD void row_frob(int r, RowMem C, RowCMem X) {
  if (r >= 12) return;
  const int q = r >> 2, k = r & 3, kk = k >> 1, c = k & 1;
  const R32 x0 = row_ld(X[4 * q + 2 * kk]), x1 = row_ld(X[4 * q + 2 * kk + 1]);
  // gamma of coefficient (q, kk): a_0 -> 1, a_1 -> G1, a_2 -> G2, a_3 -> G3, a_4 -> G4, a_5 -> G5
  const int g = kk == 0 ? q : q + 3;
  const R32 z = r_splat(0);
  const R32 g0 = rsel(g == 0, r_limbs(ONE_M), rsel(g == 1, r_limbs(FROB_G1.c0), rsel(g == 2, r_limbs(FROB_G2.c0),
                 rsel(g == 3, r_limbs(FROB_G3.c0), rsel(g == 4, r_limbs(FROB_G4.c0), r_limbs(FROB_G5.c0))))));
  const R32 g1 = rsel(g == 0, z, rsel(g == 1, r_limbs(FROB_G1.c1), rsel(g == 2, r_limbs(FROB_G2.c1),
                 rsel(g == 3, r_limbs(FROB_G3.c1), rsel(g == 4, r_limbs(FROB_G4.c1), r_limbs(FROB_G5.c1))))));
  // conj(x) gamma: c0 = x0 g0 + x1 g1, c1 = x0 g1 - x1 g0
  row_st(C[r], row_mul2(x0, rsel(c == 0, g0, g1), x1, rsel(c == 0, g1, -g0)));
}
TBG_HD void row_copy(int r, RowMem C, RowCMem X) {
  if (r < 12) row_st(C[r], row_ld(X[r]));
}
// the element gathered on one thread (plain Fp), and back
TBG_HD Fp12 row_gather(RowCMem X) {
  Fp4 A[3];
  for (int q = 0; q < 3; ++q) {
    A[q].a.c0 = fp_from_signed(X[4 * q]);
    A[q].a.c1 = fp_from_signed(X[4 * q + 1]);
    A[q].b.c0 = fp_from_signed(X[4 * q + 2]);
    A[q].b.c1 = fp_from_signed(X[4 * q + 3]);
  }
  return quad_to_fp12(A[0], A[1], A[2]);
}
TBG_HD void row_scatter(RowMem C, const Fp12& f) {
  for (int q = 0; q < 3; ++q) {
    const Fp4 A = quad_from_fp12(q, f);
    const Fp* v[4] = {&A.a.c0, &A.a.c1, &A.b.c0, &A.b.c1};
    for (int k = 0; k < 4; ++k)
      for (int j = 0; j < 16; ++j) C[4 * q + k][j] = j < NL ? (int32_t)v[k]->l[j] : 0;
  }
}
TBG_HD bool row_is_one(RowCMem X) { return fp12_is_one(row_gather(X)); }

// ---- the final exponentiation f^(3 (p^12 - 1) / r) in wide_final_exp's
// sequence; `Exec` runs a row phase on every row (device: rows of the
// workgroup, then a barrier; host: rows in turn) and `Solo` one thread's
// step (the gathered inversion).
template <class Exec>
TBG_HD void row_mul_to(Exec& ex, RowSlots& S, int dst, int x, int y) {
  ex([&](int r) { row_mul_products(r, S.v[x], S.v[y], S.r); });
  ex([&](int r) { row_mul_pc(r, S.r, S.pc); });
  ex([&](int r) { row_mul_combine(r, S.v[dst], S.pc); });
}
template <class Exec>
TBG_HD void row_cyc_sqr(Exec& ex, RowSlots& S, int x) {
  ex([&](int r) { row_cyc_products(r, S.v[x], S.r); });
  ex([&](int r) { row_cyc_combine(r, S.v[x], S.r); });
}
template <class Exec>
TBG_HD void row_pow_x(Exec& ex, RowSlots& S, int dst, int src) {
  ex([&](int r) { row_copy(r, S.v[dst], S.v[src]); });
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    row_cyc_sqr(ex, S, dst);
    if ((X_ABS >> i) & 1) row_mul_to(ex, S, dst, dst, src);
  }
  ex([&](int r) { row_conj(r, S.v[dst], S.v[dst]); });
}
// S.v[0] <- FE(S.v[0]) given S.v[5] = S.v[0]^-1; uses slots 1..5
template <class Exec>
TBG_HD void row_final_exp_inv(Exec& ex, RowSlots& S) {
  enum { F = 0, T = 1, A = 2, B = 3, C = 4, U = 5 };
  ex([&](int r) { row_conj(r, S.v[T], S.v[F]); });
  row_mul_to(ex, S, T, T, U);                                    // t = conj(f) / f
  ex([&](int r) { row_frob(r, S.v[A], S.v[T]); });              // (Frobenius out of place: a row
  ex([&](int r) { row_frob(r, S.v[U], S.v[A]); });              //  reads its partner component)
  row_mul_to(ex, S, T, U, T);                                    // t = frob^2(t) t
  row_pow_x(ex, S, A, T);
  ex([&](int r) { row_conj(r, S.v[U], S.v[T]); });
  row_mul_to(ex, S, A, A, U);                                    // a = t^x conj(t)
  row_pow_x(ex, S, B, A);
  ex([&](int r) { row_conj(r, S.v[U], S.v[A]); });
  row_mul_to(ex, S, A, B, U);                                    // a = a^x conj(a)
  row_pow_x(ex, S, B, A);
  ex([&](int r) { row_frob(r, S.v[U], S.v[A]); });
  row_mul_to(ex, S, B, B, U);                                    // b = a^x frob(a)
  row_pow_x(ex, S, C, B);
  row_pow_x(ex, S, A, C);                                        // (b^x)^x
  ex([&](int r) { row_frob(r, S.v[F], S.v[B]); });              // (F is free until the last product)
  ex([&](int r) { row_frob(r, S.v[U], S.v[F]); });
  row_mul_to(ex, S, C, A, U);                                    // c = b^(x^2) frob^2(b)
  ex([&](int r) { row_conj(r, S.v[U], S.v[B]); });
  row_mul_to(ex, S, C, C, U);                                    // c = c conj(b)
  ex([&](int r) { row_copy(r, S.v[U], S.v[T]); });
  row_cyc_sqr(ex, S, U);
  row_mul_to(ex, S, U, U, T);                                    // t3 = cyc(t) t
  row_mul_to(ex, S, F, C, U);                                    // FE = c t3
}
template <class Exec, class Solo>
TBG_HD void row_final_exp(Exec& ex, Solo& solo, RowSlots& S) {
  solo([&]() { row_scatter(S.v[5], fp12_inv(row_gather(S.v[0]))); });
  row_final_exp_inv(ex, S);
}

#if defined(__HIP__)
// device: a row phase on every row of the workgroup, then a barrier
struct RowDevExec {
  template <class Fn>
  __device__ void operator()(Fn&& fn) {
    fn((int)(threadIdx.x >> 4));
    __syncthreads();
  }
};
#endif

// ---------------------------------------------------------------------------
// Miller lines of ONE G2 point on rows (level 0's batch-wide S, -g1 folded
// in: the serial step of every level-0 launch between the bucket MSM and the
// Miller products).  T = (X, Y, Z) and Q = (x, y) are ten row values; every
// doubling is three product phases and a combination, every addition five
// and a combination (miller_dbl_g / miller_add_g's formulas, the Fp2
// products of a phase on two rows each: c0 and c1).
struct RowLineSlots {
  int32_t s[10][16];      // X0 X1 Y0 Y1 Z0 Z1 | x0 x1 y0 y1
  int32_t p[5][12][16];   // the phases' products
  int32_t k[2][16];       // nxP, yP
  int32_t l[2][6][16];    // finished lines (l0, l1, l4), double-buffered
};
enum { RL_X = 0, RL_Y = 2, RL_Z = 4, RL_QX = 6, RL_QY = 8 };
TBG_HD R32 rl_ld(const RowLineSlots& S, int i) { return row_ld(S.s[i]); }
TBG_HD R32 rl_p(const RowLineSlots& S, int ph, int i) { return row_ld(S.p[ph][i]); }
// product job: rows 2 j (c0) and 2 j + 1 (c1) of the Fp2 product a b
TBG_HD void rl_job(RowLineSlots& S, int ph, int r, const R32& a0, const R32& a1, const R32& b0, const R32& b1) {
  row_st(S.p[ph][r], row_fp2_mul_c(r & 1, a0, a1, b0, b1));
}

// ---- doubling T <- 2T and its line
TBG_HD void rl_dbl1(int r, RowLineSlots& S) {  // A = X^2, B = Y^2, ZZ = Z^2, YZ = Y Z
  if (r >= 8) return;
  const int j = r >> 1;
  const int ia = j == 0 ? RL_X : (j == 1 ? RL_Y : (j == 2 ? RL_Z : RL_Y));
  const int ib = j == 0 ? RL_X : (j == 1 ? RL_Y : RL_Z);
  rl_job(S, 0, r, rl_ld(S, ia), rl_ld(S, ia + 1), rl_ld(S, ib), rl_ld(S, ib + 1));
}
TBG_HD void rl_dbl2(int r, RowLineSlots& S) {  // C = B^2, (X + B)^2, F = E^2, X E, ZZ E, 2 YZ ZZ;  E = 3A
  if (r >= 12) return;
  const int j = r >> 1;
  const R32 E0 = r_norm(r_mul_small(rl_p(S, 0, 0), 3)), E1 = r_norm(r_mul_small(rl_p(S, 0, 1), 3));
  R32 a0, a1, b0, b1;
  if (j == 0) { a0 = b0 = rl_p(S, 0, 2); a1 = b1 = rl_p(S, 0, 3); }
  else if (j == 1) { a0 = b0 = rl_ld(S, RL_X) + rl_p(S, 0, 2); a1 = b1 = rl_ld(S, RL_X + 1) + rl_p(S, 0, 3); }
  else if (j == 2) { a0 = b0 = E0; a1 = b1 = E1; }
  else if (j == 3) { a0 = rl_ld(S, RL_X); a1 = rl_ld(S, RL_X + 1); b0 = E0; b1 = E1; }
  else if (j == 4) { a0 = rl_p(S, 0, 4); a1 = rl_p(S, 0, 5); b0 = E0; b1 = E1; }
  else { a0 = r_mul_small(rl_p(S, 0, 6), 2); a1 = r_mul_small(rl_p(S, 0, 7), 2); b0 = rl_p(S, 0, 4); b1 = rl_p(S, 0, 5); }
  rl_job(S, 1, r, a0, a1, b0, b1);
}
// D = 2((X + B)^2 - A - C), X3 = F - 2D (component c)
TBG_HD R32 rl_D(const RowLineSlots& S, int c) {
  return r_norm(r_mul_small(rl_p(S, 1, 2 + c) - rl_p(S, 0, c) - rl_p(S, 1, c), 2));
}
TBG_HD R32 rl_X3(const RowLineSlots& S, int c) { return r_norm(rl_p(S, 1, 4 + c) - r_mul_small(rl_D(S, c), 2)); }
TBG_HD void rl_dbl3(int r, RowLineSlots& S) {  // (D - X3) E, l1 = ZZ E nxP, l4 = 2 YZ ZZ yP
  if (r >= 6) return;
  const int j = r >> 1;
  R32 a0, a1, b0, b1;
  const R32 z = r_splat(0);
  if (j == 0) {
    a0 = r_norm(rl_D(S, 0) - rl_X3(S, 0));
    a1 = r_norm(rl_D(S, 1) - rl_X3(S, 1));
    b0 = r_norm(r_mul_small(rl_p(S, 0, 0), 3));
    b1 = r_norm(r_mul_small(rl_p(S, 0, 1), 3));
  } else if (j == 1) { a0 = rl_p(S, 1, 8); a1 = rl_p(S, 1, 9); b0 = row_ld(S.k[0]); b1 = z; }
  else { a0 = rl_p(S, 1, 10); a1 = rl_p(S, 1, 11); b0 = row_ld(S.k[1]); b1 = z; }
  rl_job(S, 2, r, a0, a1, b0, b1);
}
TBG_HD void rl_dbl4(int r, RowLineSlots& S, int buf) {  // new T and the line
  if (r >= 12) return;
  const int c = r & 1, j = r >> 1;
  if (j == 0) row_st(S.s[RL_X + c], row_reduce(rl_X3(S, c)));
  else if (j == 1) row_st(S.s[RL_Y + c], row_reduce(rl_p(S, 2, c) - r_mul_small(r_norm(r_mul_small(rl_p(S, 1, c), 4)), 2)));
  else if (j == 2) row_st(S.s[RL_Z + c], row_reduce(r_mul_small(rl_p(S, 0, 6 + c), 2)));
  else if (j == 3) row_st(S.l[buf][c], row_reduce(rl_p(S, 1, 6 + c) - r_mul_small(rl_p(S, 0, 2 + c), 2)));  // X E - 2B
  else if (j == 4) row_st(S.l[buf][2 + c], rl_p(S, 2, 2 + c));
  else row_st(S.l[buf][4 + c], rl_p(S, 2, 4 + c));
}

// ---- addition T <- T + Q and its line
TBG_HD void rl_add1(int r, RowLineSlots& S) {  // ZZ = Z^2, yZ = y Z
  if (r >= 4) return;
  const int ia = r < 2 ? RL_Z : RL_QY;
  rl_job(S, 0, r, rl_ld(S, ia), rl_ld(S, ia + 1), rl_ld(S, RL_Z), rl_ld(S, RL_Z + 1));
}
TBG_HD void rl_add2(int r, RowLineSlots& S) {  // U2 = x ZZ, S2 = yZ ZZ
  if (r >= 4) return;
  const R32 a0 = r < 2 ? rl_ld(S, RL_QX) : rl_p(S, 0, 2), a1 = r < 2 ? rl_ld(S, RL_QX + 1) : rl_p(S, 0, 3);
  rl_job(S, 1, r, a0, a1, rl_p(S, 0, 0), rl_p(S, 0, 1));
}
TBG_HD R32 rl_H(const RowLineSlots& S, int c) { return r_norm(rl_p(S, 1, c) - rl_ld(S, RL_X + c)); }
TBG_HD R32 rl_R(const RowLineSlots& S, int c) { return r_norm(rl_p(S, 1, 2 + c) - rl_ld(S, RL_Y + c)); }
TBG_HD void rl_add3(int r, RowLineSlots& S) {  // HH = H^2, Z3 = Z H, RR = R^2, l1 = R nxP
  if (r >= 8) return;
  const int j = r >> 1;
  const R32 z = r_splat(0);
  R32 a0, a1, b0, b1;
  if (j == 0) { a0 = b0 = rl_H(S, 0); a1 = b1 = rl_H(S, 1); }
  else if (j == 1) { a0 = rl_ld(S, RL_Z); a1 = rl_ld(S, RL_Z + 1); b0 = rl_H(S, 0); b1 = rl_H(S, 1); }
  else if (j == 2) { a0 = b0 = rl_R(S, 0); a1 = b1 = rl_R(S, 1); }
  else { a0 = rl_R(S, 0); a1 = rl_R(S, 1); b0 = row_ld(S.k[0]); b1 = z; }
  rl_job(S, 2, r, a0, a1, b0, b1);
}
TBG_HD void rl_add4(int r, RowLineSlots& S) {  // HHH = H HH, V = X HH, y Z3, R x, l4 = Z3 yP
  if (r >= 10) return;
  const int j = r >> 1;
  const R32 z = r_splat(0);
  R32 a0, a1, b0, b1;
  if (j == 0) { a0 = rl_H(S, 0); a1 = rl_H(S, 1); b0 = rl_p(S, 2, 0); b1 = rl_p(S, 2, 1); }
  else if (j == 1) { a0 = rl_ld(S, RL_X); a1 = rl_ld(S, RL_X + 1); b0 = rl_p(S, 2, 0); b1 = rl_p(S, 2, 1); }
  else if (j == 2) { a0 = rl_ld(S, RL_QY); a1 = rl_ld(S, RL_QY + 1); b0 = rl_p(S, 2, 2); b1 = rl_p(S, 2, 3); }
  else if (j == 3) { a0 = rl_R(S, 0); a1 = rl_R(S, 1); b0 = rl_ld(S, RL_QX); b1 = rl_ld(S, RL_QX + 1); }
  else { a0 = rl_p(S, 2, 2); a1 = rl_p(S, 2, 3); b0 = row_ld(S.k[1]); b1 = z; }
  rl_job(S, 3, r, a0, a1, b0, b1);
}
// X3 = RR - HHH - 2V
TBG_HD R32 rl_aX3(const RowLineSlots& S, int c) {
  return r_norm(rl_p(S, 2, 4 + c) - rl_p(S, 3, c) - r_mul_small(rl_p(S, 3, 2 + c), 2));
}
TBG_HD void rl_add5(int r, RowLineSlots& S) {  // Y HHH, (V - X3) R
  if (r >= 4) return;
  R32 a0, a1, b0, b1;
  if (r < 2) { a0 = rl_ld(S, RL_Y); a1 = rl_ld(S, RL_Y + 1); b0 = rl_p(S, 3, 0); b1 = rl_p(S, 3, 1); }
  else {
    a0 = r_norm(rl_p(S, 3, 2) - rl_aX3(S, 0));
    a1 = r_norm(rl_p(S, 3, 3) - rl_aX3(S, 1));
    b0 = rl_R(S, 0);
    b1 = rl_R(S, 1);
  }
  rl_job(S, 4, r, a0, a1, b0, b1);
}
TBG_HD void rl_add6(int r, RowLineSlots& S, int buf) {
  if (r >= 12) return;
  const int c = r & 1, j = r >> 1;
  if (j == 0) row_st(S.s[RL_X + c], row_reduce(rl_aX3(S, c)));
  else if (j == 1) row_st(S.s[RL_Y + c], row_reduce(rl_p(S, 4, 2 + c) - rl_p(S, 4, c)));
  else if (j == 2) row_st(S.s[RL_Z + c], rl_p(S, 2, 2 + c));
  else if (j == 3) row_st(S.l[buf][c], row_reduce(rl_p(S, 3, 6 + c) - rl_p(S, 3, 4 + c)));  // R x - y Z3
  else if (j == 4) row_st(S.l[buf][2 + c], rl_p(S, 2, 6 + c));
  else row_st(S.l[buf][4 + c], rl_p(S, 3, 8 + c));
}

// one finished line to HBM in line_store's order (plain limbs in [0, 2p));
// `Solo6` runs the six conversions (one Fp each) on one thread apiece
TBG_HD void rl_line_out(const RowLineSlots& S, int buf, int k, uint32_t* dst) {
  const Fp v = fp_from_signed(S.l[buf][k]);
  for (int i = 0; i < NL; ++i) dst[k * NL + i] = v.l[i];
}

// All 68 lines of Q (affine, plain limbs) with (nxP, yP) folded in, in loop
// order.  `ex` runs a row phase on every row then synchronises; `out6(buf,
// idx)` stores line buffer `buf` as line idx (six conversions).
template <class Exec, class Out>
TBG_HD void row_g2_lines(Exec& ex, Out& out6, RowLineSlots& S) {
  int idx = 0, buf = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    ex([&](int r) { rl_dbl1(r, S); });
    ex([&](int r) { rl_dbl2(r, S); });
    ex([&](int r) { rl_dbl3(r, S); });
    ex([&](int r) { rl_dbl4(r, S, buf); });
    out6(buf, idx++);
    buf ^= 1;
    if ((X_ABS >> i) & 1) {
      ex([&](int r) { rl_add1(r, S); });
      ex([&](int r) { rl_add2(r, S); });
      ex([&](int r) { rl_add3(r, S); });
      ex([&](int r) { rl_add4(r, S); });
      ex([&](int r) { rl_add5(r, S); });
      ex([&](int r) { rl_add6(r, S, buf); });
      out6(buf, idx++);
      buf ^= 1;
    }
  }
}

}  // namespace tbg
