// Lane-cooperative Fp12 arithmetic: one Fp12 element per quad of lanes.
//
// Fp12 is viewed as a cubic extension Fp4[x] / (x^3 - y) over
// Fp4 = Fp2[y] / (y^2 - xi), with x = w and y = w^3.  An element
// sum_k a_k w^k (a_k in Fp2) has Fp4 coefficients
//   A0 = (a_0, a_3) = (c0.c0, c1.c1)
//   A1 = (a_1, a_4) = (c1.c0, c0.c2)
//   A2 = (a_2, a_5) = (c0.c1, c1.c2)
// Lane q = 0, 1, 2 of a lane group (the "quad": a trio of lanes of a DPP
// row) owns A_q.  A product is Karatsuba-3 over Fp4: every lane
// computes two Fp4 products (6 Fp2 products) instead of one lane computing
// 18, and operands / partial products move between the lanes of the quad
// with DPP row shifts (full-rate VALU, no LDS).  The per-lane pieces
// are plain functions so the host build can check the algebra by emulating
// the quad (tests/hostcheck).
#pragma once
#include "bls_tower.h"

namespace tbg {

struct Fp4 { Fp2 a, b; };  // a + b y, y^2 = xi

TBG_HD Fp4 fp4_add(const Fp4& x, const Fp4& y) { return {fp2_add(x.a, y.a), fp2_add(x.b, y.b)}; }
TBG_HD Fp4 fp4_sub(const Fp4& x, const Fp4& y) { return {fp2_sub(x.a, y.a), fp2_sub(x.b, y.b)}; }
TBG_HD Fp4 fp4_reduce(const Fp4& x) { return {fp2_reduce(x.a), fp2_reduce(x.b)}; }
TBG_HD Fp4 fp4_add_l(const Fp4& x, const Fp4& y) { return {fp2_add_l(x.a, y.a), fp2_add_l(x.b, y.b)}; }
TBG_HD Fp4 fp4_sub_l(const Fp4& x, const Fp4& y) { return {fp2_sub_l(x.a, y.a), fp2_sub_l(x.b, y.b)}; }
TBG_HD Fp4 fp4_select(bool c, const Fp4& x, const Fp4& y) { return {fp2_select(c, x.a, y.a), fp2_select(c, x.b, y.b)}; }
TBG_HD Fp4 fp4_zero() { return {fp2_zero(), fp2_zero()}; }
// x * y (the Fp4 generator): (a + b y) y = xi b + a y   [lazy]
TBG_HD Fp4 fp4_mul_y(const Fp4& x) { return {fp2_mul_xi(x.b), x.a}; }

// Karatsuba: 3 Fp2 products.  Inputs < 8p, output < 2p.
TBG_HD Fp4 fp4_mul(const Fp4& x, const Fp4& y) {
  Fp2 t0 = fp2_mul(x.a, y.a);
  Fp2 t1 = fp2_mul(x.b, y.b);
  Fp2 s = fp2_mul(fp2_add_l(x.a, x.b), fp2_add(y.a, y.b));
  Fp2 c0 = fp2_reduce(fp2_add_l(fp2_mul_xi(t1), t0));
  Fp2 c1 = fp2_reduce(fp2_sub_l(s, fp2_add(t0, t1)));
  return {c0, c1};
}

TBG_HD Fp4 fp4_sqr(const Fp4& x) {
  Fp2 t0, t1;
  fp4_sqr(x.a, x.b, t0, t1);
  return {t0, fp2_reduce(t1)};
}

TBG_HD Fp4 fp4_mul_fp2(const Fp4& x, const Fp2& s) { return {fp2_mul(x.a, s), fp2_mul(x.b, s)}; }

// ---------------------------------------------------------------------------
// per-lane pieces (q = lane index 0..2 of the quad)

// After the products P = A_q B_q and Q = (A_{q+1} + A_{q+2})(B_{q+1} + B_{q+2})
// of every lane: Pn = P_{q+1}, Pp = P_{q+2}, Qx = Q of lane {0, 2, 1}[q].
//   C0 = P0 + y (Q0 - P1 - P2), C1 = Q2 - P0 - P1 + y P2, C2 = Q1 - P0 - P2 + P1
TBG_HD Fp4 quad_combine(int q, const Fp4& P, const Fp4& Pn, const Fp4& Pp, const Fp4& Qx) {
  Fp4 f1 = fp4_select(q == 1, Pp, Pn);
  Fp4 f2 = fp4_select(q == 0, Pp, P);
  Fp4 T = fp4_reduce(fp4_sub_l(Qx, fp4_add(f1, f2)));           // < 2p
  Fp4 yPn = fp4_reduce(fp4_mul_y(Pn));
  Fp4 W = fp4_select(q == 0, P, fp4_select(q == 1, yPn, Pp));
  Fp4 Ty = fp4_reduce(fp4_mul_y(T));
  return fp4_reduce(fp4_add_l(fp4_select(q == 0, Ty, T), W));
}

// Line f * (L0 + L2 x^2), L0 = (l0, l4), L2 = l1 (in Fp2):
//   C_q = A_q L0 + (q < 2 ? y : 1) A_{q+1} l1
TBG_HD Fp4 quad_line_lane(int q, const Fp4& A, const Fp4& An, const Fp2& l0, const Fp2& l1, const Fp2& l4) {
  Fp4 t = fp4_mul(A, {l0, l4});
  Fp4 u = fp4_mul_fp2(An, l1);
  Fp4 uy = fp4_reduce(fp4_mul_y(u));
  return fp4_reduce(fp4_add_l(t, fp4_select(q < 2, uy, u)));
}

// Cyclotomic squaring (Granger-Scott) per lane: T = fp4_sqr(A_q) on every
// lane, Tx = T of lane {0, 2, 1}[q].
TBG_HD Fp4 quad_cyc_lane(int q, const Fp4& A, const Fp4& Tx) {
  Fp2 s1 = fp2_select(q == 1, fp2_reduce(fp2_mul_xi(Tx.b)), Tx.a);
  Fp2 s2 = fp2_select(q == 1, Tx.a, Tx.b);
  Fp2 a2 = fp2_dbl(A.a), b2 = fp2_dbl(A.b);
  Fp2 s13 = fp2_mul_small(s1, 3), s23 = fp2_mul_small(s2, 3);
  Fp2 na = fp2_select(q == 1, fp2_add_l(s13, a2), fp2_sub_l(s13, a2));
  Fp2 nb = fp2_select(q == 1, fp2_sub_l(s23, b2), fp2_add_l(s23, b2));
  return {fp2_reduce(na), fp2_reduce(nb)};
}

// conj(f) (w -> -w): negate a_1, a_3, a_5.
TBG_HD Fp4 quad_conj_lane(int q, const Fp4& A) {
  Fp2 na = fp2_reduce(fp2_neg(A.a)), nb = fp2_reduce(fp2_neg(A.b));
  return {fp2_select(q == 1, na, A.a), fp2_select(q == 1, A.b, nb)};
}

// f^p: a_k -> conj(a_k) gamma_k.
TBG_HD Fp4 quad_frob_lane(int q, const Fp4& A) {
  Fp2 ga = fp2_select(q == 0, fp2_one(), fp2_select(q == 1, fp2_from_const(FROB_G1), fp2_from_const(FROB_G2)));
  Fp2 gb = fp2_select(q == 0, fp2_from_const(FROB_G3), fp2_select(q == 1, fp2_from_const(FROB_G4), fp2_from_const(FROB_G5)));
  return {fp2_mul(fp2_conj(A.a), ga), fp2_mul(fp2_conj(A.b), gb)};
}

// Fp4 coefficient q of a tower element, and back.
TBG_HD Fp4 quad_from_fp12(int q, const Fp12& f) {
  if (q == 0) return {f.c0.c0, f.c1.c1};
  if (q == 1) return {f.c1.c0, f.c0.c2};
  return {f.c0.c1, f.c1.c2};
}
TBG_HD Fp12 quad_to_fp12(const Fp4& A0, const Fp4& A1, const Fp4& A2) {
  Fp12 f;
  f.c0.c0 = A0.a; f.c1.c1 = A0.b;
  f.c1.c0 = A1.a; f.c0.c2 = A1.b;
  f.c0.c1 = A2.a; f.c1.c2 = A2.b;
  return f;
}

}  // namespace tbg

// ---------------------------------------------------------------------------
// Device side: the DPP exchanges and the quad-level operations.
#if defined(__HIP__)
namespace tbg {

#define TBG_DEV __device__ __forceinline__
#ifndef TBG_INLINE_QUAD
#define TBG_INLINE_QUAD TBG_INLINE_PT
#endif
#if TBG_INLINE_QUAD
#define TBG_QUAD_FN __forceinline__
#else
#define TBG_QUAD_FN __noinline__
#endif

// Lane groups: an Fp12 lives on a TRIO of consecutive lanes of a 16-lane
// DPP row -- 5 trios per row, lane 15 idle, so 60 of 64 lanes work; operands
// move with DPP row shifts (two per word plus a select).  (The round-1 quad
// layout -- lanes 4k .. 4k + 3 with lane 3 mirroring lane 2, one quad_perm
// move per word -- kept 48 of 64 lanes busy and was slower; removed.)
// exchange kinds: lane q of the group reads the value of lane ...
enum QuadXch : int {
  QP_NEXT = 0,  // (q + 1) mod 3
  QP_PREV = 1,  // (q + 2) mod 3
  QP_SW12 = 2,  // {0, 2, 1}[q]
  QP_B0 = 3,    // 0 (broadcast)
  QP_B1 = 4,    // 1
  QP_B2 = 5,    // 2
};

// bound_ctrl: a lane whose source is outside its row reads 0 -- the value the
// `old` operand gave before, but without the v_mov that initialised it for
// every exchanged word (532 of k_miller_hex's loop-body instructions)
template <int CTRL>
TBG_DEV uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}

// DPP row shifts: row_shl:n -- lane l reads lane l + n of its row; row_shr:n -- lane l - n.
constexpr int DPP_SHL1 = 0x101, DPP_SHL2 = 0x102, DPP_SHR1 = 0x111, DPP_SHR2 = 0x112;
TBG_DEV int quad_lane() { return (int)((threadIdx.x & 15u) % 3u); }
// Fp12 slot of global thread t (UINT32_MAX for the idle lane 15 of a row),
// and the threads n slots need.
TBG_HD uint32_t fp12_slot(uint32_t t) {
  const uint32_t l = t & 15u;
  return l == 15u ? 0xFFFFFFFFu : (t >> 4) * 5u + l / 3u;
}
inline uint32_t fp12_threads(uint32_t n) { return 16u * ((n + 4u) / 5u); }
template <int K>
TBG_DEV uint32_t xch_u32(uint32_t v) {
  const int q = quad_lane();
  if (K == QP_NEXT) { const uint32_t a = dpp_u32<DPP_SHL1>(v), b = dpp_u32<DPP_SHR2>(v); return q < 2 ? a : b; }
  if (K == QP_PREV) { const uint32_t a = dpp_u32<DPP_SHL2>(v), b = dpp_u32<DPP_SHR1>(v); return q == 0 ? a : b; }
  if (K == QP_SW12) { const uint32_t a = dpp_u32<DPP_SHL1>(v), b = dpp_u32<DPP_SHR1>(v); return q == 0 ? v : (q == 1 ? a : b); }
  if (K == QP_B0) { const uint32_t a = dpp_u32<DPP_SHR1>(v), b = dpp_u32<DPP_SHR2>(v); return q == 0 ? v : (q == 1 ? a : b); }
  if (K == QP_B1) { const uint32_t a = dpp_u32<DPP_SHL1>(v), b = dpp_u32<DPP_SHR1>(v); return q == 0 ? a : (q == 1 ? v : b); }
  const uint32_t a = dpp_u32<DPP_SHL2>(v), b = dpp_u32<DPP_SHL1>(v);  // QP_B2
  return q == 0 ? a : (q == 1 ? b : v);
}
// lane 0 of this thread's group (the list-slot owner of push_ident)
TBG_DEV uint32_t quad_lead_lane() { return threadIdx.x - (uint32_t)quad_lane(); }

template <int K>
TBG_DEV Fp xch(const Fp& x) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = xch_u32<K>(x.l[i]);
  return r;
}
template <int K>
TBG_DEV Fp2 xch(const Fp2& x) { return {xch<K>(x.c0), xch<K>(x.c1)}; }
template <int K>
TBG_DEV Fp4 xch(const Fp4& x) { return {xch<K>(x.a), xch<K>(x.b)}; }

// C = A * B (both quad-distributed).  The _in bodies are for kernel loops;
// the out-of-line forms serve the final exponentiation's callable loops.
TBG_DEV Fp4 quad_mul_in(const Fp4& A, const Fp4& B) {
  int q = quad_lane();
  Fp4 SA = fp4_add(xch<QP_NEXT>(A), xch<QP_PREV>(A));
  Fp4 SB = fp4_add(xch<QP_NEXT>(B), xch<QP_PREV>(B));
  Fp4 P = fp4_mul(A, B);
  Fp4 Q = fp4_mul(SA, SB);
  return quad_combine(q, P, xch<QP_NEXT>(P), xch<QP_PREV>(P), xch<QP_SW12>(Q));
}

TBG_DEV Fp4 quad_sqr_in(const Fp4& A) {
  int q = quad_lane();
  Fp4 SA = fp4_add(xch<QP_NEXT>(A), xch<QP_PREV>(A));
  Fp4 P = fp4_sqr(A);
  Fp4 Q = fp4_sqr(SA);
  return quad_combine(q, P, xch<QP_NEXT>(P), xch<QP_PREV>(P), xch<QP_SW12>(Q));
}

TBG_DEV Fp4 quad_cyc_sqr_in(const Fp4& A) {
  Fp4 T = fp4_sqr(A);
  return quad_cyc_lane(quad_lane(), A, xch<QP_SW12>(T));
}

TBG_DEV Fp4 quad_line_in(const Fp4& A, const Fp2& l0, const Fp2& l1, const Fp2& l4) {
  return quad_line_lane(quad_lane(), A, xch<QP_NEXT>(A), l0, l1, l4);
}

__device__ TBG_QUAD_FN Fp4 quad_mul(const Fp4& A, const Fp4& B) { return quad_mul_in(A, B); }
__device__ TBG_QUAD_FN Fp4 quad_sqr(const Fp4& A) { return quad_sqr_in(A); }
__device__ TBG_QUAD_FN Fp4 quad_cyc_sqr(const Fp4& A) { return quad_cyc_sqr_in(A); }
__device__ TBG_QUAD_FN Fp4 quad_line(const Fp4& A, const Fp2& l0, const Fp2& l1, const Fp2& l4) {
  return quad_line_in(A, l0, l1, l4);
}

TBG_DEV Fp4 quad_conj(const Fp4& A) { return quad_conj_lane(quad_lane(), A); }
TBG_DEV Fp4 quad_frob(const Fp4& A) { return quad_frob_lane(quad_lane(), A); }

TBG_DEV Fp4 quad_one() {
  Fp4 r = fp4_zero();
  if (quad_lane() == 0) r.a = fp2_one();
  return r;
}

// Gather the whole element on every lane (tower form).
TBG_DEV Fp12 quad_gather(const Fp4& A) { return quad_to_fp12(xch<QP_B0>(A), xch<QP_B1>(A), xch<QP_B2>(A)); }

// f^-1 via the tower inverse, replicated on the lanes of the quad.
__device__ TBG_QUAD_FN Fp4 quad_inv(const Fp4& A) { return quad_from_fp12(quad_lane(), fp12_inv(quad_gather(A))); }

// a^|x| in the cyclotomic subgroup
__device__ TBG_QUAD_FN Fp4 quad_pow_xabs(const Fp4& a) {
  Fp4 r = a;
  for (int i = 62; i >= 0; --i) {
    r = quad_cyc_sqr(r);
    if ((X_ABS >> i) & 1) r = quad_mul(r, a);
  }
  return r;
}
TBG_DEV Fp4 quad_pow_x(const Fp4& a) { return quad_conj(quad_pow_xabs(a)); }

// f^(3 (p^12 - 1) / r), as final_exp() in bls_pairing.h.
__device__ TBG_QUAD_FN Fp4 quad_final_exp(const Fp4& f) {
  Fp4 t = quad_mul(quad_conj(f), quad_inv(f));
  t = quad_mul(quad_frob(quad_frob(t)), t);
  Fp4 a = quad_mul(quad_pow_x(t), quad_conj(t));
  a = quad_mul(quad_pow_x(a), quad_conj(a));
  Fp4 b = quad_mul(quad_pow_x(a), quad_frob(a));
  Fp4 c = quad_mul(quad_pow_x(quad_pow_x(b)), quad_frob(quad_frob(b)));
  c = quad_mul(c, quad_conj(b));
  Fp4 t3 = quad_mul(quad_cyc_sqr(t), t);
  return quad_mul(c, t3);
}

// Kernel-inline forms of the final exponentiation for the level-1 group
// check (k_rlc_group_final, the per-group hot path): the 5 x 63 cyclotomic
// squarings run inline in the kernel's own loop instead of as out-of-line
// calls, each of which passed its Fp4 operands through the scratch stack
// (4.1 GB of scratch write-back per 160k-DV launch, profiles/r02/
// traffic_merge16.json).  The rare products stay out of line.  Call these
// from a kernel body only: kernels are not affected by the long-branch
// return-address hazard of out-of-line loops (see _native.py).
TBG_DEV Fp4 quad_pow_xabs_in(const Fp4& a) {
  Fp4 r = a;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    r = quad_cyc_sqr_in(r);
    if ((X_ABS >> i) & 1) r = quad_mul(r, a);
  }
  return r;
}
TBG_DEV Fp4 quad_pow_x_in(const Fp4& a) { return quad_conj(quad_pow_xabs_in(a)); }
TBG_DEV Fp4 quad_final_exp_in(const Fp4& f) {
  Fp4 t = quad_mul(quad_conj(f), quad_inv(f));
  t = quad_mul(quad_frob(quad_frob(t)), t);
  Fp4 a = quad_mul(quad_pow_x_in(t), quad_conj(t));
  a = quad_mul(quad_pow_x_in(a), quad_conj(a));
  Fp4 b = quad_mul(quad_pow_x_in(a), quad_frob(a));
  Fp4 c = quad_mul(quad_pow_x_in(quad_pow_x_in(b)), quad_frob(quad_frob(b)));
  c = quad_mul(c, quad_conj(b));
  Fp4 t3 = quad_mul(quad_cyc_sqr(t), t);
  return quad_mul(c, t3);
}

// true on every lane iff the quad's element is 1
TBG_DEV bool quad_is_one(const Fp4& A) {
  int q = quad_lane();
  bool ok = fp2_is_zero(A.b) && (q == 0 ? fp2_eq(A.a, fp2_one()) : fp2_is_zero(A.a));
  uint32_t v = ok ? 1u : 0u;
  return (xch_u32<QP_B0>(v) & xch_u32<QP_B1>(v) & xch_u32<QP_B2>(v)) != 0;
}

}  // namespace tbg
#endif
