// Lane-pair Fp2 arithmetic: one Fp2 element per pair of lanes (2k, 2k + 1).
//
// Why: a G2 point in Jacobian form is 6 Fp = 84 VGPRs per lane, and the
// point loops of decode / RLC / hash_to_G2 / Miller lines keep two or three
// points plus Fp2 temporaries live, which pushed those kernels past 256
// registers -- one wave per SIMD.  On gfx950 a lone wave issues
// v_mad_u64_u32 at ~58 % of the rate two waves reach (profiles/r02/
// valu_rates.txt: 19.0 vs 32.8 T lane-ops/s), so register-bound kernels
// cannot pass ~0.6 of the VALU peak however well they schedule.  Spreading
// every Fp2 over two lanes halves the per-lane state (a G2 point is 42
// VGPRs) at no extra multiplication work:
//
//   even lane holds c0, odd lane holds c1 (partner = lane ^ 1, one DPP
//   quad_perm move per limb); with a, b own and a', b' the partner's values
//     product   even: REDC(a b + a' (-b'))  = a0 b0 - a1 b1
//               odd:  REDC(a b' + a' b)     = a0 b1 + a1 b0
//     square    even: (a + a')(a - a'),  odd: (2 a') a
//   -- each lane runs ONE fp_mul2 (588 u32 mul-adds), exactly half of the
//   single-lane fp2_mul (2 fp_mul2).  Additions, subtractions, negation,
//   reduction and small multiples are component-wise; conj / mul-by-xi are a
//   per-lane select.  Only Fp-level work (the norm inversion of fp2_inv)
//   runs redundantly on both lanes.
//
// The per-lane pieces below are plain functions so the host build checks the
// algebra by emulating the pair (Fp2p, tests/hostcheck); the device type
// Fp2x binds them to DPP exchanges.  Both plug into the generic group law of
// bls_curve.h through the f_* overloads.
#pragma once
#include "bls_lines.h"

namespace tbg {

// ---- per-lane pieces: par = lane parity, a / b own values, ap / bp partner's
TBG_HD Fp pair_mul_lane(uint32_t par, const Fp& a, const Fp& ap, const Fp& b, const Fp& bp) {
  const Fp nbp = fp_neg_l(bp);  // (lazy: a product operand only)
  return fp_mul2(a, fp_select(par != 0, bp, b), ap, fp_select(par != 0, b, nbp));
}
// (the lane's operands a, a' normalised: a' is subtracted; the two factors
// stay lazy, fp_mul's columns take their limbs)
TBG_HD Fp pair_sqr_lane(uint32_t par, const Fp& a, const Fp& ap) {
  const Fp x = fp_add_l(fp_select(par != 0, ap, a), ap);     // even a + a', odd 2 a'
  const Fp y = fp_select(par != 0, a, fp_sub_l(a, ap));      // even a - a', odd a
  return fp_mul(x, y);
}
TBG_HD Fp pair_conj_lane(uint32_t par, const Fp& a) { return fp_select(par != 0, fp_neg(a), a); }
TBG_HD Fp pair_mul_xi_lane(uint32_t par, const Fp& a, const Fp& ap) {
  return fp_select(par != 0, fp_add(a, ap), fp_sub(a, ap));  // (a0 - a1) + (a0 + a1) u, lazy
}
// 1 / a: the norm a0^2 + a1^2 is the same on both lanes.
TBG_HD Fp pair_inv_lane(uint32_t par, const Fp& a, const Fp& ap) {
  const Fp t = fp_inv(fp_mul2(a, a, ap, ap));
  return fp_mul(pair_conj_lane(par, a), t);
}
TBG_HD Fp pair_const(uint32_t par, const Fp2Const& c) { return par ? fp_from_const(c.c1) : fp_from_const(c.c0); }

// ---- host emulation of a pair (tests only): both lanes side by side
struct Fp2p { Fp c0, c1; };
TBG_HD Fp2p f_add(const Fp2p& a, const Fp2p& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
TBG_HD Fp2p f_sub(const Fp2p& a, const Fp2p& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
TBG_HD Fp2p f_add_l(const Fp2p& a, const Fp2p& b) { return {fp_add_l(a.c0, b.c0), fp_add_l(a.c1, b.c1)}; }
TBG_HD Fp2p f_sub_l(const Fp2p& a, const Fp2p& b) { return {fp_sub_l(a.c0, b.c0), fp_sub_l(a.c1, b.c1)}; }
TBG_HD Fp2p f_neg(const Fp2p& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
TBG_HD Fp2p f_reduce(const Fp2p& a) { return {fp_reduce(a.c0), fp_reduce(a.c1)}; }
TBG_HD Fp2p f_small(const Fp2p& a, uint32_t k) { return {fp_mul_small(a.c0, k), fp_mul_small(a.c1, k)}; }
TBG_HD Fp2p f_mul(const Fp2p& a, const Fp2p& b) {
  return {pair_mul_lane(0, a.c0, a.c1, b.c0, b.c1), pair_mul_lane(1, a.c1, a.c0, b.c1, b.c0)};
}
TBG_HD Fp2p f_sqr(const Fp2p& a) { return {pair_sqr_lane(0, a.c0, a.c1), pair_sqr_lane(1, a.c1, a.c0)}; }
TBG_HD Fp2p f_inv(const Fp2p& a) { return {pair_inv_lane(0, a.c0, a.c1), pair_inv_lane(1, a.c1, a.c0)}; }
TBG_HD bool f_is_zero(const Fp2p& a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
TBG_HD bool f_eq(const Fp2p& a, const Fp2p& b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
TBG_HD Fp2p pp_conj(const Fp2p& a) { return {pair_conj_lane(0, a.c0), pair_conj_lane(1, a.c1)}; }
TBG_HD Fp2p pp_mul_xi(const Fp2p& a) { return {pair_mul_xi_lane(0, a.c0, a.c1), pair_mul_xi_lane(1, a.c1, a.c0)}; }
TBG_HD Fp2p pp_mul_const(const Fp2p& a, const Fp2Const& c) {
  return {pair_mul_lane(0, a.c0, a.c1, pair_const(0, c), pair_const(1, c)),
          pair_mul_lane(1, a.c1, a.c0, pair_const(1, c), pair_const(0, c))};
}
TBG_HD Fp2p rlc_mul_c(const Fp2p& a, const Fp& c) { return {fp_mul(a.c0, c), fp_mul(a.c1, c)}; }
TBG_HD Fp2p f_conj(const Fp2p& a) { return pp_conj(a); }
TBG_HD Fp2p f_mulc(const Fp2p& a, const Fp2Const& c) { return pp_mul_const(a, c); }
template <> TBG_HD Fp2p f_zero<Fp2p>() { return {fp_zero(), fp_zero()}; }
template <> TBG_HD Fp2p f_one<Fp2p>() { return {fp_one(), fp_zero()}; }
TBG_HD Fp2p pp_from(const Fp2& a) { return {a.c0, a.c1}; }
TBG_HD Fp2 pp_to(const Fp2p& a) { return {a.c0, a.c1}; }

// psi(P) on Jacobian coordinates: (conj(X) PSI_X, conj(Y) PSI_Y, conj(Z)).
template <class F>
TBG_HD Jac<F> g2_psi_g(const Jac<F>& p) {
  return {f_mulc(f_conj(p.X), PSI_X), f_mulc(f_conj(p.Y), PSI_Y), f_reduce(f_conj(p.Z))};
}

// Jacobian addition without the P == Q branch: when it would be needed
// (H == 0 with R == 0, a doubling) `exc` is set and the result is unusable;
// the caller redoes the item on the reference path.  P == -Q and infinities
// are handled.  Keeping the rare doubling out of the loop body is what lets
// the lane-pair kernels fit their registers.
template <class F>
TBG_HD Jac<F> jac_add_x(const Jac<F>& p, const Jac<F>& q, bool& exc) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  // add-2007-bl in an order that retires inputs early (few values live at
  // once; with TBG_SCHED_FENCE the products run in program order)
  const F Z1Z1 = f_sqr(p.Z);
  const F Z2Z2 = f_sqr(q.Z);
  const F S1 = f_mul(f_mul(p.Y, q.Z), Z2Z2);
  const F S2 = f_mul(f_mul(q.Y, p.Z), Z1Z1);
  const F Zs = f_reduce(f_sub_l(f_sqr(f_add(p.Z, q.Z)), f_add(Z1Z1, Z2Z2)));
  const F U1 = f_mul(p.X, Z2Z2);
  const F H = f_reduce(f_sub_l(f_mul(q.X, Z1Z1), U1));
  const F Rr = f_reduce(f_sub_l(S2, S1));
  if (f_is_zero(H)) {
    if (f_is_zero(Rr)) exc = true;
    return jac_inf<F>();
  }
  const F Z3 = f_mul(Zs, H);
  const F H2 = f_add(H, H);
  const F I = f_sqr(H2);
  const F J = f_mul(H, I);
  const F V = f_mul(U1, I);
  const F r2 = f_add(Rr, Rr);
  const F X3 = f_reduce(f_sub_l(f_sub_l(f_sqr(r2), J), f_add(V, V)));
  const F Y3 = f_reduce(f_sub_l(f_mul(f_sub_l(V, X3), r2), f_small(f_mul(S1, J), 2)));
  return {X3, Y3, Z3};
}

// dbl-2009-l (as jac_dbl_in) in an order that retires inputs early.
template <class F>
TBG_HD Jac<F> jac_dbl_lo(const Jac<F>& p) {
  const F YZ = f_mul(p.Y, p.Z);
  const F Z3 = f_reduce(f_add_l(YZ, YZ));
  const F B = f_sqr(p.Y);
  const F A = f_sqr(p.X);
  const F C = f_sqr(B);
  const F t = f_sub_l(f_sqr(f_add(p.X, B)), f_add(A, C));   // < 18p
  const F D = f_reduce(f_add_l(t, t));
  const F E = f_small(A, 3);                                // < 6p
  const F X3 = f_reduce(f_sub_l(f_sqr(E), f_add(D, D)));
  const F Y3 = f_reduce(f_sub_l(f_mul(f_sub_l(D, X3), E), f_small(C, 8)));
  return {X3, Y3, Z3};
}

// Mixed addition P + Q (Q affine) without the P == Q branch (see jac_add_x).
template <class F>
TBG_HD Jac<F> jac_add_aff_x(const Jac<F>& p, const Aff<F>& q, bool& exc) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  F Z1Z1 = f_sqr(p.Z);
  F U2 = f_mul(q.x, Z1Z1);
  F S2 = f_mul(f_mul(q.y, p.Z), Z1Z1);
  F H = f_reduce(f_sub_l(U2, p.X));
  F Rr = f_reduce(f_sub_l(S2, p.Y));
  if (f_is_zero(H)) {
    if (f_is_zero(Rr)) exc = true;
    return jac_inf<F>();
  }
  F HH = f_sqr(H);
  F I = f_small(HH, 4);
  F J = f_mul(H, I);
  F r2 = f_add(Rr, Rr);
  F V = f_mul(p.X, I);
  F X3 = f_reduce(f_sub_l(f_sub_l(f_sqr(r2), J), f_add(V, V)));
  F Y3 = f_reduce(f_sub_l(f_mul(f_sub_l(V, X3), r2), f_small(f_mul(p.Y, J), 2)));
  F Z3 = f_reduce(f_sub_l(f_sub_l(f_sqr(f_add(p.Z, H)), Z1Z1), HH));
  return {X3, Y3, Z3};
}

template <class F>
TBG_HD Jac<F> jac_mul_xabs_aff_x(const Aff<F>& p, bool& exc) {
  Jac<F> acc = jac_from_aff(p);
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl_lo(acc);
    if ((X_ABS >> i) & 1) acc = jac_add_aff_x(acc, p, exc);
  }
  return acc;
}

template <class F>
TBG_HD Jac<F> jac_mul_xabs_x(const Jac<F>& p, bool& exc) {
  Jac<F> acc = p;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl_lo(acc);
    if ((X_ABS >> i) & 1) acc = jac_add_x(acc, p, exc);
  }
  return acc;
}

// Budroni-Pintore cofactor clearing (RFC 9380 G.3),
//   h(P) = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P)
//        = u + [x] b,  b = [x]P + psi(P),  u = psi^2(2P) - psi(P) - [x]P - P,
// ordered so that only u, b and the accumulator are live during the second
// [x] multiplication.  Every group operation is inline; exc reports an
// addition that needed the doubling branch (see jac_add_x).
template <class F>
TBG_HD Jac<F> g2_clear_cofactor_g(const Jac<F>& p, bool& exc) {
  const Jac<F> a = jac_neg(jac_mul_xabs_x(p, exc));   // [x]P
  const Jac<F> pp = g2_psi_g(p);                       // psi(P)
  const Jac<F> b = jac_add_x(a, pp, exc);
  Jac<F> u = g2_psi_g(g2_psi_g(jac_dbl_lo(p)));       // psi^2(2P)
  u = jac_add_x(u, jac_neg(pp), exc);
  u = jac_add_x(u, jac_neg(a), exc);
  u = jac_add_x(u, jac_neg(p), exc);
  const Jac<F> c = jac_neg(jac_mul_xabs_x(b, exc));   // [x] b
  return jac_add_x(u, c, exc);
}

// Miller steps (bls_pairing.h miller_dbl_in / miller_add_in) for any Fp2
// representation; f_mulfp multiplies by an Fp scalar component-wise.  EVAL =
// false leaves P out altogether (the H(m) lines: l1, l4 stored unevaluated,
// no products by the Montgomery one -- 2 of a line's ~17 products per lane).
template <class F> struct LineG { F l0, l1, l4; };

// The steps hand each line coefficient to `sink(k, v)` (k = 0, 1, 2 for l0,
// l1, l4) as soon as it is formed, in an order that retires inputs early:
// a kernel storing them directly keeps ~6 Fp2 live instead of ~9 (k_lines_h
// spilled 91 VGPRs with the formula order).  The products are the formulas'
// own, operand for operand.
template <class F, bool EVAL = true, class S>
TBG_HD void miller_dbl_s(Jac<F>& T, const Fp& nxP, const Fp& yP, S&& sink) {
  const F ZZ = f_sqr(T.Z);
  const F YZ = f_mul(T.Y, T.Z);
  const F Z3 = f_reduce(f_add_l(YZ, YZ));
  const F l4 = f_mul(Z3, ZZ);                              // 2 Y Z^3 yP
  sink(2, EVAL ? f_mulfp(l4, yP) : l4);
  const F B = f_sqr(T.Y);
  const F C = f_sqr(B);
  const F A = f_sqr(T.X);
  const F t = f_sub_l(f_sqr(f_add(T.X, B)), f_add(A, C));
  const F D = f_reduce(f_add_l(t, t));
  const F E = f_small(A, 3);
  const F l1 = f_mul(ZZ, E);                               // -3X^2 Z^2 xP
  sink(1, EVAL ? f_mulfp(l1, nxP) : l1);
  sink(0, f_reduce(f_sub_l(f_mul(T.X, E), f_add(B, B))));  // 3X^3 - 2Y^2
  const F X3 = f_reduce(f_sub_l(f_sqr(E), f_add(D, D)));
  const F Y3 = f_reduce(f_sub_l(f_mul(f_sub_l(D, X3), E), f_small(C, 8)));
  T = {X3, Y3, Z3};
}

template <class F, bool EVAL = true, class S>
TBG_HD void miller_add_s(Jac<F>& T, const Aff<F>& Q, const Fp& nxP, const Fp& yP, S&& sink) {
  const F ZZ = f_sqr(T.Z);
  const F U2 = f_mul(Q.x, ZZ);
  const F S2 = f_mul(f_mul(Q.y, T.Z), ZZ);
  const F H = f_reduce(f_sub_l(U2, T.X));
  const F R = f_reduce(f_sub_l(S2, T.Y));
  const F Z3 = f_mul(T.Z, H);
  sink(2, EVAL ? f_mulfp(Z3, yP) : Z3);
  sink(1, EVAL ? f_mulfp(R, nxP) : R);
  sink(0, f_reduce(f_sub_l(f_mul(R, Q.x), f_mul(Q.y, Z3))));
  const F HH = f_sqr(H);
  const F HHH = f_mul(H, HH);
  const F V = f_mul(T.X, HH);
  const F X3 = f_reduce(f_sub_l(f_sub_l(f_sqr(R), HHH), f_add(V, V)));
  const F Y3 = f_reduce(f_sub_l(f_mul(f_sub_l(V, X3), R), f_mul(T.Y, HHH)));
  T = {X3, Y3, Z3};
}

template <class F, bool EVAL = true>
TBG_HD LineG<F> miller_dbl_g(Jac<F>& T, const Fp& nxP, const Fp& yP) {
  LineG<F> l;
  miller_dbl_s<F, EVAL>(T, nxP, yP, [&](int k, const F& v) { (k == 0 ? l.l0 : k == 1 ? l.l1 : l.l4) = v; });
  return l;
}

template <class F, bool EVAL = true>
TBG_HD LineG<F> miller_add_g(Jac<F>& T, const Aff<F>& Q, const Fp& nxP, const Fp& yP) {
  LineG<F> l;
  miller_add_s<F, EVAL>(T, Q, nxP, yP, [&](int k, const F& v) { (k == 0 ? l.l0 : k == 1 ? l.l1 : l.l4) = v; });
  return l;
}

TBG_HD Fp2 f_mulfp(const Fp2& a, const Fp& c) { return fp2_mul_fp(a, c); }
TBG_HD Fp2p f_mulfp(const Fp2p& a, const Fp& c) { return rlc_mul_c(a, c); }

// psi(a) == [x] a == -[|x|] a for an affine point on E2 (Scott), written for
// any Fp2 representation F with the f_* / f_conj / f_mulc overloads: the lane
// pair (Fp2x, device) and its host emulation (Fp2p).  Same schedule as
// g2_in_subgroup_aff_in (63 doublings, 5 mixed additions, inline).
template <class F>
TBG_HD bool g2_in_subgroup_aff_g(const Aff<F>& a, bool& exc) {
  const Jac<F> m = jac_mul_xabs_aff_x(a, exc);  // [|x|] a; exc: redo on the reference path
  const F px = f_mulc(f_conj(a.x), PSI_X);
  const F py = f_mulc(f_conj(a.y), PSI_Y);
  const F z2 = f_sqr(m.Z);
  const F z3 = f_mul(z2, m.Z);
  if (jac_is_inf(m)) return false;
  return f_eq(f_mul(px, z2), m.X) && f_eq(f_mul(py, z3), f_reduce(f_neg(m.Y)));
}

}  // namespace tbg

// ---------------------------------------------------------------------------
// Device: the pair as two lanes of a wave.
#if defined(__HIP__)
namespace tbg {

#ifndef TBG_DEV
#define TBG_DEV __device__ __forceinline__
#endif

struct Fp2x { Fp v; };  // this lane's component (c0 on even lanes, c1 on odd)

constexpr int QP_PAIR = 1 | (0 << 2) | (3 << 4) | (2 << 6);  // quad_perm [1, 0, 3, 2]: the partner lane

TBG_DEV uint32_t pair_par() { return threadIdx.x & 1u; }
TBG_DEV uint32_t pair_u32(uint32_t v) {
  // (every lane's source is valid; bound_ctrl spares the v_mov of `old`)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, QP_PAIR, 0xf, 0xf, true);
}
TBG_DEV Fp pair_xch(const Fp& x) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = pair_u32(x.l[i]);
  return r;
}
// true on both lanes iff true on both
TBG_DEV bool pair_all(bool b) {
  uint32_t v = b ? 1u : 0u;
  return (v & pair_u32(v)) != 0;
}

TBG_DEV Fp2x f_add(const Fp2x& a, const Fp2x& b) { return {fp_add(a.v, b.v)}; }
TBG_DEV Fp2x f_sub(const Fp2x& a, const Fp2x& b) { return {fp_sub(a.v, b.v)}; }
TBG_DEV Fp2x f_add_l(const Fp2x& a, const Fp2x& b) { return {fp_add_l(a.v, b.v)}; }
TBG_DEV Fp2x f_sub_l(const Fp2x& a, const Fp2x& b) { return {fp_sub_l(a.v, b.v)}; }
TBG_DEV Fp2x f_neg(const Fp2x& a) { return {fp_neg(a.v)}; }
TBG_DEV Fp2x f_reduce(const Fp2x& a) { return {fp_reduce(a.v)}; }
TBG_DEV Fp2x f_small(const Fp2x& a, uint32_t k) { return {fp_mul_small(a.v, k)}; }
TBG_DEV Fp2x f_mul(const Fp2x& a, const Fp2x& b) {
  return {pair_mul_lane(pair_par(), a.v, pair_xch(a.v), b.v, pair_xch(b.v))};
}
TBG_DEV Fp2x f_sqr(const Fp2x& a) { return {pair_sqr_lane(pair_par(), a.v, pair_xch(a.v))}; }
TBG_DEV Fp2x f_inv(const Fp2x& a) { return {pair_inv_lane(pair_par(), a.v, pair_xch(a.v))}; }
TBG_DEV bool f_is_zero(const Fp2x& a) { return pair_all(fp_is_zero(a.v)); }
TBG_DEV bool f_eq(const Fp2x& a, const Fp2x& b) { return pair_all(fp_eq(a.v, b.v)); }
TBG_DEV Fp2x px_conj(const Fp2x& a) { return {pair_conj_lane(pair_par(), a.v)}; }
TBG_DEV Fp2x px_mul_xi(const Fp2x& a) { return {pair_mul_xi_lane(pair_par(), a.v, pair_xch(a.v))}; }
TBG_DEV Fp2x px_mul_const(const Fp2x& a, const Fp2Const& c) {
  const uint32_t par = pair_par();
  return {pair_mul_lane(par, a.v, pair_xch(a.v), pair_const(par, c), pair_const(par ^ 1u, c))};
}
TBG_DEV Fp2x rlc_mul_c(const Fp2x& a, const Fp& c) { return {fp_mul(a.v, c)}; }  // Fp scalar: component-wise
TBG_DEV Fp2x f_mulfp(const Fp2x& a, const Fp& c) { return {fp_mul(a.v, c)}; }
TBG_DEV Fp2x f_conj(const Fp2x& a) { return px_conj(a); }
TBG_DEV Fp2x f_mulc(const Fp2x& a, const Fp2Const& c) { return px_mul_const(a, c); }
// (specialisations keep the primary templates' __host__ __device__; only the
// device body is ever instantiated)
template <> TBG_HD Fp2x f_zero<Fp2x>() { return {fp_zero()}; }
template <> TBG_HD Fp2x f_one<Fp2x>() {
#if defined(__HIP_DEVICE_COMPILE__)
  return {(threadIdx.x & 1u) ? fp_zero() : fp_one()};
#else
  return {fp_one()};
#endif
}

// this lane's component of a stored Fp2 / G2 point, and back
TBG_DEV Fp2x px_load(const Fp2& a) { return {(&a.c0)[pair_par()]}; }
TBG_DEV void px_store(Fp2& dst, const Fp2x& a) { (&dst.c0)[pair_par()] = a.v; }
TBG_DEV Aff<Fp2x> px_load(const G2A& a) { return {px_load(a.x), px_load(a.y)}; }
TBG_DEV Jac<Fp2x> px_load(const G2J& p) { return {px_load(p.X), px_load(p.Y), px_load(p.Z)}; }
TBG_DEV void px_store(G2A& dst, const Aff<Fp2x>& a) { px_store(dst.x, a.x); px_store(dst.y, a.y); }
TBG_DEV void px_store(G2J& dst, const Jac<Fp2x>& p) { px_store(dst.X, p.X); px_store(dst.Y, p.Y); px_store(dst.Z, p.Z); }
// One Miller line in the engine's layout [l0.c0, l0.c1, l1.c0, l1.c1, l4.c0,
// l4.c1] (NL words each, bls_lines.h): each lane writes its components.
TBG_DEV void px_line_store(uint32_t* dst, const LineG<Fp2x>& l) {
  const uint32_t par = pair_par();
  const Fp* f[3] = {&l.l0.v, &l.l1.v, &l.l4.v};
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int i = 0; i < NL; ++i) dst[(2 * k + par) * NL + i] = f[k]->l[i];
}

// All 68 lines of Q in loop order (g2_lines_t), Fp2 split over the pair;
// EVAL = false: P left out (nxP, yP unused).
// (each coefficient stored as the step forms it)
template <bool EVAL = true>
TBG_DEV void px_g2_lines(const Aff<Fp2x>& Q, const Fp& nxP, const Fp& yP, uint32_t* out) {
  Jac<Fp2x> T = jac_from_aff(Q);
  const uint32_t par = pair_par();
  uint32_t* dst = out;
  auto sink = [&](int k, const Fp2x& v) {
#pragma unroll
    for (int i = 0; i < NL; ++i) dst[(2 * k + par) * NL + i] = v.v.l[i];
  };
  for (int i = 62; i >= 0; --i) {
    miller_dbl_s<Fp2x, EVAL>(T, nxP, yP, sink);
    dst += LINE_WORDS;
    if ((X_ABS >> i) & 1) {
      miller_add_s<Fp2x, EVAL>(T, Q, nxP, yP, sink);
      dst += LINE_WORDS;
    }
  }
}

// the whole Fp2 on both lanes
TBG_DEV Fp2 px_gather(const Fp2x& a) {
  const Fp o = pair_xch(a.v);
  return pair_par() ? Fp2{o, a.v} : Fp2{a.v, o};
}

}  // namespace tbg
#endif
