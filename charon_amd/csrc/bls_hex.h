// Hexad Fp12: one Fp12 per SIX lanes -- the trio of bls_quad.h with every Fp2
// split over a lane pair (bls_pair.h), so the per-lane state halves.
//
// Why: the level-0 Miller-chunk kernel in the trio layout needs ~450 VGPRs
// per lane (f = one Fp4 = 56 VGPRs, the Fp4 products and the streamed line
// values on top), so it runs at ONE wave per SIMD, where gfx950 issues
// v_mad_u64_u32 at ~58 % of the two-wave rate (profiles/r02/valu_rates.txt):
// 0.49 of the VALU peak was its ceiling.  A hexad lane holds
// one COMPONENT of its trio lane's Fp4 (a_c, b_c: 28 VGPRs) and computes
// component c of every Fp2 product as one REDC(ab + cd) -- the same
// multiply count per Fp12 as the trio (half per lane, twice the lanes) at
// half the live state, so the kernel fits 256 VGPRs: two waves per SIMD.
//
// Layout: trio lane q = (lane & 15) % 3 as in bls_quad.h (5 trios per DPP
// row, lane 15 idle); component c = (lane >> 4) & 1 (rows 0 and 2 hold c0,
// rows 1 and 3 c1, partner = lane ^ 16, one ds_swizzle per word).  Trio
// exchanges stay DPP row shifts on the own component.  A wave carries 10 Fp12 values (60 of 64 lanes work).
//
// Cross-component terms (the multiplications by xi = 1 + u hidden in the
// Fp4 / Fp12 algebra) need the partner's component of ONE value per
// operation, so each product or squaring swaps its operand once (for the
// pair products) and one intermediate (for the xi term).
//
// The per-lane pieces are plain functions of (c, q, own, partner, ...) so
// the host build checks the algebra by emulating the six lanes
// (tests/hostcheck: hc_hex_*), against the tower and the trio.
#pragma once
#include "bls_quad.h"
#include "bls_pair.h"

namespace tbg {

struct Fp4h { Fp a, b; };  // component c of a trio lane's A_q = (a, b)
// An Fp2 as lane c sees it: its own component o = x_c and its partner's p =
// x_(1-c).  Products and linear maps work on this form directly, so no lane
// ever selects components out of a whole Fp2 (per-limb selects cost as much
// as a tenth of a product each).
struct Fp2o { Fp o, p; };
struct Fp4o { Fp2o a, b; };

TBG_HD Fp4h hx_select(bool k, const Fp4h& x, const Fp4h& y) { return {fp_select(k, x.a, y.a), fp_select(k, x.b, y.b)}; }
TBG_HD Fp2o hx_add(const Fp2o& x, const Fp2o& y) { return {fp_add(x.o, y.o), fp_add(x.p, y.p)}; }
// lazy (bls_field.h): for the FIRST operand of hx_mul only
TBG_HD Fp2o hx_add_l(const Fp2o& x, const Fp2o& y) { return {fp_add_l(x.o, y.o), fp_add_l(x.p, y.p)}; }
// xi x = (x0 - x1) + (x0 + x1) u seen from lane c (lazy: < x + 16p)
// (lazy limbs: only ever the first operand of a lazy sum that feeds hx_mul's
// first operand)
TBG_HD Fp2o hx_mul_xi(uint32_t c, const Fp2o& x) {
  const Fp s = fp_add_l(x.o, x.p), d0 = fp_sub_l(x.o, x.p), d1 = fp_sub_l(x.p, x.o);
  return {fp_select(c != 0, s, d0), fp_select(c != 0, d1, s)};
}
// component c of x y (one REDC(ab + cd)); x < 32p, y's partner < 16p
TBG_HD Fp hx_mul(uint32_t c, const Fp2o& x, const Fp2o& y) { return pair_mul_lane(c, x.o, x.p, y.o, y.p); }
// component c of xi x from x's own / partner components (lazy: < x0 + 16p)
// (lazy limbs: every use feeds a lazy sum into fp_reduce)
TBG_HD Fp hx_xi(uint32_t c, const Fp& own, const Fp& par) {
  return fp_select(c != 0, fp_add_l(own, par), fp_sub_l(own, par));
}
// host tests: lane c's view of a whole value
TBG_HD Fp2o hx_view(uint32_t c, const Fp2& x) { return c ? Fp2o{x.c1, x.c0} : Fp2o{x.c0, x.c1}; }
TBG_HD Fp4o hx_view4(uint32_t c, const Fp4& x) { return {hx_view(c, x.a), hx_view(c, x.b)}; }

// ---- fp4_sqr(x) = {a^2 + xi b^2, 2ab} in two phases around one exchange
// phase 1: component c of ab and s = (a + xi b)(a + b)
// (the lazy a + xi b, up to 24p, as the left operand: pair_mul_lane negates
// the right one's partner component, which must stay < 16p)
TBG_HD void hx_sqr1(uint32_t c, const Fp4o& x, Fp& ab, Fp& s) {
  ab = hx_mul(c, x.a, x.b);
  s = hx_mul(c, hx_add_l(x.a, hx_mul_xi(c, x.b)), hx_add(x.a, x.b));
}
// phase 2 (ab's partner component abp): component c of {t0, reduce(t1)}
TBG_HD Fp4h hx_sqr2(uint32_t c, const Fp& ab, const Fp& abp, const Fp& s) {
  const Fp u = fp_reduce(fp_add_l(hx_xi(c, ab, abp), ab));
  return {fp_reduce(fp_sub_l(s, u)), fp_reduce(fp_add_l(ab, ab))};
}

// ---- quad_combine for component c.  Phase 1: T and V, the value whose xi
// multiple enters C.a (T.b on lane 0, Pn.b on lane 1); phase 2 with V's
// partner component.
TBG_HD void hx_comb1(int q, const Fp4h& P, const Fp4h& Pn, const Fp4h& Pp, const Fp4h& Qx, Fp4h& T, Fp& V) {
  const Fp4h f1 = hx_select(q == 1, Pp, Pn);
  const Fp4h f2 = hx_select(q == 0, Pp, P);
  T = {fp_reduce(fp_sub_l(Qx.a, fp_add(f1.a, f2.a))), fp_reduce(fp_sub_l(Qx.b, fp_add(f1.b, f2.b)))};
  V = fp_select(q == 0, T.b, Pn.b);
}
TBG_HD Fp4h hx_comb2(uint32_t c, int q, const Fp4h& P, const Fp4h& Pn, const Fp4h& Pp, const Fp4h& T, const Fp& V,
                     const Fp& Vp) {
  const Fp xv = fp_reduce(hx_xi(c, V, Vp));
  // q = 0: (xv + P.a, T.a + P.b); q = 1: (T.a + xv, T.b + Pn.a); q = 2: (T.a + Pp.a, T.b + Pp.b)
  const Fp x0 = fp_select(q == 0, xv, T.a);
  const Fp y0 = fp_select(q == 0, P.a, fp_select(q == 1, xv, Pp.a));
  const Fp x1 = fp_select(q == 0, T.a, T.b);
  const Fp y1 = fp_select(q == 0, P.b, fp_select(q == 1, Pn.a, Pp.b));
  return {fp_reduce(fp_add_l(x0, y0)), fp_reduce(fp_add_l(x1, y1))};
}

// ---- f * line, line = L0 + L2 x^2 with L0 = (l0, l4), L2 = l1 (evaluated):
//   C_q = A_q L0 + (q < 2 ? y : 1) A_{q+1} l1   (quad_line_lane)
// phase 1: the five products' components and W, the value whose xi multiple
// enters C.a (t1, plus u.b on lanes 0, 1)
struct HxLine { Fp t0, t1, s, ua, ub, W; };
TBG_HD void hx_line_u(uint32_t c, const Fp4o& An, const Fp2o& l1, HxLine& r) {
  r.ua = hx_mul(c, An.a, l1);
  r.ub = hx_mul(c, An.b, l1);
}
TBG_HD void hx_line_t(uint32_t c, int q, const Fp4o& A, const Fp2o& l0, const Fp2o& l4, HxLine& r) {
  r.t0 = hx_mul(c, A.a, l0);
  r.t1 = hx_mul(c, A.b, l4);
  r.s = hx_mul(c, hx_add_l(A.a, A.b), hx_add(l0, l4));
  r.W = fp_add(r.t1, fp_select(q < 2, r.ub, fp_zero()));
}
// phase 2 (W's partner component Wp)
TBG_HD Fp4h hx_line2(uint32_t c, int q, const HxLine& r, const Fp& Wp) {
  const Fp xw = hx_xi(c, r.W, Wp);                                 // < 20p
  const Fp ca = fp_reduce(fp_add_l(fp_add_l(xw, r.t0), fp_select(q < 2, fp_zero(), r.ua)));
  const Fp c1 = fp_sub_l(r.s, fp_add(r.t0, r.t1));                 // < 18p
  return {ca, fp_reduce(fp_add_l(c1, fp_select(q < 2, r.ua, r.ub)))};
}

// ---- fp4_mul(x, y) = (x.a y.a + xi x.b y.b, (x.a + x.b)(y.a + y.b) - x.a y.a
// - x.b y.b), the trio's Karatsuba over Fp4, in two phases around one exchange.
// phase 1: component c of t0 = x.a y.a, t1 = x.b y.b, s = (x.a + x.b)(y.a + y.b)
TBG_HD void hx_mul1(uint32_t c, const Fp4o& x, const Fp4o& y, Fp& t0, Fp& t1, Fp& s) {
  t0 = hx_mul(c, x.a, y.a);
  t1 = hx_mul(c, x.b, y.b);
  s = hx_mul(c, hx_add_l(x.a, x.b), hx_add(y.a, y.b));
}
// phase 2 (t1's partner component t1p)
TBG_HD Fp4h hx_mul2(uint32_t c, const Fp& t0, const Fp& t1, const Fp& t1p, const Fp& s) {
  return {fp_reduce(fp_add_l(hx_xi(c, t1, t1p), t0)), fp_reduce(fp_sub_l(s, fp_add(t0, t1)))};
}

// ---- cyclotomic squaring (quad_cyc_lane) for component c: Tx = fp4_sqr of
// trio lane {0, 2, 1}[q]'s coefficient, Txbp = the partner component of Tx.b
TBG_HD Fp4h hx_cyc(uint32_t c, int q, const Fp4h& A, const Fp4h& Tx, const Fp& Txbp) {
  const Fp s1 = fp_select(q == 1, fp_reduce(hx_xi(c, Tx.b, Txbp)), Tx.a);
  const Fp s2 = fp_select(q == 1, Tx.a, Tx.b);
  const Fp a2 = fp_add(A.a, A.a), b2 = fp_add(A.b, A.b);
  const Fp s13 = fp_mul_small(s1, 3), s23 = fp_mul_small(s2, 3);
  const Fp na = fp_select(q == 1, fp_add_l(s13, a2), fp_sub_l(s13, a2));
  const Fp nb = fp_select(q == 1, fp_sub_l(s23, b2), fp_add_l(s23, b2));
  return {fp_reduce(na), fp_reduce(nb)};
}

// ---- conj (w -> -w: negate a_1, a_3, a_5), component-wise
TBG_HD Fp4h hx_conj(int q, const Fp4h& A) {
  const Fp na = fp_reduce(fp_neg(A.a)), nb = fp_reduce(fp_neg(A.b));
  return {fp_select(q == 1, na, A.a), fp_select(q == 1, A.b, nb)};
}

// ---- Frobenius (quad_frob_lane): a_k -> conj(a_k) gamma_k, with the
// partner components Ap of A
TBG_HD Fp2o hx_conj_view(uint32_t c, const Fp& own, const Fp& par) {
  const Fp no = fp_reduce(fp_neg(own)), np = fp_reduce(fp_neg(par));
  return {fp_select(c != 0, no, own), fp_select(c != 0, par, np)};  // conj(x) = (x0, -x1)
}
TBG_HD Fp2o hx_const_view(uint32_t c, const Fp2& k) { return {fp_select(c != 0, k.c1, k.c0), fp_select(c != 0, k.c0, k.c1)}; }
TBG_HD Fp4h hx_frob(uint32_t c, int q, const Fp4h& A, const Fp4h& Ap) {
  const Fp2 ga = fp2_select(q == 0, fp2_one(), fp2_select(q == 1, fp2_from_const(FROB_G1), fp2_from_const(FROB_G2)));
  const Fp2 gb = fp2_select(q == 0, fp2_from_const(FROB_G3),
                            fp2_select(q == 1, fp2_from_const(FROB_G4), fp2_from_const(FROB_G5)));
  return {hx_mul(c, hx_conj_view(c, A.a, Ap.a), hx_const_view(c, ga)),
          hx_mul(c, hx_conj_view(c, A.b, Ap.b), hx_const_view(c, gb))};
}

// this lane's part of "the element is 1": b = 0, a = 1 on (q, c) = (0, 0), 0 elsewhere
TBG_HD bool hx_is_one_lane(uint32_t c, int q, const Fp4h& A) {
  const bool a_one = fp_eq(A.a, fp_one()), a_zero = fp_is_zero(A.a);
  return fp_is_zero(A.b) && ((q == 0 && c == 0) ? a_one : a_zero);
}

}  // namespace tbg

// ---------------------------------------------------------------------------
// Device: the hexad as lanes of a wave.
#if defined(__HIP__)
namespace tbg {

// Where the component partner sits: rows 0 / 1 (and 2 / 3) of the wave hold
// components 0 / 1 of the same five trios, the partner is lane ^ 16, and the
// exchange is ONE ds_swizzle (the LDS crossbar in xor mode, no LDS memory)
// per word.  (Halves of the wave with v_permlane32_swap took a copy and a
// per-half select besides -- 3 VALU instructions per word; measured slower,
// round 4: profiles/r04/lazy/; removed.)
// Fp12 slot of global thread t (UINT32_MAX for lane 15 of a row), and the
// threads n slots need: 10 per wave.
TBG_HD uint32_t hex_slot(uint32_t t) {
  const uint32_t l = t & 15u;
  return l == 15u ? 0xFFFFFFFFu : (t >> 6) * 10u + ((t >> 5) & 1u) * 5u + l / 3u;
}
inline uint32_t hex_threads(uint32_t n) { return 64u * ((n + 9u) / 10u); }
TBG_DEV uint32_t hex_c() { return (threadIdx.x >> 4) & 1u; }
// lane (q, c) = (0, 0) of this thread's hexad: the one that takes list slots
// and writes per-entry verdicts
TBG_DEV bool hex_lead() { return quad_lane() == 0 && hex_c() == 0; }
TBG_DEV uint32_t hex_lead_lane() { return (threadIdx.x - (uint32_t)quad_lane()) & ~16u; }
// hexad kernels fit 256 VGPRs: two waves per SIMD
#ifndef TBG_HEX_WAVES
#define TBG_HEX_WAVES 2
#endif

// the partner lane's value: ds_swizzle bitmask mode within 32-lane groups
// (and 0x1f, or 0, xor 0x10 -> lane ^ 16)
TBG_DEV uint32_t hx_swap_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F); }
TBG_DEV Fp hx_swap(const Fp& x) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = hx_swap_u32(x.l[i]);
  return r;
}
TBG_DEV Fp4h hx_swap(const Fp4h& x) { return {hx_swap(x.a), hx_swap(x.b)}; }
template <int K>
TBG_DEV Fp4h hxch(const Fp4h& x) { return {xch<K>(x.a), xch<K>(x.b)}; }

TBG_DEV Fp4h hex_one() {
  Fp4h r = {fp_zero(), fp_zero()};
  if (quad_lane() == 0 && hex_c() == 0) r.a = fp_one();
  return r;
}

TBG_DEV Fp4o hx_own_par(const Fp4h& own, const Fp4h& par) { return {{own.a, par.a}, {own.b, par.b}}; }

// f^2 (quad_sqr_in on the hexad)
TBG_DEV Fp4h hex_sqr(const Fp4h& A) {
  const uint32_t c = hex_c();
  const int q = quad_lane();
  Fp ab, s;
  hx_sqr1(c, hx_own_par(A, hx_swap(A)), ab, s);
  const Fp4h P = hx_sqr2(c, ab, hx_swap(ab), s);
  const Fp4h SA = {fp_add(xch<QP_NEXT>(A.a), xch<QP_PREV>(A.a)), fp_add(xch<QP_NEXT>(A.b), xch<QP_PREV>(A.b))};
  hx_sqr1(c, hx_own_par(SA, hx_swap(SA)), ab, s);
  const Fp4h Q = hx_sqr2(c, ab, hx_swap(ab), s);
  const Fp4h Pn = hxch<QP_NEXT>(P), Pp = hxch<QP_PREV>(P), Qx = hxch<QP_SW12>(Q);
  Fp4h T;
  Fp V;
  hx_comb1(q, P, Pn, Pp, Qx, T, V);
  return hx_comb2(c, q, P, Pn, Pp, T, V, hx_swap(V));
}

// f * (l0, l1, l4) in the order that keeps the live set small: the two
// A_{q+1} l1 products first (A_{q+1}'s partner components by a swap of the
// exchanged own ones), then A_q (l0, l4) with l0 loaded only then
// (`l0_src`: the line's first 2 NL words, or null with l0 given)
TBG_DEV Fp4h hex_line_mul(const Fp4h& A, const uint32_t* l0_src, Fp2o l0, const Fp2o& l1, const Fp2o& l4) {
  const uint32_t c = hex_c();
  const int q = quad_lane();
  HxLine r;
  {
    const Fp4h An = hxch<QP_NEXT>(A);
    hx_line_u(c, hx_own_par(An, hx_swap(An)), l1, r);
  }
  if (l0_src) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      l0.o.l[i] = l0_src[c * NL + i];
      l0.p.l[i] = l0_src[(c ^ 1u) * NL + i];
    }
  }
  hx_line_t(c, q, hx_own_par(A, hx_swap(A)), l0, l4, r);
  return hx_line2(c, q, r, hx_swap(r.W));
}

// f *= line(idx) of stored (unevaluated) lines at affine P = (-x, y): lane
// (0, c) evaluates l1_c (-x), lane (1, c) l4_c y; the trio broadcasts them
// and the pair swaps the other components.  `v` is this lane's operand:
// -x on q = 0, y on q = 1 (q = 2: any, its product is not used).
TBG_DEV Fp4h hex_line_at_v(const Fp4h& A, const uint32_t* lines, int idx, const Fp& v) {
  const uint32_t c = hex_c();
  const int q = quad_lane();
  const uint32_t* src = lines + LINE_WORDS * idx;
  Fp lk;
  const int k = q == 0 ? 2 : 4;
#pragma unroll
  for (int i = 0; i < NL; ++i) lk.l[i] = src[(k + (int)c) * NL + i];
  const Fp e = fp_mul(lk, v);
  const Fp e1 = xch<QP_B0>(e), e4 = xch<QP_B1>(e);
  return hex_line_mul(A, src, Fp2o{}, Fp2o{e1, hx_swap(e1)}, Fp2o{e4, hx_swap(e4)});
}
TBG_DEV Fp4h hex_line_at(const Fp4h& A, const uint32_t* lines, int idx, const Fp& nx, const Fp& y) {
  return hex_line_at_v(A, lines, idx, fp_select(quad_lane() == 0, nx, y));
}
// this lane's evaluation operand of a point stored as (-x, y) (one Fp loaded)
TBG_DEV Fp hex_line_operand(const G1A& P) { return quad_lane() == 0 ? P.x : P.y; }
// f *= line(idx) of folded (already evaluated) lines
TBG_DEV Fp4h hex_line_folded(const Fp4h& A, const uint32_t* lines, int idx) {
  const uint32_t c = hex_c();
  const uint32_t* src = lines + LINE_WORDS * idx;
  Fp2o l[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      l[k].o.l[i] = src[(2 * k + (int)c) * NL + i];
      l[k].p.l[i] = src[(2 * k + (int)(c ^ 1u)) * NL + i];
    }
  return hex_line_mul(A, nullptr, l[0], l[1], l[2]);
}

// x y (quad_mul_in on the hexad)
TBG_DEV Fp4h hex_mul(const Fp4h& A, const Fp4h& B) {
  const uint32_t c = hex_c();
  const int q = quad_lane();
  Fp t0, t1, s;
  hx_mul1(c, hx_own_par(A, hx_swap(A)), hx_own_par(B, hx_swap(B)), t0, t1, s);
  const Fp4h P = hx_mul2(c, t0, t1, hx_swap(t1), s);
  const Fp4h SA = {fp_add(xch<QP_NEXT>(A.a), xch<QP_PREV>(A.a)), fp_add(xch<QP_NEXT>(A.b), xch<QP_PREV>(A.b))};
  const Fp4h SB = {fp_add(xch<QP_NEXT>(B.a), xch<QP_PREV>(B.a)), fp_add(xch<QP_NEXT>(B.b), xch<QP_PREV>(B.b))};
  hx_mul1(c, hx_own_par(SA, hx_swap(SA)), hx_own_par(SB, hx_swap(SB)), t0, t1, s);
  const Fp4h Q = hx_mul2(c, t0, t1, hx_swap(t1), s);
  const Fp4h Pn = hxch<QP_NEXT>(P), Pp = hxch<QP_PREV>(P), Qx = hxch<QP_SW12>(Q);
  Fp4h T;
  Fp V;
  hx_comb1(q, P, Pn, Pp, Qx, T, V);
  return hx_comb2(c, q, P, Pn, Pp, T, V, hx_swap(V));
}

// cyclotomic squaring (quad_cyc_sqr_in on the hexad)
TBG_DEV Fp4h hex_cyc_sqr(const Fp4h& A) {
  const uint32_t c = hex_c();
  Fp ab, s;
  hx_sqr1(c, hx_own_par(A, hx_swap(A)), ab, s);
  const Fp4h T = hx_sqr2(c, ab, hx_swap(ab), s);
  const Fp4h Tx = hxch<QP_SW12>(T);
  return hx_cyc(c, quad_lane(), A, Tx, hx_swap(Tx.b));
}

TBG_DEV Fp4h hex_conj(const Fp4h& A) { return hx_conj(quad_lane(), A); }
TBG_DEV Fp4h hex_frob(const Fp4h& A) { return hx_frob(hex_c(), quad_lane(), A, hx_swap(A)); }

// true on all six lanes iff the hexad's element is 1
TBG_DEV bool hex_is_one(const Fp4h& A) {
  uint32_t v = hx_is_one_lane(hex_c(), quad_lane(), A) ? 1u : 0u;
  v &= hx_swap_u32(v);
  return (xch_u32<QP_B0>(v) & xch_u32<QP_B1>(v) & xch_u32<QP_B2>(v)) != 0;
}

// f^-1: the whole element gathered on every lane, the tower inverse, this
// lane's components back -- out of line (rare: once per final
// exponentiation).  (Inline, as conj(f) (f conj(f))^-1 with the Fp6 inverse
// of the norm, the check kernels fit two waves per SIMD and ran 17 % faster
// alone but 9 % slower in the pipelined 1 %-invalid run; round 4,
// profiles/r04/hexinv/.)
__device__ __noinline__ Fp4h hex_inv_ni(const Fp4h& A) {
  const uint32_t c = hex_c();
  const Fp4h Ap = hx_swap(A);
  auto whole = [&](const Fp4h& own, const Fp4h& par) -> Fp4 {
    return {{fp_select(c != 0, par.a, own.a), fp_select(c != 0, own.a, par.a)},
            {fp_select(c != 0, par.b, own.b), fp_select(c != 0, own.b, par.b)}};
  };
  const Fp4 A0 = whole(hxch<QP_B0>(A), hxch<QP_B0>(Ap)), A1 = whole(hxch<QP_B1>(A), hxch<QP_B1>(Ap)),
            A2 = whole(hxch<QP_B2>(A), hxch<QP_B2>(Ap));
  const Fp4 r = quad_from_fp12(quad_lane(), fp12_inv(quad_to_fp12(A0, A1, A2)));
  return {fp_select(c != 0, r.a.c1, r.a.c0), fp_select(c != 0, r.b.c1, r.b.c0)};
}

// a^|x| in the cyclotomic subgroup, and the final exponentiation f^(3 (p^12
// - 1) / r) in quad_final_exp's sequence (kernel-inline squarings; the rare
// products, inversions and Frobenius maps stay calls)
__device__ __noinline__ Fp4h hex_mul_ni(const Fp4h& A, const Fp4h& B) { return hex_mul(A, B); }
__device__ __noinline__ Fp4h hex_frob_ni(const Fp4h& A) { return hex_frob(A); }
TBG_DEV Fp4h hex_pow_xabs_in(const Fp4h& a) {
  Fp4h r = a;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    r = hex_cyc_sqr(r);
    if ((X_ABS >> i) & 1) r = hex_mul_ni(r, a);
  }
  return r;
}
TBG_DEV Fp4h hex_pow_x_in(const Fp4h& a) { return hex_conj(hex_pow_xabs_in(a)); }
TBG_DEV Fp4h hex_final_exp_in(const Fp4h& f) {
  Fp4h t = hex_mul_ni(hex_conj(f), hex_inv_ni(f));
  t = hex_mul_ni(hex_frob_ni(hex_frob_ni(t)), t);
  Fp4h a = hex_mul_ni(hex_pow_x_in(t), hex_conj(t));
  a = hex_mul_ni(hex_pow_x_in(a), hex_conj(a));
  Fp4h b = hex_mul_ni(hex_pow_x_in(a), hex_frob_ni(a));
  Fp4h c = hex_mul_ni(hex_pow_x_in(hex_pow_x_in(b)), hex_frob_ni(hex_frob_ni(b)));
  c = hex_mul_ni(c, hex_conj(b));
  Fp4h t3 = hex_mul_ni(hex_cyc_sqr(t), t);
  return hex_mul_ni(c, t3);
}

// quad layout in HBM, read: lane (q, c) loads its two components
TBG_DEV Fp4h hex_load(const uint32_t* src) {
  const int q = quad_lane();
  const uint32_t c = hex_c();
  Fp4h A;
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    A.a.l[j] = src[4 * NL * q + c * NL + j];
    A.b.l[j] = src[4 * NL * q + (2 + c) * NL + j];
  }
  return A;
}

// quad layout in HBM (bls_quad.h / k_rlc.hip QUAD_WORDS = 4 NL per trio
// lane, [a.c0, a.c1, b.c0, b.c1]): lane (q, c) writes its two components
TBG_DEV void hex_store(uint32_t* dst, const Fp4h& A) {
  const int q = quad_lane();
  const uint32_t c = hex_c();
#pragma unroll
  for (int j = 0; j < NL; ++j) {
    dst[4 * NL * q + c * NL + j] = A.a.l[j];
    dst[4 * NL * q + (2 + c) * NL + j] = A.b.l[j];
  }
}

}  // namespace tbg
#endif
