// G1 (over Fp) and G2 (over Fp2) group law in Jacobian coordinates,
// ZCash compressed (de)serialisation and subgroup checks.
//
// Curve: E1: y^2 = x^3 + 4, E2: y^2 = x^3 + 4(1 + u).  The point at infinity
// is any triple with Z = 0.  Every public function returns coordinates < 2p.
// Decoding follows the ZCash format used by kryptology's G2.FromCompressed
// (reached from reference tbls/tblsconv/tblsconv.go:90-132 and
// eth2util/signing/signing.go:154-161).
#pragma once
#include "bls_tower.h"

namespace tbg {

// ---- overload set so the group law can be written once for Fp and Fp2 ----
TBG_HD Fp f_add(const Fp& a, const Fp& b) { return fp_add(a, b); }
TBG_HD Fp2 f_add(const Fp2& a, const Fp2& b) { return fp2_add(a, b); }
TBG_HD Fp f_sub(const Fp& a, const Fp& b) { return fp_sub(a, b); }
TBG_HD Fp2 f_sub(const Fp2& a, const Fp2& b) { return fp2_sub(a, b); }
// Lazy sum / difference (limbs left unnormalised, bls_field.h): for results
// that only feed f_reduce, the FIRST operand of f_mul / f_mulfp / f_mulc, the
// first operand of f_sub(_l) or f_small -- never f_sqr (its lane pieces
// subtract the operand's halves), the second operand of f_mul (negated) or
// of a subtraction, or a stored coordinate.
TBG_HD Fp f_add_l(const Fp& a, const Fp& b) { return fp_add_l(a, b); }
TBG_HD Fp2 f_add_l(const Fp2& a, const Fp2& b) { return {fp_add_l(a.c0, b.c0), fp_add_l(a.c1, b.c1)}; }
TBG_HD Fp f_sub_l(const Fp& a, const Fp& b) { return fp_sub_l(a, b); }
TBG_HD Fp2 f_sub_l(const Fp2& a, const Fp2& b) { return {fp_sub_l(a.c0, b.c0), fp_sub_l(a.c1, b.c1)}; }
TBG_HD Fp f_neg(const Fp& a) { return fp_neg(a); }
TBG_HD Fp2 f_neg(const Fp2& a) { return fp2_neg(a); }
TBG_HD Fp f_mul(const Fp& a, const Fp& b) { return fp_mul(a, b); }
TBG_HD Fp2 f_mul(const Fp2& a, const Fp2& b) { return fp2_mul(a, b); }
TBG_HD Fp f_sqr(const Fp& a) { return fp_sqr(a); }
TBG_HD Fp2 f_sqr(const Fp2& a) { return fp2_sqr(a); }
TBG_HD Fp f_reduce(const Fp& a) { return fp_reduce(a); }
TBG_HD Fp2 f_reduce(const Fp2& a) { return fp2_reduce(a); }
TBG_HD bool f_is_zero(const Fp& a) { return fp_is_zero(a); }
TBG_HD bool f_is_zero(const Fp2& a) { return fp2_is_zero(a); }
TBG_HD bool f_eq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
TBG_HD bool f_eq(const Fp2& a, const Fp2& b) { return fp2_eq(a, b); }
TBG_HD Fp f_inv(const Fp& a) { return fp_inv(a); }
TBG_HD Fp2 f_inv(const Fp2& a) { return fp2_inv(a); }
TBG_HD Fp f_small(const Fp& a, uint32_t k) { return fp_mul_small(a, k); }
TBG_HD Fp2 f_small(const Fp2& a, uint32_t k) { return fp2_mul_small(a, k); }
template <class F> TBG_HD F f_zero();
template <> TBG_HD Fp f_zero<Fp>() { return fp_zero(); }
template <> TBG_HD Fp2 f_zero<Fp2>() { return fp2_zero(); }
template <class F> TBG_HD F f_one();
template <> TBG_HD Fp f_one<Fp>() { return fp_one(); }
template <> TBG_HD Fp2 f_one<Fp2>() { return fp2_one(); }

template <class F> struct Jac { F X, Y, Z; };
template <class F> struct Aff { F x, y; };
using G1J = Jac<Fp>;
using G2J = Jac<Fp2>;
using G1A = Aff<Fp>;
using G2A = Aff<Fp2>;

template <class F> TBG_HD Jac<F> jac_inf() { return {f_one<F>(), f_one<F>(), f_zero<F>()}; }
template <class F> TBG_HD bool jac_is_inf(const Jac<F>& p) { return f_is_zero(p.Z); }
template <class F> TBG_HD Jac<F> jac_from_aff(const Aff<F>& a) { return {a.x, a.y, f_one<F>()}; }
template <class F> TBG_HD Jac<F> jac_neg(const Jac<F>& p) { return {p.X, f_reduce(f_neg(p.Y)), p.Z}; }

template <class F> TBG_NI Jac<F> jac_dbl(const Jac<F>& p);

// dbl-2009-l (a = 0). Inputs < 2p, outputs < 2p.
template <class F> TBG_HD Jac<F> jac_dbl_in(const Jac<F>& p) {
  F A = f_sqr(p.X);
  F B = f_sqr(p.Y);
  F C = f_sqr(B);
  F t = f_sub_l(f_sqr(f_add(p.X, B)), f_add(A, C));   // < 18p
  F D = f_reduce(f_add_l(t, t));
  F E = f_small(A, 3);                                // < 6p
  F Fv = f_sqr(E);
  F X3 = f_reduce(f_sub_l(Fv, f_add(D, D)));
  F Y3 = f_reduce(f_sub_l(f_mul(f_sub_l(D, X3), E), f_small(C, 8)));  // bigger operand first (fp2_mul negates b.c1)
  F YZ = f_mul(p.Y, p.Z);
  F Z3 = f_reduce(f_add_l(YZ, YZ));
  return {X3, Y3, Z3};
}

// TBG_ADD_DBL_INLINE=1: the P == Q case doubles inline (no out-of-line call
// in the caller's loop, whose live registers would otherwise be saved around
// the call site).
#if defined(TBG_ADD_DBL_INLINE) && TBG_ADD_DBL_INLINE
#define TBG_ADD_DBL(p) jac_dbl_in(p)
#else
#define TBG_ADD_DBL(p) jac_dbl(p)
#endif

// add-2007-bl with the exceptional cases handled (P == Q, P == -Q, infinity).
// INLDBL = true doubles inline in the P == Q case (no out-of-line call in the
// caller's loop; see TBG_ADD_DBL below).
template <class F, bool INLDBL = false> TBG_HD Jac<F> jac_add_in(const Jac<F>& p, const Jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = f_sqr(p.Z);
  F Z2Z2 = f_sqr(q.Z);
  F U1 = f_mul(p.X, Z2Z2);
  F U2 = f_mul(q.X, Z1Z1);
  F S1 = f_mul(f_mul(p.Y, q.Z), Z2Z2);
  F S2 = f_mul(f_mul(q.Y, p.Z), Z1Z1);
  F H = f_reduce(f_sub_l(U2, U1));
  F Rr = f_reduce(f_sub_l(S2, S1));
  if (f_is_zero(H)) {
    if (f_is_zero(Rr)) return INLDBL ? jac_dbl_in(p) : jac_dbl(p);
    return jac_inf<F>();
  }
  F H2 = f_add(H, H);
  F I = f_sqr(H2);
  F J = f_mul(H, I);
  F r2 = f_add(Rr, Rr);
  F V = f_mul(U1, I);
  F X3 = f_reduce(f_sub_l(f_sub_l(f_sqr(r2), J), f_add(V, V)));
  F Y3 = f_reduce(f_sub_l(f_mul(f_sub_l(V, X3), r2), f_small(f_mul(S1, J), 2)));
  F Zs = f_sub_l(f_sqr(f_add(p.Z, q.Z)), f_add(Z1Z1, Z2Z2));   // < 18p
  F Z3 = f_mul(f_reduce(Zs), H);
  return {X3, Y3, Z3};
}

// Mixed addition P (Jacobian) + Q (affine), exceptional cases handled.
template <class F> TBG_HD Jac<F> jac_add_aff_in(const Jac<F>& p, const Aff<F>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  F Z1Z1 = f_sqr(p.Z);
  F U2 = f_mul(q.x, Z1Z1);
  F S2 = f_mul(f_mul(q.y, p.Z), Z1Z1);
  F H = f_reduce(f_sub_l(U2, p.X));
  F Rr = f_reduce(f_sub_l(S2, p.Y));
  if (f_is_zero(H)) {
    if (f_is_zero(Rr)) return TBG_ADD_DBL(p);
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

// Out-of-line forms (one copy of the code; struct arguments travel through
// the scratch stack).  Kernels call the _in bodies from their own loops so
// the operands stay in registers (see TBG_NI in bls_field.h).
template <class F> TBG_NI Jac<F> jac_dbl(const Jac<F>& p) { return jac_dbl_in(p); }
template <class F> TBG_NI Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) { return jac_add_in(p, q); }
template <class F> TBG_NI Jac<F> jac_add_aff(const Jac<F>& p, const Aff<F>& q) { return jac_add_aff_in(p, q); }

template <class F> TBG_NI bool jac_to_aff(const Jac<F>& p, Aff<F>& out) {
  if (jac_is_inf(p)) return false;
  F zi = f_inv(p.Z);
  F zi2 = f_sqr(zi);
  out.x = f_mul(p.X, zi2);
  out.y = f_mul(p.Y, f_mul(zi2, zi));
  return true;
}

template <class F> TBG_NI bool jac_eq(const Jac<F>& p, const Jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi || qi) return pi && qi;
  F Z1Z1 = f_sqr(p.Z), Z2Z2 = f_sqr(q.Z);
  if (!f_eq(f_mul(p.X, Z2Z2), f_mul(q.X, Z1Z1))) return false;
  return f_eq(f_mul(f_mul(p.Y, q.Z), Z2Z2), f_mul(f_mul(q.Y, p.Z), Z1Z1));
}

// [k] P for a 64-bit scalar (MSB-first double and add).
template <class F> TBG_NI Jac<F> jac_mul_u64(const Jac<F>& p, uint64_t k) {
  Jac<F> acc = jac_inf<F>();
  bool started = false;
  for (int i = 63; i >= 0; --i) {
    if (started) acc = jac_dbl(acc);
    if ((k >> i) & 1) {
      acc = started ? jac_add(acc, p) : p;
      started = true;
    }
  }
  return acc;
}

// [|x|] P with |x| = 0xd201000000010000 (fixed schedule: 63 doublings, 5 additions).
template <class F> TBG_NI Jac<F> jac_mul_xabs(const Jac<F>& p) {
  Jac<F> acc = p;
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl(acc);
    if ((X_ABS >> i) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

// Same schedule with the doublings and additions inlined into the caller (call
// it from a kernel body only: the loop body is large, see bls_field.h).
template <class F> TBG_HD Jac<F> jac_mul_xabs_in(const Jac<F>& p) {
  Jac<F> acc = p;
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl_in(acc);
    if ((X_ABS >> i) & 1) acc = jac_add_in(acc, p);
  }
  return acc;
}

// Same, with the P == Q case of the additions doubled inline too (no
// out-of-line call anywhere in the loop; the lane-pair kernels need that).
template <class F> TBG_HD Jac<F> jac_mul_xabs_in2(const Jac<F>& p) {
  Jac<F> acc = p;
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl_in(acc);
    if ((X_ABS >> i) & 1) acc = jac_add_in<F, true>(acc, p);
  }
  return acc;
}

// [|x|] P for an affine P, doublings and (mixed) additions inline.
template <class F> TBG_HD Jac<F> jac_mul_xabs_aff_in(const Aff<F>& p) {
  Jac<F> acc = jac_from_aff(p);
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl_in(acc);
    if ((X_ABS >> i) & 1) acc = jac_add_aff_in(acc, p);
  }
  return acc;
}

// [k] P for a multi-word scalar (little-endian 32-bit words, nbits significant).
template <class F> TBG_NI Jac<F> jac_mul_words(const Jac<F>& p, const uint32_t* w, int nbits) {
  Jac<F> acc = jac_inf<F>();
  for (int i = nbits - 1; i >= 0; --i) {
    acc = jac_dbl(acc);
    if ((w[i >> 5] >> (i & 31)) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

// ------------------------------------------------------------------ G2 extra
// psi(x, y) = (conj(x) PSI_X, conj(y) PSI_Y); on Jacobian (conj(X) PSI_X, conj(Y) PSI_Y, conj(Z)).
TBG_HD G2J g2_psi(const G2J& p) {
  G2J r;
  r.X = fp2_mul(fp2_conj(p.X), fp2_from_const(PSI_X));
  r.Y = fp2_mul(fp2_conj(p.Y), fp2_from_const(PSI_Y));
  r.Z = fp2_reduce(fp2_conj(p.Z));
  return r;
}

// Subgroup membership for points on E2 (Scott 2021): P in G2 <=> psi(P) == [x] P.
TBG_HD bool g2_in_subgroup_in(const G2J& p) {
  if (jac_is_inf(p)) return true;
  G2J xp = jac_neg(jac_mul_xabs_in(p));  // [x]P, x < 0
  return jac_eq(g2_psi(p), xp);
}
// Affine input (decode): psi(a) == [x] a == -[|x|] a, compared in Jacobian
// coordinates (X == x' Z^2, Y == -y' Z^3) without leaving the kernel body.
TBG_HD bool g2_in_subgroup_aff_in(const G2A& a) {
  const G2J m = jac_mul_xabs_aff_in(a);  // [|x|] a
  const Fp2 px = fp2_mul(fp2_conj(a.x), fp2_from_const(PSI_X));
  const Fp2 py = fp2_mul(fp2_conj(a.y), fp2_from_const(PSI_Y));
  const Fp2 z2 = fp2_sqr(m.Z);
  const Fp2 z3 = fp2_mul(z2, m.Z);
  if (jac_is_inf(m)) return false;
  return fp2_eq(fp2_mul(px, z2), m.X) && fp2_eq(fp2_mul(py, z3), fp2_reduce(fp2_neg(m.Y)));
}
TBG_NI bool g2_in_subgroup(const G2J& p) {
  if (jac_is_inf(p)) return true;
  G2J xp = jac_neg(jac_mul_xabs(p));  // [x]P, x < 0
  return jac_eq(g2_psi(p), xp);
}

TBG_HD bool g2_on_curve_aff(const G2A& a) {
  Fp2 lhs = fp2_sqr(a.y);
  Fp2 rhs = fp2_add(fp2_mul(fp2_sqr(a.x), a.x), fp2_from_const(B2_M));
  return fp2_eq(lhs, rhs);
}

// Budroni-Pintore cofactor clearing (RFC 9380 G.3):
//   h(P) = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P)
template <bool INL>
TBG_HD G2J g2_clear_cofactor_t(const G2J& p) {
  G2J t1 = jac_neg(INL ? jac_mul_xabs_in(p) : jac_mul_xabs(p));   // [x]P
  G2J t2 = g2_psi(p);                         // psi(P)
  G2J t3 = g2_psi(g2_psi(jac_dbl(p)));        // psi^2(2P)
  t3 = jac_add(t3, jac_neg(t2));
  t2 = jac_add(t1, t2);
  t2 = jac_neg(INL ? jac_mul_xabs_in(t2) : jac_mul_xabs(t2));     // [x](xP + psi P)
  t3 = jac_add(t3, t2);
  t3 = jac_add(t3, jac_neg(t1));
  return jac_add(t3, jac_neg(p));
}
TBG_NI G2J g2_clear_cofactor(const G2J& p) { return g2_clear_cofactor_t<false>(p); }

// ------------------------------------------------------------------ G1 extra
// P in G1 <=> phi(P) == -[x^2] P, phi(x, y) = (beta x, y).
TBG_NI bool g1_in_subgroup(const G1J& p) {
  if (jac_is_inf(p)) return true;
  G1J x2p = jac_mul_xabs(jac_mul_xabs(p));   // [x^2]P (x^2 > 0)
  G1J phi = {fp_mul(p.X, fp_from_const(G1_BETA)), p.Y, p.Z};
  return jac_eq(phi, jac_neg(x2p));
}

// ------------------------------------------------------------ serialisation
enum DecodeStatus : int32_t {
  DEC_OK = 0,
  DEC_IDENTITY = 1,          // valid encoding of the point at infinity
  DEC_ERR_FLAGS = -1,        // compression flag missing / bad infinity encoding
  DEC_ERR_FIELD = -2,        // coordinate >= p
  DEC_ERR_NOT_ON_CURVE = -3,
  DEC_ERR_SUBGROUP = -4,
};

// k_decode_sigs' exponentiation window (the inline root): width 4 spills 71
// VGPRs and still runs 8.37-8.60 vs 8.73-8.89 ms per 640k signatures at width
// 3 (profiles/r06/hash/ab_r6q.txt)
#ifndef TBG_DECODE_WIN
#define TBG_DECODE_WIN 4
#endif

// 96-byte ZCash compressed G2 -> affine (Montgomery).  INL = true runs the
// subgroup check's doublings inline (kernel callers); SUBGROUP = false leaves
// the subgroup check to the caller (k_decode_sigs hands it to the lane-pair
// kernel k_subgroup_sigs, bls_pair.h).  INL also takes the square root
// inline, its input kept by `keep` (bls_tower.h); x goes to out.x before the
// root and is read back from there (a kernel decoding into its output slot
// keeps neither value in registers across the exponentiations).
template <bool INL, bool SUBGROUP = true, class Keep = RegKeep>
TBG_HD int32_t g2_decompress_t(const uint8_t* b, G2A& out, Keep keep = Keep{}) {
  uint32_t c_flag = (b[0] >> 7) & 1, i_flag = (b[0] >> 6) & 1, s_flag = (b[0] >> 5) & 1;
  if (!c_flag) return DEC_ERR_FLAGS;
  uint8_t hi[48];
  for (int j = 0; j < 48; ++j) hi[j] = b[j];
  hi[0] &= 0x1f;
  bool lt1, lt0;
  Fp x1 = fp_limbs_from_be48(hi, &lt1);
  Fp x0 = fp_limbs_from_be48(b + 48, &lt0);
  if (i_flag) {
    uint32_t o = 0;
    for (int i = 0; i < NL; ++i) o |= x0.l[i] | x1.l[i];
    return (s_flag == 0 && o == 0) ? DEC_IDENTITY : DEC_ERR_FLAGS;
  }
  if (!lt0 || !lt1) return DEC_ERR_FIELD;
  const Fp2 x = {fp_to_mont(x0), fp_to_mont(x1)};
  out.x = x;
  const Fp2 rhs = fp2_reduce(fp2_add(fp2_mul(fp2_sqr(x), x), fp2_from_const(B2_M)));
  Fp2 y;
  if (!(INL ? fp2_sqrt_in<TBG_DECODE_WIN>(rhs, y, keep) : fp2_sqrt(rhs, y))) return DEC_ERR_NOT_ON_CURVE;
  if ((uint32_t)fp2_lex_largest(y) != s_flag) y = fp2_reduce(fp2_neg(y));
  out.y = y;
  if (SUBGROUP && !(INL ? g2_in_subgroup_aff_in(out) : g2_in_subgroup(jac_from_aff(out)))) return DEC_ERR_SUBGROUP;
  return DEC_OK;
}
TBG_NI int32_t g2_decompress(const uint8_t* b, G2A& out) { return g2_decompress_t<false>(b, out); }

// 48-byte ZCash compressed G1 -> affine (Montgomery).
TBG_NI int32_t g1_decompress(const uint8_t* b, G1A& out) {
  uint32_t c_flag = (b[0] >> 7) & 1, i_flag = (b[0] >> 6) & 1, s_flag = (b[0] >> 5) & 1;
  if (!c_flag) return DEC_ERR_FLAGS;
  uint8_t xb[48];
  for (int j = 0; j < 48; ++j) xb[j] = b[j];
  xb[0] &= 0x1f;
  bool lt;
  Fp x0 = fp_limbs_from_be48(xb, &lt);
  if (i_flag) {
    uint32_t o = 0;
    for (int i = 0; i < NL; ++i) o |= x0.l[i];
    return (s_flag == 0 && o == 0) ? DEC_IDENTITY : DEC_ERR_FLAGS;
  }
  if (!lt) return DEC_ERR_FIELD;
  Fp x = fp_to_mont(x0);
  Fp rhs = fp_reduce(fp_add(fp_mul(fp_sqr(x), x), fp_from_const(FOUR_M)));
  Fp y = fp_pow_const<EXP_SQRT_BITS, EXP_SQRT_WORDS>(rhs);
  if (!fp_eq(fp_sqr(y), rhs)) return DEC_ERR_NOT_ON_CURVE;
  Fp yc = fp_from_mont(y);
  if ((uint32_t)fp_lex_largest_canon(yc) != s_flag) y = fp_reduce(fp_neg(y));
  out.x = x;
  out.y = y;
  if (!g1_in_subgroup(jac_from_aff(out))) return DEC_ERR_SUBGROUP;
  return DEC_OK;
}

// affine G2 (Montgomery) -> 96-byte compressed; identity when inf.
TBG_HD void g2_compress(const G2A& a, bool inf, uint8_t* out) {
  if (inf) {
    out[0] = 0xc0;
    for (int j = 1; j < 96; ++j) out[j] = 0;
    return;
  }
  Fp x0 = fp_from_mont(a.x.c0), x1 = fp_from_mont(a.x.c1);
  fp_limbs_to_be48(x1, out);
  fp_limbs_to_be48(x0, out + 48);
  out[0] |= 0x80;
  if (fp2_lex_largest(a.y)) out[0] |= 0x20;
}

TBG_HD void g1_compress(const G1A& a, bool inf, uint8_t* out) {
  if (inf) {
    out[0] = 0xc0;
    for (int j = 1; j < 48; ++j) out[j] = 0;
    return;
  }
  fp_limbs_to_be48(fp_from_mont(a.x), out);
  out[0] |= 0x80;
  if (fp_lex_largest_canon(fp_from_mont(a.y))) out[0] |= 0x20;
}

}  // namespace tbg
