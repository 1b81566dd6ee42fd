// Optimal-ate pairing on BLS12-381: multi-pair Miller loop over |x| with
// Jacobian G2 accumulators and sparse (0, 1, 4) line multiplication, then the
// final exponentiation f^(3 (p^12 - 1) / r) (easy part + the hard-part
// identity 3 Phi_12(p) / r = (x-1)^2 (x+p) (x^2+p^2-1) + 3).  The extra cube
// does not change "== 1" because gcd(3, r) = 1.
//
// Used by BLS CoreVerify: e(pk, H(m)) * e(-g1, sig) == 1 (kryptology
// SigEth2.Verify, reached from reference tbls/tss.go:190-197).
#pragma once
#include "bls_curve.h"

namespace tbg {

struct Line { Fp2 l0, l1, l4; };

// T <- 2T; line through T tangent, evaluated at P (scaled by 2 Y Z^3 w^3).
TBG_HD Line miller_dbl_in(G2J& T, const Fp& nxP, const Fp& yP) {
  Fp2 A = fp2_sqr(T.X);
  Fp2 B = fp2_sqr(T.Y);
  Fp2 C = fp2_sqr(B);
  Fp2 ZZ = fp2_sqr(T.Z);
  Fp2 t = fp2_sub(fp2_sqr(fp2_add(T.X, B)), fp2_add(A, C));
  Fp2 D = fp2_reduce(fp2_add(t, t));
  Fp2 E = fp2_mul_small(A, 3);
  Fp2 F = fp2_sqr(E);
  Fp2 X3 = fp2_reduce(fp2_sub(F, fp2_add(D, D)));
  Fp2 Y3 = fp2_reduce(fp2_sub(fp2_mul(fp2_sub(D, X3), E), fp2_mul_small(C, 8)));
  Fp2 YZ = fp2_mul(T.Y, T.Z);
  Fp2 Z3 = fp2_reduce(fp2_add(YZ, YZ));
  Line l;
  l.l0 = fp2_reduce(fp2_sub(fp2_mul(T.X, E), fp2_add(B, B)));   // 3X^3 - 2Y^2
  l.l1 = fp2_mul_fp(fp2_mul(ZZ, E), nxP);                        // -3X^2 Z^2 xP
  l.l4 = fp2_mul_fp(fp2_mul(Z3, ZZ), yP);                        // 2 Y Z^3 yP
  T = {X3, Y3, Z3};
  return l;
}

// T <- T + Q (Q affine); line through T and Q evaluated at P (scaled by Z3 w^3).
TBG_HD Line miller_add_in(G2J& T, const G2A& Q, const Fp& nxP, const Fp& yP) {
  Fp2 ZZ = fp2_sqr(T.Z);
  Fp2 U2 = fp2_mul(Q.x, ZZ);
  Fp2 S2 = fp2_mul(fp2_mul(Q.y, T.Z), ZZ);
  Fp2 H = fp2_reduce(fp2_sub(U2, T.X));
  Fp2 R = fp2_reduce(fp2_sub(S2, T.Y));
  Fp2 HH = fp2_sqr(H);
  Fp2 HHH = fp2_mul(H, HH);
  Fp2 V = fp2_mul(T.X, HH);
  Fp2 X3 = fp2_reduce(fp2_sub(fp2_sub(fp2_sqr(R), HHH), fp2_add(V, V)));
  Fp2 Y3 = fp2_reduce(fp2_sub(fp2_mul(fp2_sub(V, X3), R), fp2_mul(T.Y, HHH)));
  Fp2 Z3 = fp2_mul(T.Z, H);
  Line l;
  l.l0 = fp2_reduce(fp2_sub(fp2_mul(R, Q.x), fp2_mul(Q.y, Z3)));
  l.l1 = fp2_mul_fp(R, nxP);
  l.l4 = fp2_mul_fp(Z3, yP);
  T = {X3, Y3, Z3};
  return l;
}

TBG_NI Line miller_dbl(G2J& T, const Fp& nxP, const Fp& yP) { return miller_dbl_in(T, nxP, yP); }
TBG_NI Line miller_add(G2J& T, const G2A& Q, const Fp& nxP, const Fp& yP) { return miller_add_in(T, Q, nxP, yP); }

// prod_n f_{|x|, Q_n}(P_n), conjugated for x < 0.  P, Q must not be infinity.
template <int N>
TBG_NI Fp12 miller_loop(const G1A (&P)[N], const G2A (&Q)[N]) {
  G2J T[N];
  Fp nxP[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    T[n] = jac_from_aff(Q[n]);
    nxP[n] = fp_reduce(fp_neg(P[n].x));
  }
  Fp12 f = fp12_one();
  for (int i = 62; i >= 0; --i) {
    if (i != 62) f = fp12_sqr(f);
#pragma unroll
    for (int n = 0; n < N; ++n) {
      Line l = miller_dbl(T[n], nxP[n], P[n].y);
      f = fp12_mul_by_014(f, l.l0, l.l1, l.l4);
    }
    if ((X_ABS >> i) & 1) {
#pragma unroll
      for (int n = 0; n < N; ++n) {
        Line l = miller_add(T[n], Q[n], nxP[n], P[n].y);
        f = fp12_mul_by_014(f, l.l0, l.l1, l.l4);
      }
    }
  }
  return fp12_conj(f);
}

// a^|x| for a in the cyclotomic subgroup (square and multiply over the fixed
// |x|, Granger-Scott squarings)
TBG_NI Fp12 fp12_pow_xabs(const Fp12& a) {
  Fp12 r = a;
  for (int i = 62; i >= 0; --i) {
    r = fp12_cyc_sqr(r);
    if ((X_ABS >> i) & 1) r = fp12_mul(r, a);
  }
  return r;
}

// a^x for a in the cyclotomic subgroup (x < 0: inverse = conjugate)
TBG_HD Fp12 cyc_pow_x(const Fp12& a) { return fp12_conj(fp12_pow_xabs(a)); }

TBG_NI Fp12 final_exp(const Fp12& f) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  Fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));
  t = fp12_mul(fp12_frob(fp12_frob(t)), t);
  // hard part (times 3)
  Fp12 a = fp12_mul(cyc_pow_x(t), fp12_conj(t));      // t^(x-1)
  a = fp12_mul(cyc_pow_x(a), fp12_conj(a));           // t^((x-1)^2)
  Fp12 b = fp12_mul(cyc_pow_x(a), fp12_frob(a));      // a^(x+p)
  Fp12 c = fp12_mul(cyc_pow_x(cyc_pow_x(b)), fp12_frob(fp12_frob(b)));
  c = fp12_mul(c, fp12_conj(b));                      // b^(x^2+p^2-1)
  Fp12 t3 = fp12_mul(fp12_cyc_sqr(t), t);
  return fp12_mul(c, t3);
}

// BLS CoreVerify with prepared affine inputs: e(pk, h) * e(-g1, sig) == 1.
TBG_NI bool bls_verify_prepared(const G1A& pk, const G2A& h, const G2A& sig) {
  G1A P[2];
  G2A Q[2];
  P[0] = pk;
  Q[0] = h;
  P[1].x = fp_from_const(G1_X);
  P[1].y = fp_from_const(G1_NEG_Y);
  Q[1] = sig;
  Fp12 f = miller_loop<2>(P, Q);
  return fp12_is_one(final_exp(f));
}

}  // namespace tbg
