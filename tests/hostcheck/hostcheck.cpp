// Host build of the engine's device math (the same headers the HIP kernels
// use), exported as plain C for the CPU test suite.  TEST TOOLING ONLY: this
// library is never loaded by the product (charon_amd loads libtbls_gpu.so
// and fails loudly without a GPU); it lets the kernel arithmetic be checked
// against the oracle on a machine with no GPU, with value-bound assertions
// (TBG_BOUNDS_CHECK) switched on.
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <cstdlib>
#include "../../charon_amd/csrc/bls_pairing.h"
#include "../../charon_amd/csrc/bls_h2c.h"

using namespace tbg;

#if defined(TBG_COUNT_OPS)
extern "C" unsigned long long tbg_mad_count = 0;
extern "C" unsigned long long hc_count_get(void) { return tbg_mad_count; }
extern "C" void hc_count_reset(void) { tbg_mad_count = 0; }
#endif

static Fp from_be(const uint8_t* b) {
  bool lt;
  return fp_to_mont(fp_limbs_from_be48(b, &lt));
}
static void to_be(const Fp& a, uint8_t* b) { fp_limbs_to_be48(fp_from_mont(a), b); }

extern "C" {

// out = a * b mod p (48-byte big-endian canonical in/out)
void hc_fp_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { to_be(fp_mul(from_be(a), from_be(b)), out); }
void hc_fp_sqr(const uint8_t* a, uint8_t* out) { to_be(fp_sqr(from_be(a)), out); }
void hc_fp_add(const uint8_t* a, const uint8_t* b, uint8_t* out) { to_be(fp_add(from_be(a), from_be(b)), out); }
void hc_fp_sub(const uint8_t* a, const uint8_t* b, uint8_t* out) { to_be(fp_sub(from_be(a), from_be(b)), out); }
void hc_fp_inv(const uint8_t* a, uint8_t* out) { to_be(fp_inv(from_be(a)), out); }
void hc_fp_inv_fermat(const uint8_t* a, uint8_t* out) { to_be(fp_inv_fermat(from_be(a)), out); }

// Fp2 multiply: inputs (c0, c1) each 48 bytes
void hc_fp2_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  Fp2 x = {from_be(a), from_be(a + 48)}, y = {from_be(b), from_be(b + 48)};
  Fp2 r = fp2_mul(x, y);
  to_be(r.c0, out);
  to_be(r.c1, out + 48);
}
int hc_fp2_sqrt(const uint8_t* a, uint8_t* out) {
  Fp2 x = {from_be(a), from_be(a + 48)}, r;
  if (!fp2_sqrt(x, r)) return 0;
  to_be(r.c0, out);
  to_be(r.c1, out + 48);
  return 1;
}

// Fp12 multiply/square/inverse/frobenius on 12 Fp2 coefficient in order
// c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2 (each c0 || c1, 96 bytes).
static Fp12 f12_in(const uint8_t* b) {
  Fp2 c[6];
  for (int i = 0; i < 6; ++i) c[i] = {from_be(b + 96 * i), from_be(b + 96 * i + 48)};
  return {{c[0], c[1], c[2]}, {c[3], c[4], c[5]}};
}
static void f12_out(const Fp12& f, uint8_t* b) {
  const Fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
  for (int i = 0; i < 6; ++i) {
    to_be(c[i]->c0, b + 96 * i);
    to_be(c[i]->c1, b + 96 * i + 48);
  }
}
void hc_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) { f12_out(fp12_mul(f12_in(a), f12_in(b)), out); }
void hc_fp12_sqr(const uint8_t* a, uint8_t* out) { f12_out(fp12_sqr(f12_in(a)), out); }
void hc_fp12_inv(const uint8_t* a, uint8_t* out) { f12_out(fp12_inv(f12_in(a)), out); }
void hc_fp12_frob(const uint8_t* a, uint8_t* out) { f12_out(fp12_frob(f12_in(a)), out); }
void hc_fp12_cyc_sqr(const uint8_t* a, uint8_t* out) { f12_out(fp12_cyc_sqr(f12_in(a)), out); }
void hc_final_exp(const uint8_t* a, uint8_t* out) { f12_out(final_exp(f12_in(a)), out); }

// G2 decompress -> status; on success writes the recompressed encoding and
// affine coordinates (x0, x1, y0, y1; 48 bytes each).
int hc_g2_decompress(const uint8_t* in, uint8_t* aff_out) {
  G2A a, b;
  int st = g2_decompress(in, a);
  // the kernel's form (inline subgroup check on the affine point) must agree
  if (g2_decompress_t<true>(in, b) != st) return 99;
  if (st == DEC_OK) {
    to_be(a.x.c0, aff_out);
    to_be(a.x.c1, aff_out + 48);
    to_be(a.y.c0, aff_out + 96);
    to_be(a.y.c1, aff_out + 144);
  }
  return st;
}
int hc_g1_decompress(const uint8_t* in, uint8_t* aff_out) {
  G1A a;
  int st = g1_decompress(in, a);
  if (st == DEC_OK) {
    to_be(a.x, aff_out);
    to_be(a.y, aff_out + 48);
  }
  return st;
}

// H(m) -> 96-byte compressed
void hc_hash_to_g2(const uint8_t* msg, uint32_t len, uint8_t* out) {
  G2J h = hash_to_g2(msg, len);
  G2A a;
  bool ok = jac_to_aff(h, a);
  g2_compress(a, !ok, out);
}

// Miller loop of one pair (affine inputs as raw coordinates) -> Fp12 bytes
void hc_miller(const uint8_t* p_aff, const uint8_t* q_aff, uint8_t* out) {
  G1A P[1];
  G2A Q[1];
  P[0] = {from_be(p_aff), from_be(p_aff + 48)};
  Q[0] = {{from_be(q_aff), from_be(q_aff + 48)}, {from_be(q_aff + 96), from_be(q_aff + 144)}};
  f12_out(miller_loop<1>(P, Q), out);
}

// Full CoreVerify from compressed encodings: 1 true, 0 false, <0 decode error
int hc_verify(const uint8_t* pk48, const uint8_t* msg, uint32_t len, const uint8_t* sig96) {
  G1A pk;
  G2A sig;
  int s1 = g1_decompress(pk48, pk);
  if (s1 < 0) return s1;
  int s2 = g2_decompress(sig96, sig);
  if (s2 < 0) return s2;
  if (s1 == DEC_IDENTITY || s2 == DEC_IDENTITY) return 0;
  G2J h = hash_to_g2(msg, len);
  G2A ha;
  if (!jac_to_aff(h, ha)) return 0;
  return bls_verify_prepared(pk, ha, sig) ? 1 : 0;
}

// Work-model probes: each runs one item of a pipeline stage.
int hc_stage_decode_sig(const uint8_t* sig96) {
  G2A a;
  return g2_decompress_t<true>(sig96, a);  // k_decode_sigs' form
}
int hc_stage_verify(const uint8_t* pk48, const uint8_t* sig96, const uint8_t* msg, uint32_t len) {
  G1A pk;
  G2A sig, ha;
  g1_decompress(pk48, pk);
  g2_decompress(sig96, sig);
  G2J h = hash_to_g2(msg, len);
  jac_to_aff(h, ha);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  return bls_verify_prepared(pk, ha, sig) ? 1 : 0;
}
void hc_stage_hash(const uint8_t* msg, uint32_t len) {
  G2J h = hash_to_g2(msg, len);
  G2A a;
  jac_to_aff(h, a);
}

}  // extern "C"

#include "../../charon_amd/csrc/bls_tss.h"
extern "C" {
// Aggregate k decoded partials exactly as k_aggregate does (Lagrange + Straus).
int hc_stage_aggregate(const uint8_t* ids, const uint8_t* sigs96, int k, uint8_t* out96) {
  G2A pts[16];
  uint32_t lam[16][8];
  if (k > 16) return -1;
  for (int i = 0; i < k; ++i)
    if (g2_decompress_t<true>(sigs96 + 96 * i, pts[i]) != DEC_OK) return -2;  // k_decode_sigs' form
  uint8_t mask[16];
  for (int i = 0; i < k; ++i) {
    if (!lagrange_encode(ids, k, i, lam[i])) return -3;
    mask[i] = 1;
  }
  G2J acc = tss_combine(pts, &lam[0][0], mask, k);
  G2A a;
  bool ok = jac_to_aff(acc, a);
  g2_compress(a, !ok, out96);
  return ok ? 0 : -4;
}
}

#include "../../charon_amd/csrc/bls_quad.h"
// Host emulation of the quad (lane-cooperative) Fp12 pieces: the three lanes
// run in turn and the DPP exchanges become array indexing.
extern "C" {
static void q_split(const Fp12& f, Fp4 (&A)[3]) { for (int q = 0; q < 3; ++q) A[q] = quad_from_fp12(q, f); }
static const int SW12[3] = {0, 2, 1};

void hc_quad_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  Fp4 A[3], B[3], P[3], Q[3], C[3];
  q_split(f12_in(a), A);
  q_split(f12_in(b), B);
  for (int q = 0; q < 3; ++q) {
    Fp4 SA = fp4_add(A[(q + 1) % 3], A[(q + 2) % 3]), SB = fp4_add(B[(q + 1) % 3], B[(q + 2) % 3]);
    P[q] = fp4_mul(A[q], B[q]);
    Q[q] = fp4_mul(SA, SB);
  }
  for (int q = 0; q < 3; ++q) C[q] = quad_combine(q, P[q], P[(q + 1) % 3], P[(q + 2) % 3], Q[SW12[q]]);
  f12_out(quad_to_fp12(C[0], C[1], C[2]), out);
}
void hc_quad_sqr(const uint8_t* a, uint8_t* out) {
  Fp4 A[3], P[3], Q[3], C[3];
  q_split(f12_in(a), A);
  for (int q = 0; q < 3; ++q) {
    P[q] = fp4_sqr(A[q]);
    Q[q] = fp4_sqr(fp4_add(A[(q + 1) % 3], A[(q + 2) % 3]));
  }
  for (int q = 0; q < 3; ++q) C[q] = quad_combine(q, P[q], P[(q + 1) % 3], P[(q + 2) % 3], Q[SW12[q]]);
  f12_out(quad_to_fp12(C[0], C[1], C[2]), out);
}
void hc_quad_cyc_sqr(const uint8_t* a, uint8_t* out) {
  Fp4 A[3], T[3], C[3];
  q_split(f12_in(a), A);
  for (int q = 0; q < 3; ++q) T[q] = fp4_sqr(A[q]);
  for (int q = 0; q < 3; ++q) C[q] = quad_cyc_lane(q, A[q], T[SW12[q]]);
  f12_out(quad_to_fp12(C[0], C[1], C[2]), out);
}
// f * line where line = (l0, l1, l4) each 96 bytes
void hc_quad_line(const uint8_t* a, const uint8_t* l, uint8_t* out) {
  Fp4 A[3], C[3];
  q_split(f12_in(a), A);
  Fp2 l0 = {from_be(l), from_be(l + 48)}, l1 = {from_be(l + 96), from_be(l + 144)}, l4 = {from_be(l + 192), from_be(l + 240)};
  for (int q = 0; q < 3; ++q) C[q] = quad_line_lane(q, A[q], A[(q + 1) % 3], l0, l1, l4);
  f12_out(quad_to_fp12(C[0], C[1], C[2]), out);
}
void hc_quad_frob(const uint8_t* a, uint8_t* out) {
  Fp4 A[3], C[3];
  q_split(f12_in(a), A);
  for (int q = 0; q < 3; ++q) C[q] = quad_frob_lane(q, A[q]);
  f12_out(quad_to_fp12(C[0], C[1], C[2]), out);
}
void hc_quad_conj(const uint8_t* a, uint8_t* out) {
  Fp4 A[3], C[3];
  q_split(f12_in(a), A);
  for (int q = 0; q < 3; ++q) C[q] = quad_conj_lane(q, A[q]);
  f12_out(quad_to_fp12(C[0], C[1], C[2]), out);
}
}

#include "../../charon_amd/csrc/bls_hex.h"
// Host emulation of the hexad (bls_hex.h): trio lane q and component c run
// in turn, the pair swap and the DPP exchanges become array indexing.
extern "C" {
static void hx_split(const Fp12& f, Fp4 (&A)[3]) { q_split(f, A); }
static Fp12 hx_join(const Fp4h (&R)[3][2]) {
  Fp4 C[3];
  for (int q = 0; q < 3; ++q) C[q] = {{R[q][0].a, R[q][1].a}, {R[q][0].b, R[q][1].b}};
  return quad_to_fp12(C[0], C[1], C[2]);
}
void hc_hex_sqr(const uint8_t* a, uint8_t* out) {
  Fp4 A[3];
  hx_split(f12_in(a), A);
  Fp ab[3][2], s[3][2], V[3][2];
  Fp4h P[3][2], Q[3][2], T[3][2], R[3][2];
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) hx_sqr1(c, hx_view4(c, A[q]), ab[q][c], s[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) P[q][c] = hx_sqr2(c, ab[q][c], ab[q][c ^ 1], s[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) hx_sqr1(c, hx_view4(c, fp4_add(A[(q + 1) % 3], A[(q + 2) % 3])), ab[q][c], s[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) Q[q][c] = hx_sqr2(c, ab[q][c], ab[q][c ^ 1], s[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c)
      hx_comb1(q, P[q][c], P[(q + 1) % 3][c], P[(q + 2) % 3][c], Q[SW12[q]][c], T[q][c], V[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c)
      R[q][c] = hx_comb2(c, q, P[q][c], P[(q + 1) % 3][c], P[(q + 2) % 3][c], T[q][c], V[q][c], V[q][c ^ 1]);
  f12_out(hx_join(R), out);
}
// f * line where line = (l0, l1, l4) each 96 bytes
void hc_hex_line(const uint8_t* a, const uint8_t* l, uint8_t* out) {
  Fp4 A[3];
  hx_split(f12_in(a), A);
  Fp2 l0 = {from_be(l), from_be(l + 48)}, l1 = {from_be(l + 96), from_be(l + 144)}, l4 = {from_be(l + 192), from_be(l + 240)};
  HxLine r[3][2];
  Fp4h R[3][2];
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) {
      hx_line_u(c, hx_view4(c, A[(q + 1) % 3]), hx_view(c, l1), r[q][c]);
      hx_line_t(c, q, hx_view4(c, A[q]), hx_view(c, l0), hx_view(c, l4), r[q][c]);
    }
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) R[q][c] = hx_line2(c, q, r[q][c], r[q][c ^ 1].W);
  f12_out(hx_join(R), out);
}
}

#include "../../charon_amd/csrc/bls_lines.h"
// Whole quad verify emulated on the host (same per-lane pieces as
// k_verify_quad): lines precomputed with g2_lines, Miller accumulation and
// final exponentiation on the 3-lane split representation.
namespace qe {
struct Q3 { Fp4 v[3]; };
static Q3 mul(const Q3& A, const Q3& B) {
  Q3 P, Q, C;
  for (int q = 0; q < 3; ++q) {
    P.v[q] = fp4_mul(A.v[q], B.v[q]);
    Q.v[q] = fp4_mul(fp4_add(A.v[(q + 1) % 3], A.v[(q + 2) % 3]), fp4_add(B.v[(q + 1) % 3], B.v[(q + 2) % 3]));
  }
  for (int q = 0; q < 3; ++q) C.v[q] = quad_combine(q, P.v[q], P.v[(q + 1) % 3], P.v[(q + 2) % 3], Q.v[SW12[q]]);
  return C;
}
static Q3 sqr(const Q3& A) {
  Q3 P, Q, C;
  for (int q = 0; q < 3; ++q) {
    P.v[q] = fp4_sqr(A.v[q]);
    Q.v[q] = fp4_sqr(fp4_add(A.v[(q + 1) % 3], A.v[(q + 2) % 3]));
  }
  for (int q = 0; q < 3; ++q) C.v[q] = quad_combine(q, P.v[q], P.v[(q + 1) % 3], P.v[(q + 2) % 3], Q.v[SW12[q]]);
  return C;
}
static Q3 cyc(const Q3& A) {
  Q3 T, C;
  for (int q = 0; q < 3; ++q) T.v[q] = fp4_sqr(A.v[q]);
  for (int q = 0; q < 3; ++q) C.v[q] = quad_cyc_lane(q, A.v[q], T.v[SW12[q]]);
  return C;
}
static Q3 line(const Q3& A, const Fp2& l0, const Fp2& l1, const Fp2& l4) {
  Q3 C;
  for (int q = 0; q < 3; ++q) C.v[q] = quad_line_lane(q, A.v[q], A.v[(q + 1) % 3], l0, l1, l4);
  return C;
}
static Q3 conj(const Q3& A) { Q3 C; for (int q = 0; q < 3; ++q) C.v[q] = quad_conj_lane(q, A.v[q]); return C; }
static Q3 frob(const Q3& A) { Q3 C; for (int q = 0; q < 3; ++q) C.v[q] = quad_frob_lane(q, A.v[q]); return C; }
static Q3 inv(const Q3& A) {
  Fp12 r = fp12_inv(quad_to_fp12(A.v[0], A.v[1], A.v[2]));
  Q3 C; for (int q = 0; q < 3; ++q) C.v[q] = quad_from_fp12(q, r); return C;
}
static Q3 pow_x(const Q3& a) {
  Q3 r = a;
  for (int i = 62; i >= 0; --i) { r = cyc(r); if ((X_ABS >> i) & 1) r = mul(r, a); }
  return conj(r);
}
static Q3 final_exp(const Q3& f) {
  Q3 t = mul(conj(f), inv(f));
  t = mul(frob(frob(t)), t);
  Q3 a = mul(pow_x(t), conj(t));
  a = mul(pow_x(a), conj(a));
  Q3 b = mul(pow_x(a), frob(a));
  Q3 c = mul(pow_x(pow_x(b)), frob(frob(b)));
  c = mul(c, conj(b));
  Q3 t3 = mul(cyc(t), t);
  return mul(c, t3);
}
}  // namespace qe

// The hexad's final-exponentiation pieces (hex_mul, hex_cyc_sqr, hex_frob,
// hex_conj, hex_inv, hex_final_exp_in) emulated lane by lane: H6.v[q][c] is
// what lane (q, c) holds, c ^ 1 the ds_swizzle partner.
namespace he {
struct H6 { Fp4h v[3][2]; };
static H6 split(const Fp12& f) {
  Fp4 A[3];
  q_split(f, A);
  H6 r;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) r.v[q][c] = {c ? A[q].a.c1 : A[q].a.c0, c ? A[q].b.c1 : A[q].b.c0};
  return r;
}
static Fp12 join(const H6& h) { return hx_join(h.v); }
static Fp4o own_par(const H6& h, int q, uint32_t c) {
  return {{h.v[q][c].a, h.v[q][c ^ 1].a}, {h.v[q][c].b, h.v[q][c ^ 1].b}};
}
static H6 sum_others(const H6& h) {
  H6 r;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c)
      r.v[q][c] = {fp_add(h.v[(q + 1) % 3][c].a, h.v[(q + 2) % 3][c].a),
                   fp_add(h.v[(q + 1) % 3][c].b, h.v[(q + 2) % 3][c].b)};
  return r;
}
static H6 fp4mul(const H6& A, const H6& B) {
  Fp t0[3][2], t1[3][2], s[3][2];
  H6 P;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) hx_mul1(c, own_par(A, q, c), own_par(B, q, c), t0[q][c], t1[q][c], s[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) P.v[q][c] = hx_mul2(c, t0[q][c], t1[q][c], t1[q][c ^ 1], s[q][c]);
  return P;
}
static H6 fp4sqr(const H6& A) {
  Fp ab[3][2], s[3][2];
  H6 P;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) hx_sqr1(c, own_par(A, q, c), ab[q][c], s[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) P.v[q][c] = hx_sqr2(c, ab[q][c], ab[q][c ^ 1], s[q][c]);
  return P;
}
static H6 combine(const H6& P, const H6& Q) {
  Fp4h T[3][2];
  Fp V[3][2];
  H6 R;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c)
      hx_comb1(q, P.v[q][c], P.v[(q + 1) % 3][c], P.v[(q + 2) % 3][c], Q.v[SW12[q]][c], T[q][c], V[q][c]);
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c)
      R.v[q][c] = hx_comb2(c, q, P.v[q][c], P.v[(q + 1) % 3][c], P.v[(q + 2) % 3][c], T[q][c], V[q][c], V[q][c ^ 1]);
  return R;
}
static H6 mul(const H6& A, const H6& B) { return combine(fp4mul(A, B), fp4mul(sum_others(A), sum_others(B))); }
static H6 cyc(const H6& A) {
  const H6 T = fp4sqr(A);
  H6 R;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) R.v[q][c] = hx_cyc(c, q, A.v[q][c], T.v[SW12[q]][c], T.v[SW12[q]][c ^ 1].b);
  return R;
}
static H6 conj(const H6& A) {
  H6 R;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) R.v[q][c] = hx_conj(q, A.v[q][c]);
  return R;
}
static H6 frob(const H6& A) {
  H6 R;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) R.v[q][c] = hx_frob(c, q, A.v[q][c], A.v[q][c ^ 1]);
  return R;
}
static H6 inv(const H6& A) { return split(fp12_inv(join(A))); }
static bool is_one(const H6& A) {
  bool ok = true;
  for (int q = 0; q < 3; ++q)
    for (uint32_t c = 0; c < 2; ++c) ok = ok && hx_is_one_lane(c, q, A.v[q][c]);
  return ok;
}
static H6 pow_x(const H6& a) {
  H6 r = a;
  for (int i = 62; i >= 0; --i) { r = cyc(r); if ((X_ABS >> i) & 1) r = mul(r, a); }
  return conj(r);
}
static H6 final_exp(const H6& f) {
  H6 t = mul(conj(f), inv(f));
  t = mul(frob(frob(t)), t);
  H6 a = mul(pow_x(t), conj(t));
  a = mul(pow_x(a), conj(a));
  H6 b = mul(pow_x(a), frob(a));
  H6 c = mul(pow_x(pow_x(b)), frob(frob(b)));
  c = mul(c, conj(b));
  H6 t3 = mul(cyc(t), t);
  return mul(c, t3);
}
}  // namespace he

extern "C" {
void hc_hex_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  f12_out(he::join(he::mul(he::split(f12_in(a)), he::split(f12_in(b)))), out);
}
void hc_hex_cyc_sqr(const uint8_t* a, uint8_t* out) { f12_out(he::join(he::cyc(he::split(f12_in(a)))), out); }
void hc_hex_frob(const uint8_t* a, uint8_t* out) { f12_out(he::join(he::frob(he::split(f12_in(a)))), out); }
void hc_hex_conj(const uint8_t* a, uint8_t* out) { f12_out(he::join(he::conj(he::split(f12_in(a)))), out); }
// the final exponentiation; returns whether the result is 1 by the lanes' test
int hc_hex_final_exp(const uint8_t* a, uint8_t* out) {
  const he::H6 r = he::final_exp(he::split(f12_in(a)));
  f12_out(he::join(r), out);
  return he::is_one(r) ? 1 : 0;
}
}

extern "C" {
static uint32_t g_sig_lines[LINES_WORDS], g_h_lines[LINES_WORDS];
// stage 1: line precomputation for one partial (signature lines) and its message (H lines)
int hc_stage_lines(const uint8_t* sig96, const uint8_t* msg, uint32_t len) {
  G2A sig, ha;
  if (g2_decompress(sig96, sig) != DEC_OK) return -1;
  G2J h = hash_to_g2(msg, len);
  jac_to_aff(h, ha);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));
  g2_lines(sig, nx, fp_from_const(G1_NEG_Y), g_sig_lines);
#if defined(TBG_COUNT_OPS)
  unsigned long long sig_cost = tbg_mad_count;
#endif
  g2_lines(ha, fp_one(), fp_one(), g_h_lines);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = sig_cost;  // report the per-signature share; H lines are per message
#endif
  return 0;
}
// stage 2: quad verify of that partial against pk, using the stored lines
int hc_stage_verify_quad(const uint8_t* pk48) {
  G1A pk;
  if (g1_decompress(pk48, pk) != DEC_OK) return -1;
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  Fp nx = fp_reduce(fp_neg(pk.x));
  qe::Q3 f;
  f.v[0] = {fp2_one(), fp2_zero()};
  f.v[1] = fp4_zero();
  f.v[2] = fp4_zero();
  int idx = 0;
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = qe::sqr(f);
    int steps = ((X_ABS >> b) & 1) ? 2 : 1;
    for (int s = 0; s < steps; ++s, ++idx) {
      Line a = line_load(g_sig_lines + LINE_WORDS * idx);
      f = qe::line(f, a.l0, a.l1, a.l4);
      Line h = line_load(g_h_lines + LINE_WORDS * idx);
      f = qe::line(f, h.l0, fp2_mul_fp(h.l1, nx), fp2_mul_fp(h.l4, pk.y));
    }
  }
  f = qe::final_exp(qe::conj(f));
  Fp12 r = quad_to_fp12(f.v[0], f.v[1], f.v[2]);
  return fp12_is_one(r) ? 1 : 0;
}
}

#include "../../charon_amd/csrc/bls_rlc.h"
// RLC scalar application (k_rlc_partial) against plain scalar multiplication,
// and per-stage operation counts of the RLC schedule (tools/count_work.py).
extern "C" {
static G1A hc_xpk(const G1A& pk) {
  G1A x;
  jac_to_aff(jac_neg(jac_mul_xabs(jac_from_aff(pk))), x);
  return x;
}
// r_words: the scalar sum a_k x^k mod r as 8 little-endian u32 words.
int hc_rlc_check(const uint8_t* sig96, const uint8_t* pk48, uint64_t r64, const uint32_t* r_words) {
  G2A s;
  G1A pk;
  if (g2_decompress(sig96, s) != DEC_OK || g1_decompress(pk48, pk) != DEC_OK) return -1;
  uint32_t a[4];
  rlc_digits(r64, a);
  G2J S = rlc_mul_g2(s, a);
  G1J P = rlc_mul_g1(pk, hc_xpk(pk), a);
  G2J S2;
  G1J P2;
  rlc_mul_both(s, pk, hc_xpk(pk), a, S2, P2);
  G2J S_ref = jac_mul_words(jac_from_aff(s), r_words, 255);
  G1J P_ref = jac_mul_words(jac_from_aff(pk), r_words, 255);
  return (jac_eq(S, S_ref) && jac_eq(S2, S_ref) ? 1 : 0) | (jac_eq(P, P_ref) && jac_eq(P2, P_ref) ? 2 : 0);
}
uint64_t hc_rlc_scalar(const uint8_t* seed32, uint32_t i) {
  uint32_t seed[8];
  for (int k = 0; k < 8; ++k)
    seed[k] = ((uint32_t)seed32[4 * k] << 24) | ((uint32_t)seed32[4 * k + 1] << 16) | ((uint32_t)seed32[4 * k + 2] << 8) | seed32[4 * k + 3];
  return rlc_scalar(seed, i);
}

static G2A g_sig;
static G1A g_pk, g_xpk;
static G2A g_h;
int hc_stage_setup(const uint8_t* sig96, const uint8_t* pk48, const uint8_t* msg, uint32_t len) {
  if (g2_decompress(sig96, g_sig) != DEC_OK || g1_decompress(pk48, g_pk) != DEC_OK) return -1;
  g_xpk = hc_xpk(g_pk);
  jac_to_aff(hash_to_g2(msg, len), g_h);
  return 0;
}
// one non-lead partial of k_rlc_partial (PRF + both digit products)
void hc_stage_rlc_partial(uint64_t r64) {
  uint32_t a[4];
  rlc_digits(r64, a);
  G2J S;
  G1J P;
  rlc_mul_both(g_sig, g_pk, g_xpk, a, S, P);
  (void)S;
  (void)P;
}
// k_rlc_duty_sum for n partials: n-1 Jacobian additions per group + G1 affine
void hc_stage_duty_sum(int n) {
  G1J P = jac_from_aff(g_pk), P1 = jac_dbl(P);
  G2J S = jac_from_aff(g_sig), S1 = jac_dbl(S);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  G1J accP = P;
  G2J accS = S;
  for (int k = 1; k < n; ++k) {
    accP = jac_add(accP, P1);
    accS = jac_add(accS, S1);
  }
  G1A a;
  jac_to_aff(accP, a);
}
// k_rlc_group_lines for G duties
void hc_stage_group_lines(int G) {
  G2J S = jac_from_aff(g_sig), S1 = jac_dbl(S);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  G2J acc = S;
  for (int k = 1; k < G; ++k) acc = jac_add(acc, S1);
  G2A a;
  jac_to_aff(acc, a);
  Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));
  g2_lines(a, nx, fp_from_const(G1_NEG_Y), g_sig_lines);
}
// one k_rlc_miller_chunks quad: `pairs` duty pairs (+ the folded S pair)
void hc_stage_miller_chunk(int pairs, int with_folded) {
  Fp nx0 = fp_reduce(fp_neg(fp_from_const(G1_X)));
  g2_lines(g_sig, nx0, fp_from_const(G1_NEG_Y), g_sig_lines);
  g2_lines(g_h, fp_one(), fp_one(), g_h_lines);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  qe::Q3 f;
  f.v[0] = {fp2_one(), fp2_zero()};
  f.v[1] = fp4_zero();
  f.v[2] = fp4_zero();
  int idx = 0;
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = qe::sqr(f);
    int steps = ((X_ABS >> b) & 1) ? 2 : 1;
    for (int s = 0; s < steps; ++s, ++idx) {
      if (with_folded) {
        Line a = line_load(g_sig_lines + LINE_WORDS * idx);
        f = qe::line(f, a.l0, a.l1, a.l4);
      }
      for (int k = 0; k < pairs; ++k) {
        Line h = line_load(g_h_lines + LINE_WORDS * idx);
        Fp nx = fp_reduce(fp_neg(g_pk.x));
        // lanes 0 / 1 evaluate l1 (-x) / l4 y; lane 2 repeats lane 1's product
        Fp2 e1 = fp2_mul_fp(h.l1, nx), e4 = fp2_mul_fp(h.l4, g_pk.y);
        (void)fp2_mul_fp(h.l4, g_pk.y);
        f = qe::line(f, h.l0, e1, e4);
      }
    }
  }
}
// one k_rlc_group_final quad: nch - 1 products and the final exponentiation
void hc_stage_group_final(int nch) {
  qe::Q3 f;
  f.v[0] = {fp2_one(), fp2_one()};
  f.v[1] = {fp2_one(), fp2_zero()};
  f.v[2] = fp4_zero();
  for (int c = 1; c < nch; ++c) f = qe::mul(f, f);
  f = qe::final_exp(qe::conj(f));
}
}

#include "../../charon_amd/csrc/bls_pair.h"
// Lane-pair Fp2 (bls_pair.h), host-emulated: the two lanes' pieces side by side.
extern "C" {
// out: mul(a, b), sqr(a), inv(a), conj(a), mul_xi(a), a * PSI_X -- 6 x 96 bytes (c0 || c1 canonical BE)
static void f2_out_pp(const Fp2p& x, uint8_t* out) {
  fp_limbs_to_be48(fp_from_mont(x.c0), out);
  fp_limbs_to_be48(fp_from_mont(x.c1), out + 48);
}
static Fp2p f2_in_pp(const uint8_t* in) {
  bool lt;
  return {fp_to_mont(fp_limbs_from_be48(in, &lt)), fp_to_mont(fp_limbs_from_be48(in + 48, &lt))};
}
void hc_pair_ops(const uint8_t* a96, const uint8_t* b96, uint8_t* out) {
  Fp2p a = f2_in_pp(a96), b = f2_in_pp(b96);
  f2_out_pp(f_mul(a, b), out);
  f2_out_pp(f_sqr(a), out + 96);
  f2_out_pp(f_inv(a), out + 192);
  f2_out_pp(f_reduce(pp_conj(a)), out + 288);
  f2_out_pp(f_reduce(pp_mul_xi(a)), out + 384);
  f2_out_pp(pp_mul_const(a, PSI_X), out + 480);
}
// k_lines_h (pair-emulated miller_dbl_g / miller_add_g) against the
// single-lane g2_lines of the same point, and the pair-emulated cofactor
// clearing (g2_clear_cofactor_g, k_hash_clear_*) against g2_clear_cofactor:
// bit 1 lines equal, bit 2 clearing equal (or the doubling exception taken),
// bit 4 the unevaluated lines equal.
int hc_pair_lines_clear(const uint8_t* sig96) {
  G2A q;
  if (g2_decompress_t<true, false>(sig96, q) != DEC_OK) return -1;  // (no subgroup check: E2 points too)
  static uint32_t ref[LINES_WORDS];
  const Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X))), y = fp_from_const(G1_NEG_Y);
  g2_lines(q, nx, y, ref);
  Aff<Fp2p> Q{pp_from(q.x), pp_from(q.y)};
  Jac<Fp2p> T = jac_from_aff(Q);
  int idx = 0, out = 1;
  auto same = [&](const LineG<Fp2p>& l) {
    const Line r = line_load(ref + LINE_WORDS * idx++);
    if (!fp2_eq(pp_to(l.l0), r.l0) || !fp2_eq(pp_to(l.l1), r.l1) || !fp2_eq(pp_to(l.l4), r.l4)) out = 0;
  };
  for (int i = 62; i >= 0; --i) {
    same(miller_dbl_g(T, nx, y));
    if ((X_ABS >> i) & 1) same(miller_add_g(T, Q, nx, y));
  }
  // the unevaluated form (k_lines_h, EVAL = false) against P = (1, 1): bit 4
  g2_lines(q, fp_one(), fp_one(), ref);
  T = jac_from_aff(Q);
  idx = 0;
  const int before = out;
  out = 1;
  for (int i = 62; i >= 0; --i) {
    same(miller_dbl_g<Fp2p, false>(T, nx, y));
    if ((X_ABS >> i) & 1) same(miller_add_g<Fp2p, false>(T, Q, nx, y));
  }
  out = before | (out ? 4 : 0);
  bool exc = false;
  const Jac<Fp2p> c = g2_clear_cofactor_g(Jac<Fp2p>{Q.x, Q.y, f_one<Fp2p>()}, exc);
  const G2J cg{pp_to(c.X), pp_to(c.Y), pp_to(c.Z)};
  if (exc || jac_eq(cg, g2_clear_cofactor(jac_from_aff(q)))) out |= 2;
  return out;
}
// k_decode_sigs + k_subgroup_sigs: decode without the subgroup check, then the
// pair-emulated check; returns a DecodeStatus like g2_decompress.
int hc_pair_decode_sig(const uint8_t* sig96) {
  G2A a;
  int st = g2_decompress_t<true, false>(sig96, a);
  if (st != DEC_OK) return st;
  Aff<Fp2p> p{pp_from(a.x), pp_from(a.y)};
  bool exc = false;
  bool ok = g2_in_subgroup_aff_g(p, exc);
  if (exc) ok = g2_in_subgroup(jac_from_aff(a));
  return ok ? DEC_OK : DEC_ERR_SUBGROUP;
}
}

// [r] pk from the per-key window table (bls_rlc.h rlc_mul_key_w2, the table
// built entry by entry as k_pubkey_tables does) against the plain
// double-and-add [r mod order] pk: 1 on a match.
extern "C" int hc_rlc_check_w2(const uint8_t* pk48, uint64_t r64, const uint32_t* r_words) {
  G1A pk;
  if (g1_decompress(pk48, pk) != DEC_OK) return -1;
  uint32_t a[4];
  rlc_digits(r64, a);
  const G1A xpk = hc_xpk(pk);
  G1A tab[PK_TAB_W2];
  for (int k = 0; k < (int)PK_TAB_W2; ++k)
    if (!jac_to_aff(rlc_key_table_w2_entry(pk, xpk, k), tab[k])) return -2;
  return jac_eq(rlc_mul_key_w2(tab, fp_from_const(G1_BETA), a), jac_mul_words(jac_from_aff(pk), r_words, 255)) ? 1 : 0;
}

// Inversion-free RLC products (bls_rlc.h *_j, the split kernels k_rlc_g1 /
// k_rlc_g2_pair): G1, single-lane G2 and the pair-emulated G2, each against
// the plain 255-bit double-and-add [r mod order] P.  Bits 1 | 2 | 4.
extern "C" int hc_rlc_check_j(const uint8_t* sig96, const uint8_t* pk48, uint64_t r64, const uint32_t* r_words) {
  G2A s;
  G1A pk;
  if (g2_decompress(sig96, s) != DEC_OK || g1_decompress(pk48, pk) != DEC_OK) return -1;
  uint32_t a[4];
  rlc_digits(r64, a);
  G2J S_ref = jac_mul_words(jac_from_aff(s), r_words, 255);
  G1J P_ref = jac_mul_words(jac_from_aff(pk), r_words, 255);
  int out = 0;
  if (jac_eq(rlc_mul_g1_j(pk, hc_xpk(pk), a), P_ref)) out |= 1;
  {
    G2A ps = g2_psi_aff(s);
    G2J ap, am;
    rlc_pair_jac(s, ps, ap, am);
    if (jac_eq(rlc_mul_table_j(ap, am, fp_from_const(PSI2_X), a), S_ref)) out |= 2;
  }
  {
    Aff<Fp2p> sp{pp_from(s.x), pp_from(s.y)};
    Aff<Fp2p> psp{f_mulc(f_conj(sp.x), PSI_X), f_mulc(f_conj(sp.y), PSI_Y)};
    Jac<Fp2p> ap, am;
    rlc_pair_jac(sp, psp, ap, am);
    Jac<Fp2p> S = rlc_mul_table_j(ap, am, fp_from_const(PSI2_X), a);
    G2J Sg{pp_to(S.X), pp_to(S.Y), pp_to(S.Z)};
    if (jac_eq(Sg, S_ref)) out |= 4;
  }
  return out;
}

// [k] P through the base-|x| digits (bls_tss.h g2_mul_base_x, the
// k_aggregate_finish MSM) against the plain 255-bit double-and-add.  Writes
// the four digits to d4; returns 1 on agreement.
extern "C" int hc_base_x_check(const uint8_t* sig96, const uint32_t* k_words, uint64_t* d4) {
  G2A s;
  if (g2_decompress(sig96, s) != DEC_OK) return -1;
  uint32_t w[8];
  for (int j = 0; j < 8; ++j) w[j] = k_words[j];
  uint64_t d[4];
  base_x_digits(w, d);
  for (int i = 0; i < 4; ++i) d4[i] = d[i];
  const G2J p = jac_from_aff(s);
  return jac_eq(g2_mul_base_x(p, d), jac_mul_words(p, w, 256)) ? 1 : 0;
}

#include "../../charon_amd/csrc/bls_msm.h"
// Level-0 bucket MSM (k_msm.hip) against the per-partial RLC products:
// sum_i [r_i] s_i by buckets == sum_i rlc_mul_g2(s_i, digits(r_i)).
extern "C" {
int hc_msm_check(const uint8_t* sigs96, const uint64_t* r, uint32_t n) {
  static G2J buckets[32768];
  G2A s[64];
  if (n > 64) return -2;
  G2J ref = jac_inf<Fp2>();
  for (uint32_t i = 0; i < n; ++i) {
    if (g2_decompress(sigs96 + 96ull * i, s[i]) != DEC_OK) return -1;
    uint32_t a[4];
    rlc_digits(r[i], a);
    ref = jac_add(ref, rlc_mul_g2(s[i], a));
  }
  G2J got = msm_reference(s, r, n, buckets);
  return jac_eq(got, ref) ? 1 : 0;
}

// Level 1's group MSM (k_gmsm.hip, 4-bit windows of the psi digits) against
// the per-partial RLC products; partial `lead` takes r = 1.
int hc_gm_check(const uint8_t* sigs96, const uint64_t* r, uint32_t n, uint32_t lead) {
  G2A s[64];
  if (n > 64) return -2;
  G2J ref = jac_inf<Fp2>();
  for (uint32_t i = 0; i < n; ++i) {
    if (g2_decompress(sigs96 + 96ull * i, s[i]) != DEC_OK) return -1;
    if (i == lead) {
      ref = jac_add(ref, jac_from_aff(s[i]));
      continue;
    }
    uint32_t a[4];
    rlc_digits(r[i], a);
    ref = jac_add(ref, rlc_mul_g2(s[i], a));
  }
  return jac_eq(gm_reference(s, r, n, lead), ref) ? 1 : 0;
}
}  // extern "C"

// Level-0 stages (tools/count_work.py): one partial's G1 product from the
// key's pair table plus its 4 bucket additions; the G1-only duty sum; one
// bucket's [2j + 1]; one tree addition.
extern "C" {
// the key's window table (k_pubkey_tables), built at key load
static void hc_key_table_w2(G1A (&tab)[PK_TAB_W2]) {
  for (int k = 0; k < (int)PK_TAB_W2; ++k) jac_to_aff(rlc_key_table_w2_entry(g_pk, g_xpk, k), tab[k]);
}
void hc_stage_l0_partial(uint64_t r64) {
  G1A tab[PK_TAB_W2];
  hc_key_table_w2(tab);  // at key load
  G2J acc = jac_dbl(jac_from_aff(g_sig));
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  uint32_t u[4];
  rlc_digits(r64, u);
  G1J P = rlc_mul_key_w2(tab, fp_from_const(G1_BETA), u);
  (void)P;
  for (uint32_t k = 0; k < 4; ++k) {
    bool neg;
    (void)msm_bucket(u[k], neg);
    G2A p = msm_psi_k(g_sig, k);
    if (neg) p.y = fp2_reduce(fp2_neg(p.y));
    acc = jac_add_aff_in(acc, p);
  }
}
void hc_stage_duty_sum_p(int n) {
  G1J P = jac_from_aff(g_pk), P1 = jac_dbl(P);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  G1J accP = P;
  for (int k = 1; k < n; ++k) accP = jac_add(accP, P1);
  G1A a;
  jac_to_aff(accP, a);
}
void hc_stage_l0_bucket_scale(uint32_t m) {
  G2J b = jac_dbl(jac_from_aff(g_sig));
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  G2J acc = b;
  const int top = 31 - __builtin_clz(m);
  for (int bit = top - 1; bit >= 0; --bit) {
    acc = jac_dbl_in(acc);
    if ((m >> bit) & 1u) acc = jac_add_in<Fp2, true>(acc, b);
  }
}
void hc_stage_g2_add(void) {
  G2J a = jac_dbl(jac_from_aff(g_sig)), b = jac_dbl(a);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  a = jac_add_in<Fp2, true>(a, b);
}
}  // extern "C"

// expand_message_xmd / hash_to_field: the word-oriented register form the
// kernels use against the byte-stream reference form.
extern "C" int hc_h2f_check(const uint8_t* msg, uint32_t len) {
  Fp2 a0, a1, b0, b1;
  hash_to_field_fp2(msg, len, a0, a1);
  hash_to_field_fp2_bytes(msg, len, b0, b1);
  return fp2_eq(a0, b0) && fp2_eq(a1, b1) ? 1 : 0;
}

// Per-kernel work probes (tools/count_work.py -> profiles/work_model.json
// "kernels"): each runs the single-lane equivalent of ONE item of one kernel
// of the level-0 chain, so bench.py can price the dominant kernel alone.
extern "C" {
// k_decode_sigs: flags, field, Fp2 square root (no subgroup check)
int hc_k_decode_sigs(const uint8_t* sig96) {
  G2A a;
  return g2_decompress_t<true, false>(sig96, a);
}
// k_subgroup_sigs: psi(a) == [x] a on the decoded point
int hc_k_subgroup_sigs(const uint8_t* sig96) {
  G2A a;
  if (g2_decompress_t<true, false>(sig96, a) != DEC_OK) return -1;
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  return g2_in_subgroup_aff_in(a) ? 1 : 0;
}
// k_hash_map: hash_to_field, the SSWU denominators, their inverse (fp2_inv;
// count_work.py prices the batched form) and each map's x1
static Fp2 g_hu0, g_hu1, g_hx10, g_hx11;
void hc_k_hash_map(const uint8_t* msg, uint32_t len) {
  hash_to_field_fp2(msg, len, g_hu0, g_hu1);
  SswuPair w;
  const Fp2 di = fp2_inv(sswu_pair_den(g_hu0, g_hu1, w));
  g_hx10 = sswu_x1(fp2_mul(w.den[1], di));
  g_hx11 = sswu_x1(fp2_mul(w.den[0], di));
}
// k_hash_sswu: both maps of the message (two lanes) as the kernel runs them:
// root at window width SSWU_WIN, x and y, the isogeny
void hc_k_hash_sswu(void) {
  const Fp2* u[2] = {&g_hu0, &g_hu1};
  const Fp2* x1[2] = {&g_hx10, &g_hx11};
  for (int j = 0; j < 2; ++j) {
    Fp2 r, x, y;
    bool sq;
    if (!fp2_sqrt_or_z_in<SSWU_WIN>(sswu_gx(*x1[j]), r, sq)) continue;
    sswu_xy(*u[j], *x1[j], r, sq, x, y);
    (void)iso3_to_jac_in(x, y);
  }
}
// the split map agrees with the reference map (map_to_curve_g2, RFC 9380
// 6.6.2) on the message's two field elements: 1 when both affine points match
extern "C" int hc_sswu_split_check(const uint8_t* msg, uint32_t len) {
  hc_k_hash_map(msg, len);
  const Fp2* u[2] = {&g_hu0, &g_hu1};
  const Fp2* x1[2] = {&g_hx10, &g_hx11};
  for (int j = 0; j < 2; ++j) {
    G2J q;
    if (!sswu_map_x1(*u[j], *x1[j], q)) return -1;
    const G2J ref = map_to_curve_g2(*u[j]);
    if (!jac_eq(q, ref)) return 0;
  }
  return 1;
}
// k_hash_clear_x1 / _x2 / _fin on the message's two mapped points
static G2J g_hq, g_hq0, g_hq1, g_ht1, g_hu;
void hc_k_hash_clear_setup(const uint8_t* msg, uint32_t len) {
  Fp2 u0, u1;
  hash_to_field_fp2(msg, len, u0, u1);
  map_to_curve_g2_pair(u0, u1, g_hq0, g_hq1);
}
void hc_k_hash_clear_x1(void) {
  g_hq = jac_add_in<Fp2, true>(g_hq0, g_hq1);  // Q0 + Q1 (moved here from k_hash_map)
  g_ht1 = jac_neg(jac_mul_xabs_in2(g_hq));
  g_hu = jac_add_in<Fp2, true>(g_ht1, g2_psi(g_hq));
}
void hc_k_hash_clear_x2(void) { g_hu = jac_neg(jac_mul_xabs_in2(g_hu)); }
void hc_k_hash_clear_fin(void) {
  G2J t3 = g2_psi(g2_psi(jac_dbl_in(g_hq)));
  t3 = jac_add_in<Fp2, true>(t3, jac_neg(g2_psi(g_hq)));
  t3 = jac_add_in<Fp2, true>(t3, g_hu);
  t3 = jac_add_in<Fp2, true>(t3, jac_neg(g_ht1));
  (void)jac_add_in<Fp2, true>(t3, jac_neg(g_hq));
}
// k_hash_affine: one G2 to-affine conversion
void hc_k_g2_affine(void) {
  G2A a;
  (void)jac_to_aff(jac_dbl(jac_from_aff(g_sig)), a);
}
// k_rlc_g1_l0: [r] pk from the key's pair table (the bucket additions are k_msm_bucket_part's)
void hc_k_rlc_g1_l0(uint64_t r64) {
  G1A tab[PK_TAB_W2];
  hc_key_table_w2(tab);  // at key load
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  uint32_t u[4];
  rlc_digits(r64, u);
  (void)rlc_mul_key_w2(tab, fp_from_const(G1_BETA), u);
}
// k_msm_bucket_part: one bucket entry (psi^k of a signature, one mixed addition)
void hc_k_msm_entry(uint32_t k) {
  G2J acc = jac_dbl(jac_from_aff(g_sig));
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  G2A p = msm_psi_k(g_sig, k);
  (void)jac_add_aff_in(acc, p);
}
}  // extern "C"

#include "../../charon_amd/csrc/bls_batchinv.h"
// Montgomery's trick over workgroups (bls_batchinv.h, the device kernels'
// batched to-affine / SSWU inversions), emulated lane by lane: n canonical
// 48-byte big-endian values, present[i] = 0 marks an absent value (it takes
// part as 1 and gets 1 back).  Also the work-model probes of its cost.
extern "C" {
void hc_batch_inv(const uint8_t* in48, const uint8_t* present, int n, int waves, uint8_t* out48) {
  static Fp z[4096], r[4096];
  static bool pr[4096];
  if (n > 4096 || waves < 1 || waves > 16) return;
  for (int i = 0; i < n; ++i) {
    bool lt;
    z[i] = fp_to_mont(fp_limbs_from_be48(in48 + 48 * i, &lt));
    pr[i] = present[i] != 0;
  }
  batch_inv_emulate(z, pr, r, n, waves);
  for (int i = 0; i < n; ++i) fp_limbs_to_be48(fp_from_mont(r[i]), out48 + 48 * i);
}
// u32 mul-adds of one fp_inv, and of the batched trick over n values
void hc_fp_inv_once(void) {
  Fp a = fp_from_const(ONE_M);
  a = fp_add(a, a);
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  (void)fp_inv(a);
}
void hc_batch_inv_cost(int n, int waves) {
  static Fp z[4096], r[4096];
  static bool pr[4096];
  Fp a = fp_from_const(ONE_M);
  for (int i = 0; i < n && i < 4096; ++i) {
    a = fp_add(a, fp_from_const(ONE_M));
    z[i] = fp_reduce(a);
    pr[i] = true;
  }
#if defined(TBG_COUNT_OPS)
  tbg_mad_count = 0;
#endif
  batch_inv_emulate(z, pr, r, n, waves);
}
}  // extern "C"


#include "../../charon_amd/csrc/bls_row.h"
// Row Fp (bls_row.h): the row algorithms themselves, the row held whole on
// the host.  Limbs in and out as 14 signed 32-bit values.
extern "C" {
static R32 row_in(const int32_t* l) {
  R32 r;
  for (int k = 0; k < ROW_N; ++k) r.v[k] = k < NL ? l[k] : 0;
  return r;
}
static void row_out(const R32& r, int32_t* l) {
  for (int k = 0; k < NL; ++k) l[k] = r.v[k];
}
// returns the largest |limb| of the result (and checks lanes 14, 15 stay 0)
int hc_row_mul2(const int32_t* a, const int32_t* b, const int32_t* c, const int32_t* d, int32_t* out) {
  const R32 r = row_mul2(row_in(a), row_in(b), row_in(c), row_in(d));
  row_out(r, out);
  if (r.v[14] != 0 || r.v[15] != 0) return -1;
  int32_t mx = 0;
  for (int k = 0; k < NL - 1; ++k) mx = std::max(mx, std::abs(r.v[k]));
  return mx;
}
int hc_row_mul(const int32_t* a, const int32_t* b, int32_t* out) {
  const R32 r = row_mul(row_in(a), row_in(b));
  row_out(r, out);
  return (r.v[14] != 0 || r.v[15] != 0) ? -1 : 0;
}
void hc_row_reduce(const int32_t* a, int32_t* out) { row_out(row_reduce(r_norm(row_in(a))), out); }
void hc_row_norm(const int32_t* a, int32_t* out) { row_out(r_norm(row_in(a)), out); }
}
struct RowHostExec {
  template <class Fn>
  void operator()(Fn&& fn) {
    for (int r = 0; r < 64; ++r) fn(r);
  }
};
struct RowHostSolo {
  template <class Fn>
  void operator()(Fn&& fn) { fn(); }
};
static RowSlots g_rs;
extern "C" {
void hc_row_fp12_mul(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  RowHostExec ex;
  row_scatter(g_rs.v[1], f12_in(a));
  row_scatter(g_rs.v[2], f12_in(b));
  row_mul_to(ex, g_rs, 0, 1, 2);
  f12_out(row_gather(g_rs.v[0]), out);
}
void hc_row_fp12_cyc(const uint8_t* a, uint8_t* out) {
  RowHostExec ex;
  row_scatter(g_rs.v[0], f12_in(a));
  row_cyc_sqr(ex, g_rs, 0);
  f12_out(row_gather(g_rs.v[0]), out);
}
void hc_row_fp12_frob(const uint8_t* a, uint8_t* out) {
  RowHostExec ex;
  row_scatter(g_rs.v[1], f12_in(a));
  ex([&](int r) { row_frob(r, g_rs.v[0], g_rs.v[1]); });
  f12_out(row_gather(g_rs.v[0]), out);
}
int hc_row_final_exp(const uint8_t* a, uint8_t* out) {
  RowHostExec ex;
  RowHostSolo solo;
  row_scatter(g_rs.v[0], f12_in(a));
  row_final_exp(ex, solo, g_rs);
  f12_out(row_gather(g_rs.v[0]), out);
  return row_is_one(g_rs.v[0]) ? 1 : 0;
}
}
extern "C" {
// Bernstein-Yang inversion against Fermat: 0 on agreement
int hc_inv_bgcd(const uint8_t* a48, uint8_t* out48) {
  const Fp a = from_be(a48);
  const Fp r = fp_inv_bgcd(a), f = fp_inv_fermat(a);
  to_be(fp_canon(r), out48);
  return fp_eq(r, f) ? 0 : 1;
}
// the same value as a + p in [p, 2p) (device callers pass such values)
int hc_inv_bgcd_plus_p(const uint8_t* a48, uint8_t* out48) {
  const Fp a = from_be(a48);
  const Fp r = fp_inv_bgcd(fp_add(a, fp_from_const(P_L))), f = fp_inv_fermat(a);
  to_be(fp_canon(r), out48);
  return fp_eq(r, f) ? 0 : 1;
}
}
extern "C" {
// The 68 -g1-folded lines of an affine G2 point (4 x 48-byte coordinates,
// x.c0 x.c1 y.c0 y.c1) on rows (bls_row.h) against g2_lines: mismatching Fp count
int hc_row_lines(const uint8_t* q192) {
  static RowLineSlots S;
  static uint32_t ref[LINES_WORDS], got[LINES_WORDS];
  G2A Q{{from_be(q192), from_be(q192 + 48)}, {from_be(q192 + 96), from_be(q192 + 144)}};
  const Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X))), y = fp_from_const(G1_NEG_Y);
  g2_lines(Q, nx, y, ref);
  const Fp c[10] = {Q.x.c0, Q.x.c1, Q.y.c0, Q.y.c1, fp_one(), fp_zero(), Q.x.c0, Q.x.c1, Q.y.c0, Q.y.c1};
  for (int i = 0; i < 10; ++i) row_st(S.s[i], row_from_limbs(c[i].l));
  row_st(S.k[0], row_from_limbs(nx.l));
  row_st(S.k[1], row_from_limbs(y.l));
  RowHostExec ex;
  auto out6 = [&](int buf, int idx) {
    for (int k = 0; k < 6; ++k) rl_line_out(S, buf, k, got + LINE_WORDS * idx);
  };
  row_g2_lines(ex, out6, S);
  int bad = 0;
  for (int i = 0; i < N_LINES * 6; ++i) {
    Fp a, b;
    for (int j = 0; j < NL; ++j) { a.l[j] = ref[i * NL + j]; b.l[j] = got[i * NL + j]; }
    if (!fp_eq(a, b)) ++bad;
  }
  return bad;
}
}

#include "../../charon_amd/csrc/bls_rlc.h"
extern "C" {
// The batched subgroup test's coefficients of partial i (sgb_digits).
void hc_sgb_digits(const uint32_t* seed8, uint32_t i, int32_t* out18) {
  uint32_t seed[8];
  for (int k = 0; k < 8; ++k) seed[k] = seed8[k];
  int32_t c[18];
  sgb_digits(seed, i, c);
  for (int k = 0; k < 18; ++k) out18[k] = c[k];
}
// k_sgb.hip's test of one group, lane pairs emulated (Fp2p): the n 96-byte
// signatures of partials i0 .. i0 + n - 1 decoded WITHOUT the subgroup check
// (a decode failure leaves the partial out, as in the kernels), the 18
// bucket sums of each combination, Q_k by running sums, psi(Q_k) == [x] Q_k.
// Returns the bit mask of the combinations that failed (-1: bad argument).
int hc_sgb_group(const uint8_t* sigs96, int n, const uint32_t* seed8, uint32_t i0) {
  if (n < 0 || n > 512) return -1;
  uint32_t seed[8];
  for (int k = 0; k < 8; ++k) seed[k] = seed8[k];
  static G2A pts[512];
  static bool ok[512];
  for (int i = 0; i < n; ++i) ok[i] = g2_decompress_t<false, false>(sigs96 + 96 * i, pts[i]) == DEC_OK;
  int mask = 0;
  for (int k = 0; k < 18; ++k) {
    Jac<Fp2p> bucket[6];
    for (auto& b : bucket) b = jac_inf<Fp2p>();
    for (int i = 0; i < n; ++i) {
      if (!ok[i]) continue;
      int32_t c[18];
      sgb_digits(seed, i0 + (uint32_t)i, c);
      if (!c[k]) continue;
      Aff<Fp2p> p{pp_from(pts[i].x), f_reduce(pp_from(pts[i].y))};
      if (c[k] < 0) p.y = f_reduce(f_neg(p.y));
      bucket[(c[k] < 0 ? -c[k] : c[k]) - 1] = jac_add_aff_in(bucket[(c[k] < 0 ? -c[k] : c[k]) - 1], p);
    }
    Jac<Fp2p> run = jac_inf<Fp2p>(), q = run;
    for (int v = 6; v >= 1; --v) {
      run = jac_add_in<Fp2p, true>(run, bucket[v - 1]);
      q = jac_add_in<Fp2p, true>(q, run);
    }
    bool pass = true;
    if (!jac_is_inf(q)) {
      bool exc = false;
      const Jac<Fp2p> m = jac_mul_xabs_x(q, exc);
      if (exc || jac_is_inf(m)) {
        pass = false;
      } else {
        const Jac<Fp2p> ps = g2_psi_g(q);
        const Fp2p z1 = f_sqr(ps.Z), z2 = f_sqr(m.Z);
        pass = f_eq(f_mul(ps.X, z2), f_mul(m.X, z1)) &&
               f_eq(f_mul(f_mul(ps.Y, m.Z), z2), f_reduce(f_neg(f_mul(f_mul(m.Y, ps.Z), z1))));
      }
    }
    if (!pass) mask |= 1 << k;
  }
  return mask;
}
}
