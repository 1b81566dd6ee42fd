// Host build of the engine's device math (the same headers the HIP kernels
// use), exported as plain C for the CPU test suite.  TEST TOOLING ONLY: this
// library is never loaded by the product (charon_amd loads libtbls_gpu.so
// and fails loudly without a GPU); it lets the kernel arithmetic be checked
// against the oracle on a machine with no GPU, with value-bound assertions
// (TBG_BOUNDS_CHECK) switched on.
#include <cstdint>
#include <cstring>
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
void hc_final_exp(const uint8_t* a, uint8_t* out) { f12_out(final_exp(f12_in(a)), out); }

// G2 decompress -> status; on success writes the recompressed encoding and
// affine coordinates (x0, x1, y0, y1; 48 bytes each).
int hc_g2_decompress(const uint8_t* in, uint8_t* aff_out) {
  G2A a;
  int st = g2_decompress(in, a);
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
  return g2_decompress(sig96, a);
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
    if (g2_decompress(sigs96 + 96 * i, pts[i]) != DEC_OK) return -2;
  for (int i = 0; i < k; ++i)
    if (!lagrange_at_zero_words(ids, k, i, lam[i])) return -3;
  G2J acc = jac_inf<Fp2>();
  for (int bit = 254; bit >= 0; --bit) {
    acc = jac_dbl(acc);
    for (int j = 0; j < k; ++j)
      if ((lam[j][bit >> 5] >> (bit & 31)) & 1) acc = jac_add_aff(acc, pts[j]);
  }
  G2A a;
  bool ok = jac_to_aff(acc, a);
  g2_compress(a, !ok, out96);
  return ok ? 0 : -4;
}
}
