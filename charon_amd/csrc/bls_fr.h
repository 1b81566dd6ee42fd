// Scalar field Fr of BLS12-381 (r, 255 bits): 10 limbs of 28 bits,
// Montgomery R = 2^280.  Only used for the Lagrange coefficients of the
// threshold recombination (kryptology CombineSignatures, reached from
// reference tbls/tss.go:142-149), so it favours simplicity over speed.
#pragma once
#include "bls_field.h"

namespace tbg {

struct Fr { uint32_t l[NLR]; };

TBG_HD Fr fr_zero() {
  Fr r;
  for (int i = 0; i < NLR; ++i) r.l[i] = 0;
  return r;
}

TBG_HD Fr fr_from_limbs(const uint32_t (&c)[NLR]) {
  Fr r;
  for (int i = 0; i < NLR; ++i) r.l[i] = c[i];
  return r;
}

// r = a - b mod r for canonical a, b (< r)
TBG_HD Fr fr_sub(const Fr& a, const Fr& b) {
  Fr d;
  int32_t borrow = 0;
  for (int i = 0; i < NLR; ++i) {
    int32_t s = (int32_t)a.l[i] - (int32_t)b.l[i] + borrow;
    d.l[i] = (uint32_t)s & LMASK;
    borrow = s >> 28;
  }
  if (borrow < 0) {
    uint32_t c = 0;
    for (int i = 0; i < NLR; ++i) {
      uint32_t s = d.l[i] + R_L[i] + c;
      d.l[i] = s & LMASK;
      c = s >> 28;
    }
  }
  return d;
}

// conditional subtract r (input < 2r)
TBG_HD Fr fr_csub(const Fr& a) {
  Fr d;
  int32_t borrow = 0;
  for (int i = 0; i < NLR; ++i) {
    int32_t s = (int32_t)a.l[i] - (int32_t)R_L[i] + borrow;
    d.l[i] = (uint32_t)s & LMASK;
    borrow = s >> 28;
  }
  return borrow < 0 ? a : d;
}

// Montgomery product, canonical output (< r).
TBG_HD Fr fr_mul(const Fr& a, const Fr& b) {
  uint32_t m[NLR];
  Fr r;
  uint64_t acc = 0;
  for (int k = 0; k < NLR; ++k) {
    uint64_t s = acc;
    for (int i = 0; i <= k; ++i) s += (uint64_t)a.l[i] * b.l[k - i];
    for (int i = 0; i < k; ++i) s += (uint64_t)m[i] * R_L[k - i];
    m[k] = ((uint32_t)s * RNINV) & LMASK;
    s += (uint64_t)m[k] * R_L[0];
    acc = s >> 28;
  }
  for (int k = NLR; k < 2 * NLR - 1; ++k) {
    uint64_t s = acc;
    for (int i = k - NLR + 1; i < NLR; ++i) s += (uint64_t)a.l[i] * b.l[k - i] + (uint64_t)m[i] * R_L[k - i];
    r.l[k - NLR] = (uint32_t)s & LMASK;
    acc = s >> 28;
  }
  r.l[NLR - 1] = (uint32_t)acc;
  return fr_csub(r);
}

TBG_HD Fr fr_from_u32(uint32_t v) {
  Fr a = fr_zero();
  a.l[0] = v & LMASK;
  a.l[1] = v >> 28;
  return fr_mul(a, fr_from_limbs(R_R2_M));
}

TBG_NI Fr fr_inv(const Fr& a) {
  Fr r = a;
  for (int i = EXP_R_INV_BITS - 2; i >= 0; --i) {
    r = fr_mul(r, r);
    if ((EXP_R_INV_WORDS[i >> 5] >> (i & 31)) & 1) r = fr_mul(r, a);
  }
  return r;
}

TBG_HD bool fr_is_zero(const Fr& a) {
  uint32_t o = 0;
  for (int i = 0; i < NLR; ++i) o |= a.l[i];
  return o == 0;
}

// Montgomery -> canonical little-endian 32-bit words (8 words, 255 bits used)
TBG_HD void fr_to_words(const Fr& a, uint32_t (&w)[8]) {
  Fr one = fr_zero();
  one.l[0] = 1;
  Fr c = fr_mul(a, one);
  for (int i = 0; i < 8; ++i) w[i] = 0;
  for (int i = 0; i < NLR; ++i) {
    int bit = 28 * i;
    w[bit >> 5] |= c.l[i] << (bit & 31);
    if ((bit & 31) > 4 && (bit >> 5) + 1 < 8) w[(bit >> 5) + 1] |= c.l[i] >> (32 - (bit & 31));
  }
}

}  // namespace tbg
