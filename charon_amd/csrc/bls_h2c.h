// hash_to_curve for G2 (RFC 9380 suite BLS12381G2_XMD:SHA-256_SSWU_RO_) with
// the proof-of-possession DST used by kryptology's SigEth2 (reference
// tbls/tss.go:28-31): expand_message_xmd(SHA-256) -> hash_to_field (Fp2, 2
// elements) -> simplified SWU on E2' -> 3-isogeny -> sum -> cofactor clearing.
#pragma once
#include "bls_curve.h"

namespace tbg {

// ------------------------------------------------------------------ SHA-256
struct Sha256 {
  uint32_t h[8];
  uint8_t buf[64];
  uint32_t nbuf;
  uint64_t total;
};

TBG_HD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

TBG_HD void sha256_init(Sha256& s) {
  const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                          0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  for (int i = 0; i < 8; ++i) s.h[i] = iv[i];
  s.nbuf = 0;
  s.total = 0;
}

TBG_NI void sha256_block(uint32_t (&h)[8], const uint8_t* blk) {
  const uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + K[i] + w[i];
    uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

TBG_HD void sha256_byte(Sha256& s, uint8_t v) {
  s.buf[s.nbuf++] = v;
  s.total++;
  if (s.nbuf == 64) {
    sha256_block(s.h, s.buf);
    s.nbuf = 0;
  }
}

TBG_HD void sha256_update(Sha256& s, const uint8_t* p, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) sha256_byte(s, p[i]);
}

TBG_HD void sha256_final(Sha256& s, uint8_t* out) {
  uint64_t bits = s.total * 8;
  sha256_byte(s, 0x80);
  while (s.nbuf != 56) sha256_byte(s, 0);
  for (int i = 7; i >= 0; --i) sha256_byte(s, (uint8_t)(bits >> (8 * i)));
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(s.h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(s.h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(s.h[i] >> 8);
    out[4 * i + 3] = (uint8_t)s.h[i];
  }
}

// DST = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_" (43 bytes)
constexpr int DST_LEN = 43;
TBG_HD uint8_t dst_byte(int i) {
  const char d[DST_LEN + 1] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
  return (uint8_t)d[i];
}
TBG_HD void sha256_dst_prime(Sha256& s) {
  for (int i = 0; i < DST_LEN; ++i) sha256_byte(s, dst_byte(i));
  sha256_byte(s, (uint8_t)DST_LEN);
}

// expand_message_xmd(msg, DST, 256): out[256]  (byte-stream reference form;
// the kernels use the word form of hash_to_field_fp2 below)
TBG_NI void expand_message_xmd_256(const uint8_t* msg, uint32_t msg_len, uint8_t* out) {
  Sha256 s;
  sha256_init(s);
  for (int i = 0; i < 64; ++i) sha256_byte(s, 0);
  sha256_update(s, msg, msg_len);
  sha256_byte(s, 0x01);  // l_i_b_str = I2OSP(256, 2)
  sha256_byte(s, 0x00);
  sha256_byte(s, 0x00);  // I2OSP(0, 1)
  sha256_dst_prime(s);
  uint8_t b0[32];
  sha256_final(s, b0);
  uint8_t bi[32];
  for (int i = 1; i <= 8; ++i) {
    sha256_init(s);
    if (i == 1) {
      sha256_update(s, b0, 32);
    } else {
      for (int j = 0; j < 32; ++j) sha256_byte(s, b0[j] ^ bi[j]);
    }
    sha256_byte(s, (uint8_t)i);
    sha256_dst_prime(s);
    sha256_final(s, bi);
    for (int j = 0; j < 32; ++j) out[32 * (i - 1) + j] = bi[j];
  }
}

// ---- word-oriented form: every block is 16 big-endian words built in
// registers and compressed with a fully unrolled, 16-word rolling schedule
// (the byte-stream form above keeps its buffers and the 64-word schedule in
// scratch memory: ~14 KB of scratch traffic per message).
TBG_HD constexpr uint32_t dstp_byte(int i) {  // DST_prime = DST || I2OSP(len(DST), 1)
  return i < DST_LEN ? (uint32_t)(uint8_t)"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"[i] : (uint32_t)DST_LEN;
}
TBG_HD constexpr uint32_t dstp_word(int i) {  // big-endian word of DST_prime bytes [i, i + 4)
  return (dstp_byte(i) << 24) | (dstp_byte(i + 1) << 16) | (dstp_byte(i + 2) << 8) | dstp_byte(i + 3);
}

TBG_HD void sha256_compress(uint32_t (&h)[8], uint32_t (&w)[16]) {
  constexpr uint32_t K[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    if (i >= 16) {
      const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
      const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
      w[i & 15] += s0 + w[(i - 7) & 15] + s1;
    }
    const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + K[i] + w[i & 15];
    const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

TBG_HD void sha256_iv(uint32_t (&h)[8]) {
  h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
  h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
}

// Byte p of b_0's input after Z_pad: msg || I2OSP(256, 2) || I2OSP(0, 1) ||
// DST_prime || 0x80 || 0...; the last 8 bytes of block nb - 1 carry the bit
// length (with Z_pad) and are filled in by the caller.
TBG_HD uint32_t b0_stream_byte(const uint8_t* msg, uint32_t L, uint32_t p) {
  if (p < L) return msg[p];
  if (p == L) return 0x01;
  if (p < L + 3) return 0x00;
  if (p < L + 3 + DST_LEN + 1) return dstp_byte((int)(p - L - 3));
  return p == L + 3 + DST_LEN + 1 ? 0x80u : 0u;
}

// 32 big-endian bytes -> 14 limbs (value < 2^256)
TBG_HD Fp limbs_from_be32(const uint8_t* b) {
  Fp r = fp_zero();
  for (int j = 0; j < 32; ++j) {
    int bit = 8 * (31 - j);
    uint32_t v = b[j];
    int li = bit / 28, off = bit % 28;
    r.l[li] |= (v << off) & LMASK;
    if (off > 20) r.l[li + 1] |= v >> (28 - off);
  }
  return r;
}

// 64 big-endian bytes mod p, in Montgomery form: REDC(hi * 2^256 R^2 + lo * R^2)
TBG_HD Fp fp_from_be64_mod(const uint8_t* b) {
  Fp hi = limbs_from_be32(b), lo = limbs_from_be32(b + 32);
  Fp ca = fp_from_const(R2_2E256_M), cb = fp_from_const(R2_M);
  return fp_mul2(hi, ca, lo, cb);
}

// 8 big-endian words (a 256-bit value) -> 14 limbs
TBG_HD Fp limbs_from_be_words8(const uint32_t* w) {
  Fp r = fp_zero();
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int bit = 32 * (7 - j);  // position of word j's lowest bit
    const uint32_t v = w[j];
    const int li = bit / 28, off = bit % 28;
    r.l[li] |= (v << off) & LMASK;
    if (li + 1 < NL) r.l[li + 1] |= (v >> (28 - off)) & LMASK;
    if (off > 24 && li + 2 < NL) r.l[li + 2] |= v >> (56 - off);
  }
  return r;
}

// 16 big-endian words mod p, in Montgomery form (as fp_from_be64_mod)
TBG_HD Fp fp_from_be_words16_mod(const uint32_t* w) {
  Fp hi = limbs_from_be_words8(w), lo = limbs_from_be_words8(w + 8);
  Fp ca = fp_from_const(R2_2E256_M), cb = fp_from_const(R2_M);
  return fp_mul2(hi, ca, lo, cb);
}

// expand_message_xmd's b_1 .. b_8 in pairs: pair k (b_(2k+1) || b_(2k+2)) is
// the 16 words of one hash_to_field element, converted as soon as it is
// complete (a per-pair loop keeps every word index static: no 64-word array
// in scratch).
TBG_HD void hash_to_field_fp2(const uint8_t* msg, uint32_t L, Fp2& u0, Fp2& u1) {
  uint32_t h[8], w[16];
  sha256_iv(h);
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = 0;
  sha256_compress(h, w);  // Z_pad: one block of zeros
  const uint32_t tail = L + 3 + DST_LEN + 1;
  const uint32_t nb = (tail + 1 + 8 + 63) / 64;
  const uint64_t bits = 8ull * (64 + tail);
#pragma unroll 1
  for (uint32_t blk = 0; blk < nb; ++blk) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t p = 64 * blk + 4 * k;
      w[k] = (b0_stream_byte(msg, L, p) << 24) | (b0_stream_byte(msg, L, p + 1) << 16) |
             (b0_stream_byte(msg, L, p + 2) << 8) | b0_stream_byte(msg, L, p + 3);
    }
    if (blk == nb - 1) {
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    sha256_compress(h, w);
  }
  uint32_t b0[8], bi[8], grp[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    b0[k] = h[k];
    bi[k] = 0;
  }
  Fp e[4] = {fp_zero(), fp_zero(), fp_zero(), fp_zero()};
#pragma unroll 1
  for (uint32_t pr = 0; pr < 4; ++pr) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const uint32_t i = 2 * pr + half + 1;
#pragma unroll
      for (int k = 0; k < 8; ++k) w[k] = b0[k] ^ bi[k];
      w[8] = (i << 24) | (dstp_byte(0) << 16) | (dstp_byte(1) << 8) | dstp_byte(2);
#pragma unroll
      for (int k = 9; k < 16; ++k) w[k] = dstp_word(3 + 4 * (k - 9));
      sha256_iv(h);
      sha256_compress(h, w);
      w[0] = dstp_word(31);
      w[1] = dstp_word(35);
      w[2] = dstp_word(39);
      w[3] = (dstp_byte(43) << 24) | 0x800000u;
#pragma unroll
      for (int k = 4; k < 15; ++k) w[k] = 0;
      w[15] = 77 * 8;
      sha256_compress(h, w);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bi[k] = h[k];
        grp[8 * half + k] = h[k];
      }
    }
    const Fp v = fp_from_be_words16_mod(grp);
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = fp_select(pr == (uint32_t)k, v, e[k]);
  }
  u0 = Fp2{e[0], e[1]};
  u1 = Fp2{e[2], e[3]};
}

// the byte-stream reference form (host tests compare the two)
TBG_HD void hash_to_field_fp2_bytes(const uint8_t* msg, uint32_t msg_len, Fp2& u0, Fp2& u1) {
  uint8_t uni[256];
  expand_message_xmd_256(msg, msg_len, uni);
  u0.c0 = fp_from_be64_mod(uni);
  u0.c1 = fp_from_be64_mod(uni + 64);
  u1.c0 = fp_from_be64_mod(uni + 128);
  u1.c1 = fp_from_be64_mod(uni + 192);
}

TBG_NI G2J iso3_to_jac(const Fp2& x, const Fp2& y);

// Simplified SWU to E2' then the 3-isogeny to E2, output Jacobian on E2.
// Reference form (straight from RFC 9380 section 6.6.2); hash_to_g2 uses
// map_to_curve_g2_pair below and falls back here only on exceptional inputs.
TBG_NI G2J map_to_curve_g2(const Fp2& u) {
  Fp2 A = fp2_from_const(SSWU_A), B = fp2_from_const(SSWU_B), Z = fp2_from_const(SSWU_Z);
  Fp2 u2 = fp2_sqr(u);
  Fp2 zu2 = fp2_mul(Z, u2);
  Fp2 den = fp2_reduce(fp2_add(fp2_sqr(zu2), zu2));
  Fp2 x1;
  if (fp2_is_zero(den)) {
    x1 = fp2_from_const(SSWU_B_OVER_ZA);
  } else {
    Fp2 t = fp2_reduce(fp2_add(fp2_one(), fp2_inv(den)));
    x1 = fp2_mul(fp2_from_const(SSWU_NEG_B_OVER_A), t);
  }
  Fp2 gx1 = fp2_reduce(fp2_add(fp2_add(fp2_mul(fp2_sqr(x1), x1), fp2_mul(A, x1)), B));
  Fp2 x, y;
  if (fp2_sqrt(gx1, y)) {
    x = x1;
  } else {
    x = fp2_mul(zu2, x1);
    Fp2 gx2 = fp2_reduce(fp2_add(fp2_add(fp2_mul(fp2_sqr(x), x), fp2_mul(A, x)), B));
    fp2_sqrt(gx2, y);  // always a square when gx1 is not
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_reduce(fp2_neg(y));
  return iso3_to_jac(x, y);
}

// 3-isogeny E2' -> E2 of an affine point: x = x_num / x_den, y = y' y_num /
// y_den, as Jacobian (X, Y, Z) = (x_num y_den Z, y' y_num x_den Z^2, Z) with
// Z = x_den y_den (X / Z^2 = x_num / x_den, Y / Z^3 = y' y_num / y_den).  The
// four polynomials by Horner's rule in x (K13 and K33 are in Fp): 15 Fp2
// products, two of them by an Fp constant, and few live
// values (the output's coordinates are written as soon as they are formed --
// Out is a G2J in registers, or a kernel's slot in memory).
template <class Out>
TBG_HD void iso3_emit(const Fp2& x, const Fp2& y, Out& r) {
  auto hstep = [&](const Fp2& acc, const Fp2Const& k) { return fp2_reduce(fp2_add(fp2_mul(acc, x), fp2_from_const(k))); };
  const Fp2 xden = hstep(fp2_reduce(fp2_add(x, fp2_from_const(ISO_K21))), ISO_K20);
  const Fp2 yden = hstep(hstep(fp2_reduce(fp2_add(x, fp2_from_const(ISO_K42))), ISO_K41), ISO_K40);
  const Fp2 z = fp2_mul(xden, yden);
  r.Z = z;
  const Fp2 xnum = hstep(hstep(fp2_reduce(fp2_add(fp2_mul_fp(x, fp_from_const(ISO_K13.c0)), fp2_from_const(ISO_K12))), ISO_K11),
                         ISO_K10);
  r.X = fp2_mul(fp2_mul(xnum, yden), z);
  const Fp2 ynum = hstep(hstep(fp2_reduce(fp2_add(fp2_mul_fp(x, fp_from_const(ISO_K33.c0)), fp2_from_const(ISO_K32))), ISO_K31),
                         ISO_K30);
  r.Y = fp2_mul(fp2_mul(fp2_mul(y, ynum), xden), fp2_sqr(z));
}
TBG_HD G2J iso3_to_jac_in(const Fp2& x, const Fp2& y) {
  G2J r;
  iso3_emit(x, y, r);
  return r;
}
TBG_NI G2J iso3_to_jac(const Fp2& x, const Fp2& y) { return iso3_to_jac_in(x, y); }

// Root of a or of Z a, whichever is a square (a non-square in Fp2 times the
// non-square Z is a square), from one Fp exponentiation on the norm plus one
// for the root (norm method, as fp2_sqrt).  sq reports which.  False on the
// inputs the closed form does not cover (a.c1 == 0 or (Z a).c1 == 0), which
// the caller routes to the reference path.
// (RegKeep, the keeper of fp2_sqrt_or_z_in's input: bls_tower.h)
// k_hash_sswu's exponentiation window: width 4 (eight odd powers) spills 27
// VGPRs there and still runs 4.99 vs 5.24 ms per 160k-message launch at
// width 3 (profiles/r06/hash).
#ifndef TBG_SSWU_WIN
#define TBG_SSWU_WIN 4
#endif
constexpr int SSWU_WIN = TBG_SSWU_WIN;
template <int WIN = 4, class Keep = RegKeep>
TBG_HD bool fp2_sqrt_or_z_in(const Fp2& a_in, Fp2& root, bool& sq, Keep keep = Keep{}) {
  Fp2 a = fp2_reduce(a_in);
  keep.put(a);
  Fp gamma = fp_pow_const_in<EXP_SQRT_BITS, EXP_SQRT_WORDS, WIN>(fp_mul2(a.c0, a.c0, a.c1, a.c1));
  a = keep.get();
  sq = fp_eq(fp_sqr(gamma), fp_mul2(a.c0, a.c0, a.c1, a.c1));
  if (!sq) {
    // gamma^2 = -norm(a); K gamma is a root of norm(Z) norm(a) = norm(Z a)
    a = fp2_reduce(fp2_mul(fp2_from_const(SSWU_Z), a));
    gamma = fp_mul(gamma, fp_from_const(SSWU_SQRT_NEG_NORM_Z));
  }
  if (fp_is_zero(a.c1)) return false;
  keep.put(a);
  const Fp inv2 = fp_from_const(INV2_M);
  const Fp delta = fp_mul(fp_add(a.c0, gamma), inv2);
  const Fp t = fp_pow_const_in<EXP_PM3D4_BITS, EXP_PM3D4_WORDS, WIN>(delta);  // delta^((p-3)/4)
  a = keep.get();
  const Fp x0 = fp_mul(delta, t);
  const Fp h = fp_mul(fp_mul(a.c1, t), inv2);
  const bool res = fp_eq(fp_sqr(x0), delta);
  const Fp2 r = {fp_select(res, x0, h), fp_select(res, h, fp_reduce(fp_neg(x0)))};
  root = r;
  return fp2_eq(fp2_sqr(r), a);
}
TBG_NI bool fp2_sqrt_or_z(const Fp2& a_in, Fp2& root, bool& sq) { return fp2_sqrt_or_z_in(a_in, root, sq); }

// SSWU of both hash_to_field outputs with uniform control flow: one Fp2
// inversion for the two denominators (Montgomery's trick) and one square
// root per map -- when g(x1) is not a square, x2 = Z u^2 x1 and
// g(x2) = Z^3 u^6 g(x1), so sqrt(g(x2)) = Z u^3 sqrt(Z g(x1)).
// (The reference form tries sqrt(g(x1)), then sqrt(g(x2)): 1-2 roots and
// an inversion per map, divergent across a wave.)
// In two halves around that inversion, so a kernel can batch it across its
// workgroup (k_hash_map, bls_batchinv.h): sswu_pair_den forms the product dd
// of the two denominators, sswu_pair_finish takes di = 1 / dd.
struct SswuPair {
  Fp2 den[2];
};
// den = (Z u^2)^2 + Z u^2 of one map
TBG_HD Fp2 sswu_den(const Fp2& u) {
  const Fp2 zu2 = fp2_reduce(fp2_mul(fp2_from_const(SSWU_Z), fp2_sqr(u)));
  return fp2_reduce(fp2_add(fp2_sqr(zu2), zu2));
}
TBG_HD Fp2 sswu_pair_den(const Fp2& u0, const Fp2& u1, SswuPair& w) {
  w.den[0] = sswu_den(u0);
  w.den[1] = sswu_den(u1);
  return fp2_reduce(fp2_mul(w.den[0], w.den[1]));
}
// x1 = -B/A (1 + 1/den) of one map from its inverse denominator.
TBG_HD Fp2 sswu_x1(const Fp2& inv) {
  return fp2_mul(fp2_from_const(SSWU_NEG_B_OVER_A), fp2_reduce(fp2_add(fp2_one(), inv)));
}
// One map from its u and x1 (the second half of k_hash.hip's split), in
// three steps a kernel can keep apart: g(x1); the root of g(x1) or of Z g(x1)
// (fp2_sqrt_or_z_in); x, y (Z u^2 recomputed, as sswu_pair_den forms it).
TBG_HD Fp2 sswu_gx(const Fp2& x1) {
  const Fp2 A = fp2_from_const(SSWU_A), B = fp2_from_const(SSWU_B);
  return fp2_reduce(fp2_add(fp2_add(fp2_mul(fp2_sqr(x1), x1), fp2_mul(A, x1)), B));
}
TBG_HD void sswu_xy(const Fp2& u, const Fp2& x1, const Fp2& r, bool sq, Fp2& x, Fp2& y) {
  const Fp2 Z = fp2_from_const(SSWU_Z);
  const Fp2 u2 = fp2_sqr(u);
  x = sq ? x1 : fp2_mul(fp2_reduce(fp2_mul(Z, u2)), x1);
  y = sq ? r : fp2_mul(fp2_mul(Z, fp2_mul(u2, u)), r);
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_reduce(fp2_neg(y));
}
// ... composed; false on the exceptional inputs fp2_sqrt_or_z does not cover
TBG_HD bool sswu_map_x1(const Fp2& u, const Fp2& x1, G2J& q) {
  Fp2 r, x, y;
  bool sq;
  if (!fp2_sqrt_or_z_in<SSWU_WIN>(sswu_gx(x1), r, sq)) return false;  // (k_hash_sswu's window width)
  sswu_xy(u, x1, r, sq, x, y);
  iso3_emit(x, y, q);
  return true;
}
TBG_NI void sswu_pair_finish(const Fp2& u0, const Fp2& u1, const SswuPair& w, bool ok, const Fp2& di, G2J& q0,
                             G2J& q1) {
  const Fp2* u[2] = {&u0, &u1};
  Fp2 inv[2] = {fp2_mul(w.den[1], di), fp2_mul(w.den[0], di)};
  G2J* out[2] = {&q0, &q1};
  for (int j = 0; j < 2 && ok; ++j)
    if (!sswu_map_x1(*u[j], sswu_x1(inv[j]), *out[j])) ok = false;
  if (!ok) {  // exceptional inputs (probability ~2^-380 per hash): reference path
    q0 = map_to_curve_g2(u0);
    q1 = map_to_curve_g2(u1);
  }
}
TBG_NI void map_to_curve_g2_pair(const Fp2& u0, const Fp2& u1, G2J& q0, G2J& q1) {
  SswuPair w;
  const Fp2 dd = sswu_pair_den(u0, u1, w);
  const bool ok = !fp2_is_zero(dd);
  sswu_pair_finish(u0, u1, w, ok, fp2_inv(dd), q0, q1);
}

// H(m) in G2 (Jacobian).  INL = true inlines the cofactor clearing's
// doublings (kernel callers only).
template <bool INL>
TBG_HD G2J hash_to_g2_t(const uint8_t* msg, uint32_t msg_len) {
  Fp2 u0, u1;
  hash_to_field_fp2(msg, msg_len, u0, u1);
  G2J q0, q1;
  map_to_curve_g2_pair(u0, u1, q0, q1);
  return g2_clear_cofactor_t<INL>(jac_add(q0, q1));
}
TBG_NI G2J hash_to_g2(const uint8_t* msg, uint32_t msg_len) { return hash_to_g2_t<false>(msg, msg_len); }

}  // namespace tbg
