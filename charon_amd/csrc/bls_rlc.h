// Random-linear-combination scalars and their application (k_rlc.hip).
//
// r_i is 64 secret random bits read as four 16-bit digits a_k of
//   r_i = a_0 + a_1 x + a_2 x^2 + a_3 x^3   (x = -0xd201000000010000).
// Distinct digit vectors give distinct r_i mod r (2^16 < |x| and
// 2^16 |x|^3 < r), so the usual RLC bound (a false accept <= 1/2^64) holds.
// For a signature s that passed the subgroup check psi(s) = [x] s, and on G1
// [x^2] = -phi (phi(x, y) = (beta x, y)), so
//   [r] s  = sum_k a_k psi^k(s)
//   [r] pk = a_0 pk + a_1 [x]pk - a_2 phi(pk) - a_3 phi([x]pk)
// are four-point Straus products with 16-bit scalars (15 doublings instead
// of 63), given [x]pk from the resident key table.
#pragma once
#include "bls_h2c.h"

namespace tbg {

// 64 bits of SHA-256's compression function keyed by the 32-byte batch seed.
TBG_HD uint64_t rlc_scalar(const uint32_t (&seed)[8], uint32_t i) {
  uint8_t blk[64];
  for (int k = 0; k < 8; ++k) {
    blk[4 * k] = (uint8_t)(seed[k] >> 24);
    blk[4 * k + 1] = (uint8_t)(seed[k] >> 16);
    blk[4 * k + 2] = (uint8_t)(seed[k] >> 8);
    blk[4 * k + 3] = (uint8_t)seed[k];
  }
  for (int k = 32; k < 64; ++k) blk[k] = 0;
  blk[32] = (uint8_t)(i >> 24);
  blk[33] = (uint8_t)(i >> 16);
  blk[34] = (uint8_t)(i >> 8);
  blk[35] = (uint8_t)i;
  blk[36] = 0x80;
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  sha256_block(h, blk);
  uint64_t r = ((uint64_t)h[0] << 32) | h[1];
  return r ? r : 1;
}

TBG_HD void rlc_digits(uint64_t r, uint32_t (&a)[4]) {
  for (int k = 0; k < 4; ++k) a[k] = (uint32_t)((r >> (16 * k)) & 0xFFFF);
}

TBG_HD G2A g2_psi_aff(const G2A& a) {
  return {fp2_mul(fp2_conj(a.x), fp2_from_const(PSI_X)), fp2_mul(fp2_conj(a.y), fp2_from_const(PSI_Y))};
}

// sum_k a_k psi^k(s) for s in G2 (affine), a_k < 2^16 (steps inlined: kernel callers)
TBG_HD G2J rlc_mul_g2(const G2A& s, const uint32_t (&a)[4]) {
  G2A q[4];
  q[0] = s;
  q[1] = g2_psi_aff(q[0]);
  q[2] = g2_psi_aff(q[1]);
  q[3] = g2_psi_aff(q[2]);
  G2J acc = jac_inf<Fp2>();
  bool started = false;
  for (int bit = 15; bit >= 0; --bit) {
    if (started) acc = jac_dbl_in(acc);
    for (int k = 0; k < 4; ++k)
      if ((a[k] >> bit) & 1) {
        acc = jac_add_aff_in(acc, q[k]);
        started = true;
      }
  }
  return acc;
}

// a_0 pk + a_1 xpk - a_2 phi(pk) - a_3 phi(xpk), xpk = [x]pk (steps inlined: kernel callers)
TBG_HD G1J rlc_mul_g1(const G1A& pk, const G1A& xpk, const uint32_t (&a)[4]) {
  const Fp beta = fp_from_const(G1_BETA);
  G1A q[4];
  q[0] = pk;
  q[1] = xpk;
  q[2] = {fp_mul(pk.x, beta), fp_reduce(fp_neg(pk.y))};
  q[3] = {fp_mul(xpk.x, beta), fp_reduce(fp_neg(xpk.y))};
  G1J acc = jac_inf<Fp>();
  bool started = false;
  for (int bit = 15; bit >= 0; --bit) {
    if (started) acc = jac_dbl_in(acc);
    for (int k = 0; k < 4; ++k)
      if ((a[k] >> bit) & 1) {
        acc = jac_add_aff_in(acc, q[k]);
        started = true;
      }
  }
  return acc;
}

}  // namespace tbg
