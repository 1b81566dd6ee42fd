// Threshold recombination (kryptology SigEth2.CombineSignatures, reached from
// reference tbls/tss.go:142-149 and :181): sigma = sum_i lambda_i(0) sigma_i,
// lambda_i(0) = prod_{j != i} x_j / (x_j - x_i) mod r, x_i = Identifier.
#pragma once
#include "bls_fr.h"
#include "bls_curve.h"

namespace tbg {

// lambda_i(0) as canonical scalar words; false when two identifiers collide.
// ids: identifiers of the k participating partials, i: index into ids.
TBG_NI bool lagrange_at_zero_words(const uint8_t* ids, int k, int i, uint32_t (&w)[8]) {
  Fr one = fr_from_u32(1);
  Fr num = one, den = one;
  Fr xi = fr_from_u32(ids[i]);
  for (int j = 0; j < k; ++j) {
    if (j == i) continue;
    Fr xj = fr_from_u32(ids[j]);
    num = fr_mul(num, xj);
    den = fr_mul(den, fr_sub(xj, xi));
  }
  if (fr_is_zero(den)) return false;
  fr_to_words(fr_mul(num, fr_inv(den)), w);
  return true;
}

}  // namespace tbg
