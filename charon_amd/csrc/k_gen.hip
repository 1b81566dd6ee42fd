#include "tbls_launch.h"
#include "bls_h2c.h"

namespace tbg {

// ---- test-vector / benchmark-input generation (tbls.Sign / PartialSign,
// reference tbls/tss.go:200-217; sk -> pk as bls_sig.SecretKey.GetPublicKey) ----
// The results of [sk]G and [sk]H(m) are converted to affine with Fermat's
// constant-time inversion: their Z depends on the secret key.
// The double-and-add itself is not hardened (test-vector generation only,
// include/tbls_gpu.h).
template <class F>
__device__ bool jac_to_aff_ct(const Jac<F>& p, Aff<F>& out);
template <>
__device__ bool jac_to_aff_ct<Fp>(const G1J& p, G1A& out) {
  if (jac_is_inf(p)) return false;
  const Fp zi = fp_inv_fermat(p.Z), zi2 = fp_sqr(zi);
  out.x = fp_mul(p.X, zi2);
  out.y = fp_mul(p.Y, fp_mul(zi2, zi));
  return true;
}
template <>
__device__ bool jac_to_aff_ct<Fp2>(const G2J& p, G2A& out) {
  if (jac_is_inf(p)) return false;
  // 1 / (a + bu) = (a - bu) / (a^2 + b^2), the norm inverted by Fermat
  const Fp t = fp_inv_fermat(fp_mul2(p.Z.c0, p.Z.c0, p.Z.c1, p.Z.c1));
  const Fp2 zi = {fp_mul(p.Z.c0, t), fp_mul(fp_neg(fp_reduce(p.Z.c1)), t)};
  const Fp2 zi2 = fp2_sqr(zi);
  out.x = fp2_mul(p.X, zi2);
  out.y = fp2_mul(p.Y, fp2_mul(zi2, zi));
  return true;
}

TBG_HD void sk_words_from_be32(const uint8_t* b, uint32_t (&w)[8]) {
  for (int i = 0; i < 8; ++i)
    w[i] = ((uint32_t)b[31 - 4 * i]) | ((uint32_t)b[30 - 4 * i] << 8) | ((uint32_t)b[29 - 4 * i] << 16) |
           ((uint32_t)b[28 - 4 * i] << 24);
}

__global__ void __launch_bounds__(64) k_sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* pk48) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  sk_words_from_be32(sk32 + 32ull * i, w);
  G1J g = {fp_from_const(G1_X), fp_from_const(G1_Y), fp_one()};
  G1J p = jac_mul_words(g, w, 256);
  G1A a;
  bool ok = jac_to_aff_ct(p, a);
  uint8_t enc[48];
  g1_compress(a, !ok, enc);
  for (int j = 0; j < 48; ++j) pk48[48ull * i + j] = enc[j];
}

__global__ void __launch_bounds__(64) k_sign(const uint8_t* sk32, const uint32_t* item_msg, uint32_t n, const G2A* h_aff,
                                             const int32_t* h_status, uint8_t* sig96) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  sk_words_from_be32(sk32 + 32ull * i, w);
  uint32_t m = item_msg[i];
  G2A a;
  bool ok = false;
  if (h_status[m] == 0) {
    G2J p = jac_mul_words(jac_from_aff(h_aff[m]), w, 256);
    ok = jac_to_aff_ct(p, a);
  }
  uint8_t enc[96];
  g2_compress(a, !ok, enc);
  for (int j = 0; j < 96; ++j) sig96[96ull * i + j] = enc[j];
}

void launch_sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* pk48, hipStream_t st) {
  if (n) TBG_KLAUNCH(k_sk_to_pk, grid_for(n), dim3(kBlock), st, sk32, n, pk48);
}
void launch_sign(const uint8_t* sk32, const uint32_t* item_msg, uint32_t n, const G2A* h_aff, const int32_t* h_status,
                 uint8_t* sig96, hipStream_t st) {
  if (n) TBG_KLAUNCH(k_sign, grid_for(n), dim3(kBlock), st, sk32, item_msg, n, h_aff, h_status, sig96);
}

}  // namespace tbg
