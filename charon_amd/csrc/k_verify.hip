// Per-partial BLS CoreVerify e(pk, H(m)) e(-g1, sig) == 1 (tbls.Verify,
// reference tbls/tss.go:190-197), in two stages:
//   k_lines_sig / k_lines_h   68 Miller lines per signature (with -g1 folded
//                             in) and per message (G1 factor left out), one
//                             thread per G2 point
//   k_verify_quad             one quad of lanes per partial: the 2-pair Miller
//                             accumulation over the stored lines and the
//                             final exponentiation, Fp12 split over the
//                             lanes (bls_quad.h)
#include "tbls_launch.h"
#include "bls_lines.h"
#include "bls_quad.h"

#ifndef TBG_VERIFY_WAVES
#define TBG_VERIFY_WAVES 1  // minimum waves per SIMD requested for k_verify_quad
#endif

namespace tbg {

__global__ void __launch_bounds__(64) k_lines_sig(DevBatch B) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials) return;
  if (B.partial_status[i] != TBG_PS_NOT_VERIFIED) return;
  Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));   // P = -g1: -x = -G1_X, y = -G1_Y
  Fp y = fp_from_const(G1_NEG_Y);
  g2_lines(B.sig_aff[i], nx, y, B.sig_lines + (size_t)LINES_WORDS * i);
}

__global__ void __launch_bounds__(64) k_lines_h(DevBatch B) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B.n_msgs) return;
  if (B.h_status[m] != 0) return;
  g2_lines(B.h_aff[m], fp_one(), fp_one(), B.h_lines + (size_t)LINES_WORDS * m);
}

__global__ void __launch_bounds__(64, TBG_VERIFY_WAVES) k_verify_quad(DevBatch B, const G1A* pk_aff, const int32_t* pk_status,
                                                    uint32_t n_pk) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t i = t >> 2;
  if (i >= B.n_partials) return;  // whole quads leave together
  const bool lead = (t & 3) == 0;
  if (B.partial_status[i] != TBG_PS_NOT_VERIFIED) return;  // decode error already recorded
  uint32_t pid = B.pubkey_ids[i];
  if (pid >= n_pk || pk_status[pid] != DEC_OK) {
    if (lead) B.partial_status[i] = TBG_PS_ERR_PUBKEY;
    return;
  }
  uint32_t m = B.duty_msg[B.partial_duty[i]];
  if (B.h_status[m] != 0) {
    if (lead) B.partial_status[i] = TBG_PS_INVALID;
    return;
  }
  G1A pk = pk_aff[pid];
  Fp nx = fp_reduce(fp_neg(pk.x));
  const uint32_t* ls = B.sig_lines + (size_t)LINES_WORDS * i;
  const uint32_t* lh = B.h_lines + (size_t)LINES_WORDS * m;
  Fp4 f = quad_one();
  int idx = 0;
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = quad_sqr(f);
    int steps = ((X_ABS >> b) & 1) ? 2 : 1;
    for (int s = 0; s < steps; ++s, ++idx) {
      Line a = line_load(ls + LINE_WORDS * idx);
      f = quad_line(f, a.l0, a.l1, a.l4);
      Line h = line_load(lh + LINE_WORDS * idx);
      f = quad_line(f, h.l0, fp2_mul_fp(h.l1, nx), fp2_mul_fp(h.l4, pk.y));
    }
  }
  f = quad_final_exp(quad_conj(f));
  bool ok = quad_is_one(f);
  if (lead) B.partial_status[i] = ok ? TBG_PS_VALID : TBG_PS_INVALID;
}

void launch_lines(const DevBatch& B, hipStream_t st_sig, hipStream_t st_h) {
  if (B.n_partials) hipLaunchKernelGGL(k_lines_sig, grid_for(B.n_partials), dim3(kBlock), 0, st_sig, B);
  if (B.n_msgs) hipLaunchKernelGGL(k_lines_h, grid_for(B.n_msgs), dim3(kBlock), 0, st_h, B);
}

void launch_verify(const DevBatch& B, const G1A* pk_aff, const int32_t* pk_status, uint32_t n_pk, hipStream_t st) {
  if (B.n_partials)
    hipLaunchKernelGGL(k_verify_quad, grid_for(4 * B.n_partials), dim3(kBlock), 0, st, B, pk_aff, pk_status, n_pk);
}

}  // namespace tbg
