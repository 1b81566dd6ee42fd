// hash_to_G2 per distinct message (the H(m) of SigEth2.Verify, tss.go:190-197),
// in three kernels so each phase runs at the occupancy its own footprint
// allows (bls_pair.h):
//   k_hash_map     one lane per message: expand_message_xmd, hash_to_field,
//                  the two SSWU maps and 3-isogenies (Fp exponentiations),
//                  Q = Q0 + Q1 (Jacobian) into h_jac;
//   k_hash_clear   one lane per message: Budroni-Pintore cofactor clearing
//                  (one wave per SIMD: three live G2 points);
//   k_hash_affine  one lane per message: to affine (one inversion), status.
// The P == Q case of the mixed addition doubles inline (bls_curve.h): no
// out-of-line call inside the kernels' point loops.
#define TBG_ADD_DBL_INLINE 1
#include "tbls_launch.h"
#include "bls_h2c.h"

namespace tbg {

__global__ void TBG_LAUNCH_N(TBG_DECODE_WAVES) k_hash_map(DevBatch B) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B.n_msgs) return;
  const uint32_t off = B.msg_off[m], len = B.msg_off[m + 1] - off;
  Fp2 u0, u1;
  hash_to_field_fp2(B.msgs + off, len, u0, u1);
  G2J q0, q1;
  map_to_curve_g2_pair(u0, u1, q0, q1);
  B.h_jac[m] = jac_add(q0, q1);
}

__global__ void TBG_LAUNCH_N(TBG_DECODE_WAVES) k_hash_affine(DevBatch B) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B.n_msgs) return;
  G2A a;
  const bool ok = jac_to_aff(B.h_jac[m], a);
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  B.h_aff[m] = a;
  B.h_status[m] = ok ? 0 : 1;
}

void launch_hash_msgs(const DevBatch& B, hipStream_t st) {
  if (!B.n_msgs) return;
  TBG_KLAUNCH(k_hash_map, grid_for(B.n_msgs), dim3(kBlock), st, B);
  launch_hash_clear(B, st);  // k_hash_clear.hip
  TBG_KLAUNCH(k_hash_affine, grid_for(B.n_msgs), dim3(kBlock), st, B);
}

}  // namespace tbg
