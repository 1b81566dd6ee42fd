// hash_to_G2 per distinct message (the H(m) of SigEth2.Verify, tss.go:190-197),
// in three kernels so each phase runs at the occupancy its own footprint
// allows (bls_pair.h):
//   k_hash_map     one lane per message: expand_message_xmd, hash_to_field,
//                  the two SSWU maps and 3-isogenies (Fp exponentiations),
//                  Q0 and Q1 (Jacobian) into h_jac (k_hash_clear_x1 adds them);
//   k_hash_clear   one lane per message: Budroni-Pintore cofactor clearing
//                  (one wave per SIMD: three live G2 points);
//   k_hash_affine  one lane per message: to affine (inversion batched over
//                  the workgroup), status.
// The P == Q case of the mixed addition doubles inline (bls_curve.h): no
// out-of-line call inside the kernels' point loops.
#define TBG_ADD_DBL_INLINE 1
#include "tbls_launch.h"
#include "bls_h2c.h"
#include "bls_batchinv.h"

namespace tbg {

// The SSWU denominators' inversion and the affine conversion are batched
// over the workgroup (Montgomery's trick, bls_batchinv.h): one field
// inversion per BINV_BLOCK messages instead of one per message.
__global__ void __launch_bounds__(BINV_BLOCK, TBG_DECODE_WAVES) k_hash_map(DevBatch B) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = m < B.n_msgs;
  Fp2 u0 = fp2_zero(), u1 = fp2_zero();
  if (in) {
    const uint32_t off = B.msg_off[m], len = B.msg_off[m + 1] - off;
    hash_to_field_fp2(B.msgs + off, len, u0, u1);
  }
  SswuPair w;
  const Fp2 dd = sswu_pair_den(u0, u1, w);
  const bool ok = in && !fp2_is_zero(dd);
  const Fp2 di = block_batch_inv2<BINV_WAVES>(dd, ok);  // every thread of the workgroup
  if (!in) return;
  G2J q0, q1;
  sswu_pair_finish(u0, u1, w, ok, di, q0, q1);
  // Q0 + Q1 is the first step of k_hash_clear_x1 (a lane pair per message):
  // here the out-of-line G2 addition saved and restored ~360 callee-saved
  // VGPR words through scratch per message
  B.h_jac[m] = q0;
  B.h_jac[B.n_msgs + m] = q1;
}

__global__ void __launch_bounds__(BINV_BLOCK, TBG_DECODE_WAVES) k_hash_affine(DevBatch B) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = m < B.n_msgs;
  const G2J p = in ? B.h_jac[m] : jac_inf<Fp2>();
  G2A a;
  const bool ok = block_jac_to_aff<BINV_WAVES>(p, in, a);  // every thread of the workgroup
  if (!in) return;
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  B.h_aff[m] = a;
  B.h_status[m] = ok ? 0 : 1;
}

void launch_hash_msgs(const DevBatch& B, hipStream_t st) {
  if (!B.n_msgs) return;
  const dim3 grid((B.n_msgs + BINV_BLOCK - 1) / BINV_BLOCK);
  TBG_KLAUNCH(k_hash_map, grid, dim3(BINV_BLOCK), st, B);
  launch_hash_clear(B, st);  // k_hash_clear.hip
  TBG_KLAUNCH(k_hash_affine, grid, dim3(BINV_BLOCK), st, B);
}

}  // namespace tbg
