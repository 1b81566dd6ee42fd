// hash_to_G2 per distinct message (the H(m) of SigEth2.Verify, tss.go:190-197).
// The P == Q case of the mixed addition doubles inline (bls_curve.h): no
// out-of-line call inside the kernels' point loops.
#define TBG_ADD_DBL_INLINE 1
#include "tbls_launch.h"
#include "bls_h2c.h"

namespace tbg {

__global__ void TBG_LAUNCH k_hash_msgs(DevBatch B) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B.n_msgs) return;
  uint32_t off = B.msg_off[m], len = B.msg_off[m + 1] - off;
  G2J h = hash_to_g2_t<true>(B.msgs + off, len);
  G2A a;
  bool ok = jac_to_aff(h, a);
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  B.h_aff[m] = a;
  B.h_status[m] = ok ? 0 : 1;
}

void launch_hash_msgs(const DevBatch& B, hipStream_t st) {
  if (B.n_msgs) TBG_KLAUNCH(k_hash_msgs, grid_for(B.n_msgs), dim3(kBlock), st, B);
}

}  // namespace tbg
