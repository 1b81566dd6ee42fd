// Cofactor clearing of hash_to_G2 (the middle kernel of k_hash.hip's chain),
// in its own translation unit: device functions shared with the two-wave
// kernels of k_hash.hip would otherwise be compiled for this kernel's
// unconstrained register budget, and a kernel inherits its callees' count
// (k_hash_map dropped to one wave per SIMD that way).
#define TBG_ADD_DBL_INLINE 1
#include "tbls_launch.h"
#include "bls_h2c.h"

namespace tbg {

// Cofactor clearing stays one lane per message at one wave per SIMD: its
// live state (three G2 points across the second [x] multiplication) does
// not fit 256 VGPRs even split over a lane pair (measured: 1,271 spilled
// VGPRs for the pair form, tools notes in DESIGN.md).  Splitting it off is
// what lets k_hash_map run at two waves per SIMD.
__global__ void TBG_LAUNCH k_hash_clear(DevBatch B) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B.n_msgs) return;
  B.h_jac[m] = g2_clear_cofactor_t<true>(B.h_jac[m]);
}

void launch_hash_clear(const DevBatch& B, hipStream_t st) {
  if (B.n_msgs) TBG_KLAUNCH(k_hash_clear, grid_for(B.n_msgs), dim3(kBlock), st, B);
}

}  // namespace tbg
