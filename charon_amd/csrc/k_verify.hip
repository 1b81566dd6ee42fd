// Miller lines of every H(m) of a batch (G1 factor left out, evaluated per
// public key by the product checks of k_rlc.hip): one lane PAIR per message,
// the Fp2 coordinates split over the pair (bls_pair.h), two waves per SIMD.
// H(m) is shared by all partials of a duty (tbls.Verify, reference
// tbls/tss.go:190-197, recomputes it per call).
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernel in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_lines.h"
#include "bls_pair.h"

namespace tbg {

__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_lines_h(DevBatch B) {
  const uint32_t m = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // both lanes of a pair take the same branches
  if (m >= B.n_msgs) return;
  if (B.h_status[m] != 0) return;
  px_g2_lines<false>(px_load(B.h_aff[m]), fp_one(), fp_one(), B.h_lines + (size_t)LINES_WORDS * m);
}

void launch_h_lines(const DevBatch& B, hipStream_t st) {
  if (B.n_msgs) TBG_KLAUNCH(k_lines_h, grid_for(2 * B.n_msgs), dim3(kBlock), st, B);
}

}  // namespace tbg
