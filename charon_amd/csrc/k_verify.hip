// Miller lines of every H(m) of a batch (G1 factor left out, evaluated per
// public key by the product checks of k_rlc.hip): one thread per message.
// H(m) is shared by all partials of a duty (tbls.Verify, reference
// tbls/tss.go:190-197, recomputes it per call).
#include "tbls_launch.h"
#include "bls_lines.h"
#include "bls_quad.h"

namespace tbg {

__global__ void TBG_LAUNCH k_lines_h(DevBatch B) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= B.n_msgs) return;
  if (B.h_status[m] != 0) return;
  g2_lines_t<true>(B.h_aff[m], fp_one(), fp_one(), B.h_lines + (size_t)LINES_WORDS * m);
}

void launch_h_lines(const DevBatch& B, hipStream_t st) {
  if (B.n_msgs) TBG_KLAUNCH(k_lines_h, grid_for(B.n_msgs), dim3(kBlock), st, B);
}

}  // namespace tbg
