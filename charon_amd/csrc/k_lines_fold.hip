// Miller lines of affine G2 points with the -g1 factor folded in (the S side
// of every RLC product check), one lane PAIR per point with the Fp2
// coordinates split over the pair (bls_pair.h, two waves per SIMD).  The
// producers in k_rlc.hip form the sums and their affine points in
// DevBatch::pend_pts (one inversion per lane); a single lane computing the 68
// lines of a point was the latency of the group-lines and fallback-lines
// kernels (157 waves for a 10k-DV batch's 625 groups).
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernel in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_lines.h"
#include "bls_pair.h"

namespace tbg {

template <int KIND>
__device__ __forceinline__ void lines_fold_one(const DevBatch& B, uint32_t k) {
  uint32_t* out;
  if (KIND == FOLD_GROUPS) {
    if (k >= (B.n_duties + B.rlc_group - 1) / B.rlc_group || B.grp_state[k] != GRP_LINES) return;
    out = B.grp_lines;
  } else if (KIND == FOLD_CHUNKS) {
    if (k >= B.counters[CNT_CHUNKS] || !fb_in_pass(B, k) || (B.chunk_list[k] & CHUNK_DEGENERATE)) return;
    out = B.chunk_lines;
  } else if (KIND == FOLD_CID) {
    if (k >= B.counters[CNT_CID] || !fb_in_pass(B, k) || (B.cid_list[k] & ID_DEGENERATE)) return;
    out = B.cid_lines;
  } else if (KIND == FOLD_GID) {
    if (k >= B.counters[CNT_GID] || !fb_in_pass(B, k) || (B.gid_list[k] & ID_DEGENERATE)) return;
    out = B.gid_lines;
  } else {  // FOLD_IDENT
    if (k >= B.counters[CNT_DUTIES] || !fb_in_pass(B, k) || (B.id_list[k] & ID_DEGENERATE)) return;
    out = B.id_lines;
  }
  const Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));
  px_g2_lines(px_load(B.pend_pts[k]), nx, fp_from_const(G1_NEG_Y),
              out + (KIND == FOLD_GROUPS ? (size_t)LINES_WORDS * k : fb_slot(B, k)));
}

template <int KIND>
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_lines_fold(DevBatch B) {
  // both lanes of a pair take the same branches; the fallback kinds run in
  // passes of fb_window list positions from fb_base (launch_rlc_check), a
  // grid smaller than the pass looping over it (fb_pass_loop)
  const uint32_t pr = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (KIND == FOLD_GROUPS) {
    lines_fold_one<KIND>(B, pr);
    return;
  }
  const uint32_t count = KIND == FOLD_CHUNKS ? B.counters[CNT_CHUNKS]
                         : KIND == FOLD_CID  ? B.counters[CNT_CID]
                         : KIND == FOLD_GID  ? B.counters[CNT_GID]
                                             : B.counters[CNT_DUTIES];
  fb_pass_loop(B, pr, (gridDim.x * blockDim.x) >> 1, count, [&](uint32_t k) { lines_fold_one<KIND>(B, k); });
}

void launch_lines_fold(const DevBatch& B, int kind, uint32_t max_entries, hipStream_t st) {
  if (!max_entries) return;
  const dim3 grid = grid_for(2 * max_entries);
  switch (kind) {
    case FOLD_GROUPS: TBG_KLAUNCH(k_lines_fold<FOLD_GROUPS>, grid, dim3(kBlock), st, B); break;
    case FOLD_CHUNKS: TBG_KLAUNCH(k_lines_fold<FOLD_CHUNKS>, grid, dim3(kBlock), st, B); break;
    case FOLD_CID: TBG_KLAUNCH(k_lines_fold<FOLD_CID>, grid, dim3(kBlock), st, B); break;
    case FOLD_GID: TBG_KLAUNCH(k_lines_fold<FOLD_GID>, grid, dim3(kBlock), st, B); break;
    default: TBG_KLAUNCH(k_lines_fold<FOLD_IDENT>, grid, dim3(kBlock), st, B); break;
  }
}

}  // namespace tbg
