// The level-0 and level-1 Miller products on hexads (bls_hex.h): each Fp12
// spread over six lanes instead of a trio's three, so the kernel fits 256
// VGPRs and runs at two waves per SIMD.  Output in the trio's quad layout
// (chunk_f, batch_f): the level-0 fold / tree / final kernels and the group
// levels read it with trio kernels.  Reference: the pairing products behind tbls.Verify
// (tbls/tss.go:190-197), batched per k_rlc.hip's header.
//
// Products are kept in program order (TBG_SCHED_FENCE): interleaving two
// independent Montgomery products for ILP is what pushes a kernel past 256
// registers, and the second wave per SIMD hides the latency instead.
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1
#endif
#include "tbls_launch.h"
#include "bls_lines.h"
#include "bls_hex.h"

namespace tbg {

#ifndef TBG_HEX_HOIST
#define TBG_HEX_HOIST 1
#endif
constexpr uint32_t HEX_HOIST_MAX = 16;

// One hexad per (group, chunk of rlc_chunk duties), then the S hexads (S
// hexads evaluate one line per step instead of C: in waves of their own they
// finish early instead of each holding a P chunk's wave slot):
//   MILLER_L0       ONE S hexad for level 0's batch-wide S (batch lines, -g1 folded)
//   MILLER_GROUPS   one S hexad per group (group lines); groups without
//                   candidates skipped, a degenerate group S keeps its P chunks
//   MILLER_GROUP_S  after a level-0 failure: the groups' S hexads only (level
//                   0's P-chunk products serve the group checks as they are)
template <int MODE>
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_miller_hex(DevBatch B) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t G = B.rlc_group, C = B.rlc_chunk;
  const uint32_t n_groups = (B.n_duties + G - 1) / G;
  const uint32_t nch = (G + C - 1) / C, nq = nch + 1;
  const uint32_t np_q = MODE == MILLER_GROUP_S ? 0u : n_groups * nch;
  const uint32_t qd = hex_slot(t);
  if (qd == 0xFFFFFFFFu || qd >= np_q + (MODE == MILLER_L0 ? 1u : n_groups)) return;
  if (MODE == MILLER_GROUP_S && B.counters[CNT_L0_OK]) return;  // level 0 accepted the batch
  const bool s_quad = qd >= np_q;
  const uint32_t* ls = nullptr;
  uint32_t* dst;
  uint32_t d0 = 0, d1 = 0;
  if (MODE == MILLER_L0 && s_quad) {
    if (B.counters[CNT_L0_BAD]) return;
    ls = B.batch_lines;
    dst = B.batch_f;
  } else {
    const uint32_t g = s_quad ? qd - np_q : qd / nch, c = s_quad ? nch : qd % nch;
    if (MODE != MILLER_L0) {
      const int32_t gs = B.grp_state[g];
      if (gs == GRP_EMPTY || (gs == GRP_FAIL && s_quad)) return;
    }
    if (s_quad) {
      ls = B.grp_lines + (size_t)LINES_WORDS * g;
    } else {
      d0 = g * G + c * C;
      d1 = min(d0 + C, min(g * G + G, B.n_duties));
    }
    dst = B.chunk_f + (size_t)3 * 4 * NL * (g * nq + c);
  }
  Fp4h f = hex_one();
  int idx = 0;
#if TBG_HEX_HOIST
  // The chunk's duties are decided once, not at every one of the 68 steps:
  // a bit per duty whose line products run (combined, H(m) usable) and its
  // message index in LDS, so a step's line loads do not wait behind the
  // dv_state -> duty_msg -> h_status load chain.  Chunks longer than
  // HEX_HOIST_MAX duties keep the per-step test.
  __shared__ uint32_t s_msg[kBlock * HEX_HOIST_MAX];
  uint32_t* my_msg = s_msg + HEX_HOIST_MAX * threadIdx.x;
  const bool hoist = d1 - d0 <= HEX_HOIST_MAX;
  uint32_t run = 0;
  if (hoist) {
    for (uint32_t d = d0; d < d1; ++d) {
      if (B.dv_state[d] != RLC_COMBINED) continue;
      const uint32_t m = B.duty_msg[d];
      if (B.h_status[m] != 0) continue;  // the check fails in k_l0_fold / k_rlc_group_final
      my_msg[d - d0] = m;
      run |= 1u << (d - d0);
    }
  }
#endif
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = hex_sqr(f);
    const int steps = ((X_ABS >> b) & 1) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < steps; ++s, ++idx) {
      if (s_quad) f = hex_line_folded(f, ls, idx);
#if TBG_HEX_HOIST
      if (hoist) {
#pragma unroll 1
        for (uint32_t bits = run; bits; bits &= bits - 1) {
          const uint32_t j = __builtin_ctz(bits);
          const G1A& P = B.dv_p[d0 + j];
          f = hex_line_at(f, B.h_lines + (size_t)LINES_WORDS * my_msg[j], idx, fp_reduce(fp_neg(P.x)), P.y);
        }
        continue;
      }
#endif
#pragma unroll 1
      for (uint32_t d = d0; d < d1; ++d) {
        if (B.dv_state[d] != RLC_COMBINED) continue;
        const uint32_t m = B.duty_msg[d];
        if (B.h_status[m] != 0) continue;  // the check fails in k_l0_fold / k_rlc_group_final
        const G1A& P = B.dv_p[d];
        f = hex_line_at(f, B.h_lines + (size_t)LINES_WORDS * m, idx, fp_reduce(fp_neg(P.x)), P.y);
      }
    }
  }
  hex_store(dst, f);
}

void launch_l0_miller_hex(const DevBatch& B, hipStream_t st) {
  const uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
  const uint32_t nch = (B.rlc_group + B.rlc_chunk - 1) / B.rlc_chunk;
  TBG_KLAUNCH(k_miller_hex<MILLER_L0>, grid_for(hex_threads(n_groups * nch + 1)), dim3(kBlock), st, B);
}
void launch_groups_miller_hex(const DevBatch& B, hipStream_t st) {
  const uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
  const uint32_t nch = (B.rlc_group + B.rlc_chunk - 1) / B.rlc_chunk;
  TBG_KLAUNCH(k_miller_hex<MILLER_GROUPS>, grid_for(hex_threads(n_groups * (nch + 1))), dim3(kBlock), st, B);
}
void launch_group_s_miller_hex(const DevBatch& B, hipStream_t st) {
  const uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
  TBG_KLAUNCH(k_miller_hex<MILLER_GROUP_S>, grid_for(hex_threads(n_groups)), dim3(kBlock), st, B);
}

}  // namespace tbg
