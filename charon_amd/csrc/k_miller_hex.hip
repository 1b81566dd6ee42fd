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

// H(m) lines staged through LDS one line-step ahead (the
// row-N2 A/B): while a hexad multiplies f by the line of step t, the LDS-DMA
// (global_load_lds, no VGPR destination) of step t + 1's line is in flight
// into the other of two buffers, so the line loads no longer stall the wave.
// Each lane stages ONE Fp of its hexad's next line (component 2q + c of
// (l0, l1, l4)) as 14 lane-linear dwords; the hexad then reads the pieces it
// needs from its neighbours' slots.  The buffers are two distinct __shared__
// objects and the step loop is unrolled by two, so the compiler's alias-aware
// LDS-DMA waits retire only the buffer being read (vmcnt(14), not 0).
#ifndef TBG_HEX_PREFETCH
#define TBG_HEX_PREFETCH 0
#endif

#if TBG_HEX_PREFETCH
// whether a squaring of f precedes line idx (the first line of every bit but the top one)
struct HexSqrMask { uint64_t lo, hi; };
constexpr HexSqrMask hex_sqr_mask() {
  HexSqrMask m{0, 0};
  int idx = 0;
  for (int b = 62; b >= 0; --b) {
    if (b != 62) {
      if (idx < 64) m.lo |= 1ull << idx;
      else m.hi |= 1ull << (idx - 64);
    }
    idx += ((X_ABS >> b) & 1) ? 2 : 1;
  }
  return m;
}
constexpr HexSqrMask kHexSqr = hex_sqr_mask();
static_assert(N_LINES <= 128, "line mask");

constexpr uint32_t HEX_PF_WORDS = 64 * NL;  // one buffer: limb i of lane L at [64 i + L]
__shared__ uint32_t s_pf_a[HEX_PF_WORDS];
__shared__ uint32_t s_pf_b[HEX_PF_WORDS];

// stage component (2q + c) of line idx of message m into buf (every lane of
// the hexad); `after` only orders the issue after the value it depends on
// (its operand loads' wait then retires before this DMA is in flight)
template <int BUF>
TBG_DEV void hex_pf_issue(const uint32_t* h_lines, uint32_t m, int idx, uint32_t after = 0) {
  uint32_t* buf = BUF ? s_pf_b : s_pf_a;
  const uint32_t k = 2u * (uint32_t)quad_lane() + hex_c();
  uint32_t z = 0;
  asm volatile("" : "+v"(z) : "v"(after));  // z stays 0
  const uint32_t* src = h_lines + (size_t)LINES_WORDS * m + LINE_WORDS * idx + k * NL + z;
#pragma unroll
  for (int i = 0; i < NL; ++i)
    __builtin_amdgcn_global_load_lds((const void*)(src + i), (__attribute__((address_space(3))) void*)(buf + 64 * i), 4,
                                     0, 0);
}
// the Fp that lane L staged in buf
template <int BUF>
TBG_DEV Fp hex_pf_read(uint32_t L) {
  const uint32_t* buf = BUF ? s_pf_b : s_pf_a;
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = buf[64 * i + L];
  return r;
}

// One line step of the staged schedule: f *= line(idx) of message m at
// P = dv_p[d]; the next step's line (nm, nidx) is issued into the other
// buffer once this step's evaluation has its operands (the last step
// re-stages a line: no branch around the issue).
template <int BUF>
TBG_DEV Fp4h hex_pf_step(const Fp4h& A, const DevBatch& B, uint32_t d, uint32_t nm, int nidx) {
  const uint32_t c = hex_c();
  const int q = quad_lane();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t base = (lane & ~16u) - (uint32_t)q;  // lane (0, 0) of this hexad
  // this lane's G1 operand: -x_P on q = 0, y_P on q = 1 (q = 2: unused)
  const Fp nv = hex_line_operand(B.dv_p[d]);
  // lk = l1_c (q = 0) or l4_c (q = 1, 2), staged by lane (1, c) / (2, c)
  const Fp lk = hex_pf_read<BUF>(base + (q == 0 ? 1u : 2u) + (c << 4));
  const Fp e = fp_mul(lk, nv);
  hex_pf_issue<BUF ^ 1>(B.h_lines, nm, nidx < 0 ? N_LINES - 1 : nidx, e.l[0]);
  const Fp e1 = xch<QP_B0>(e), e4 = xch<QP_B1>(e);
  HxLine r;
  {
    const Fp4h An = hxch<QP_NEXT>(A);
    hx_line_u(c, hx_own_par(An, hx_swap(An)), Fp2o{e1, hx_swap(e1)}, r);
  }
  // l0 = (l0_c, l0_(1-c)), staged by lanes (0, c) and (0, 1 - c)
  const Fp2o l0{hex_pf_read<BUF>(base + (c << 4)), hex_pf_read<BUF>(base + ((c ^ 1u) << 4))};
  hx_line_t(c, q, hx_own_par(A, hx_swap(A)), l0, Fp2o{e4, hx_swap(e4)}, r);
  return hx_line2(c, q, r, hx_swap(r.W));
}

// The chunk's Miller product over its hoisted duties (run bits, messages in
// my_msg) with the lines staged through LDS.  Line steps t = 0 .. 68 n - 1
// run duty by duty within each line index; the loop is unrolled by two so
// each half reads a fixed buffer.
TBG_DEV Fp4h hex_chunk_staged(const DevBatch& B, uint32_t d0, uint32_t run, const uint32_t* my_msg) {
  Fp4h f = hex_one();
  if (!run) return f;
  uint32_t bits = run;  // duties of the current line index still to go
  int idx = 0;
  uint32_t j = __builtin_ctz(bits);
  hex_pf_issue<0>(B.h_lines, my_msg[j], 0);
  // the step after (j, idx): next duty of this index, else the first of the next
  auto advance = [&](uint32_t& nj, int& nidx) {
    const uint32_t rest = bits & (bits - 1);
    if (rest) {
      nj = __builtin_ctz(rest);
      nidx = idx;
    } else {
      nj = __builtin_ctz(run);
      nidx = idx + 1 < N_LINES ? idx + 1 : -1;
    }
  };
  auto sqr_before = [](int i) {
    return i < 64 ? ((kHexSqr.lo >> i) & 1u) != 0 : ((kHexSqr.hi >> (i - 64)) & 1u) != 0;
  };
#pragma unroll 1
  for (;;) {
    uint32_t nj;
    int nidx;
    // even step: buffer A
    if (bits == run && sqr_before(idx)) f = hex_sqr(f);
    advance(nj, nidx);
    f = hex_pf_step<0>(f, B, d0 + j, my_msg[nj], nidx);
    if (nidx < 0) break;
    bits = bits & (bits - 1);
    if (!bits) bits = run;
    idx = nidx;
    j = nj;
    // odd step: buffer B (68 n steps: always even in number)
    if (bits == run && sqr_before(idx)) f = hex_sqr(f);
    advance(nj, nidx);
    f = hex_pf_step<1>(f, B, d0 + j, my_msg[nj], nidx);
    if (nidx < 0) break;
    bits = bits & (bits - 1);
    if (!bits) bits = run;
    idx = nidx;
    j = nj;
  }
  // the last (unused) DMA lands before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return f;
}
#endif

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
#if TBG_HEX_PREFETCH
  if (hoist && !s_quad) {
    hex_store(dst, hex_chunk_staged(B, d0, run, my_msg));
    return;
  }
#endif
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
          f = hex_line_at_v(f, B.h_lines + (size_t)LINES_WORDS * my_msg[j], idx, hex_line_operand(B.dv_p[d0 + j]));
        }
        continue;
      }
#endif
#pragma unroll 1
      for (uint32_t d = d0; d < d1; ++d) {
        if (B.dv_state[d] != RLC_COMBINED) continue;
        const uint32_t m = B.duty_msg[d];
        if (B.h_status[m] != 0) continue;  // the check fails in k_l0_fold / k_rlc_group_final
        f = hex_line_at_v(f, B.h_lines + (size_t)LINES_WORDS * m, idx, hex_line_operand(B.dv_p[d]));
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
