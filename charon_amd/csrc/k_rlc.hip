// Batched partial-signature verification by random linear combination (RLC)
// with per-item fallback -- the engine's default schedule for the per-partial
// CoreVerify calls of tbls.Verify / tbls.VerifyAndAggregate (reference
// tbls/tss.go:153-197).
//
// Every partial i of duty d signs the duty's message m_d under its own public
// share pk_i:  e(pk_i, H(m_d)) == e(g1, s_i).  With secret 64-bit scalars r_i
// (r = 1 for the first candidate of a duty) drawn after the inputs are fixed,
//
//   level 1, group of G duties:  prod_d e(P_d, H(m_d)) * e(-g1, S) == 1,
//            P_d = sum_i r_i pk_i,  S = sum_d S_d,  S_d = sum_i r_i s_i,
//   level 2, one duty:           e(P_d, H(m_d)) * e(-g1, S_d) == 1,
//   level 3, one partial:        e(pk_i, H(m_d)) * e(-g1, s_i) == 1.
//
// A group that passes accepts all its candidates (a false accept needs the
// scalars to hit a root of a nonzero relation: probability <= 2^-64).  A
// group that fails is split into its duties, a duty that fails into its
// partials, and level 3 is the exact per-item check -- so every partial's
// verdict is the one tbls.Verify would return.  One quad of lanes runs each
// product check (bls_quad.h) over Miller lines stored in HBM: the H(m) lines
// are shared by all partials of a message, the -g1 factor is folded into the
// lines of S / S_d / s_i.  Work lists for levels 2 and 3 are compacted on the
// device (atomic counters), so a clean batch launches them over empty lists.
#include "tbls_launch.h"
#include "bls_h2c.h"
#include "bls_lines.h"
#include "bls_quad.h"

namespace tbg {

// r_i: 64 bits of SHA-256's compression function keyed by the batch seed.
TBG_HD uint64_t rlc_scalar(const uint32_t (&seed)[8], uint32_t i) {
  uint8_t blk[64];
  for (int k = 0; k < 8; ++k) {
    blk[4 * k] = (uint8_t)(seed[k] >> 24);
    blk[4 * k + 1] = (uint8_t)(seed[k] >> 16);
    blk[4 * k + 2] = (uint8_t)(seed[k] >> 8);
    blk[4 * k + 3] = (uint8_t)seed[k];
  }
  for (int k = 32; k < 64; ++k) blk[k] = 0;
  blk[32] = (uint8_t)(i >> 24);
  blk[33] = (uint8_t)(i >> 16);
  blk[34] = (uint8_t)(i >> 8);
  blk[35] = (uint8_t)i;
  blk[36] = 0x80;
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  sha256_block(h, blk);
  uint64_t r = ((uint64_t)h[0] << 32) | h[1];
  return r ? r : 1;
}

// Candidate = decoded fine (status still NOT_VERIFIED) with a usable pubkey.
__device__ __forceinline__ bool rlc_candidate(const DevBatch& B, uint32_t i) {
  return B.partial_status[i] == TBG_PS_NOT_VERIFIED;
}

// ------------------------------------------------------------------ level 0
// One thread per duty: flag unusable pubkeys, then P_d and S_d by a
// shared-doubling (Straus) 64-bit multi-scalar multiplication.
__global__ void __launch_bounds__(64) k_rlc_combine(DevBatch B, const G1A* pk_aff, const int32_t* pk_status, uint32_t n_pk) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= B.n_duties) return;
  uint32_t first = B.duty_first[d], last = B.duty_first[d + 1];
  int cand = 0;
  for (uint32_t i = first; i < last; ++i) {
    if (!rlc_candidate(B, i)) continue;
    uint32_t pid = B.pubkey_ids[i];
    if (pid >= n_pk || pk_status[pid] != DEC_OK) {
      B.partial_status[i] = TBG_PS_ERR_PUBKEY;
      continue;
    }
    ++cand;
  }
  if (cand == 0) {
    B.dv_state[d] = RLC_NONE;
    return;
  }
  // Chunks of up to 8 candidates: the scalars of a chunk stay in registers
  // and its 64 doublings are shared (Straus); chunk sums are added up.
  G1J P = jac_inf<Fp>();
  G2J S = jac_inf<Fp2>();
  bool lead = true;
  uint32_t i = first;
  while (i < last) {
    uint32_t idx[8];
    uint64_t r[8];
    int k = 0;
    for (; i < last && k < 8; ++i) {
      if (!rlc_candidate(B, i)) continue;
      idx[k] = i;
      r[k] = lead ? 1ull : rlc_scalar(B.rlc_seed, i);
      lead = false;
      ++k;
    }
    uint64_t any = 0;
    for (int j = 0; j < k; ++j) any |= r[j];
    G1J Pc = jac_inf<Fp>();
    G2J Sc = jac_inf<Fp2>();
    bool started = false;
    for (int bit = 63 - __builtin_clzll(any | 1); bit >= 0; --bit) {
      if (started) {
        Pc = jac_dbl(Pc);
        Sc = jac_dbl(Sc);
      }
      for (int j = 0; j < k; ++j) {
        if ((r[j] >> bit) & 1) {
          Pc = jac_add_aff(Pc, pk_aff[B.pubkey_ids[idx[j]]]);
          Sc = jac_add_aff(Sc, B.sig_aff[idx[j]]);
          started = true;
        }
      }
    }
    P = jac_add(P, Pc);
    S = jac_add(S, Sc);
  }
  G1A Pa;
  if (!jac_to_aff(P, Pa) || jac_is_inf(S)) {
    B.dv_state[d] = RLC_EACH;  // degenerate combination: check the partials one by one
    return;
  }
  B.dv_p[d] = Pa;
  B.dv_s[d] = S;
  B.dv_state[d] = RLC_COMBINED;
}

// One thread per group: S = sum of the group's S_d, its Miller lines (-g1 folded in).
__global__ void __launch_bounds__(64) k_rlc_group_lines(DevBatch B) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t G = B.rlc_group;
  uint32_t n_groups = (B.n_duties + G - 1) / G;
  if (g >= n_groups) return;
  uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
  G2J S = jac_inf<Fp2>();
  int n = 0;
  for (uint32_t d = d0; d < d1; ++d)
    if (B.dv_state[d] == RLC_COMBINED) {
      S = jac_add(S, B.dv_s[d]);
      ++n;
    }
  G2A Sa;
  if (n == 0) {
    B.grp_state[g] = GRP_EMPTY;
    return;
  }
  if (!jac_to_aff(S, Sa)) {
    B.grp_state[g] = GRP_FAIL;
    return;
  }
  Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));
  g2_lines(Sa, nx, fp_from_const(G1_NEG_Y), B.grp_lines + (size_t)LINES_WORDS * g);
  B.grp_state[g] = GRP_LINES;
}

// f *= line(H(m) lines at step idx) evaluated at affine P = (-x, y).
__device__ __forceinline__ Fp4 quad_line_at(const Fp4& f, const uint32_t* lines, int idx, const Fp& nx, const Fp& y) {
  Line h = line_load(lines + LINE_WORDS * idx);
  return quad_line(f, h.l0, fp2_mul_fp(h.l1, nx), fp2_mul_fp(h.l4, y));
}
__device__ __forceinline__ Fp4 quad_line_folded(const Fp4& f, const uint32_t* lines, int idx) {
  Line a = line_load(lines + LINE_WORDS * idx);
  return quad_line(f, a.l0, a.l1, a.l4);
}

// Level 1: one quad per group.
__global__ void __launch_bounds__(64) k_rlc_check_groups(DevBatch B) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t g = t >> 2;
  uint32_t G = B.rlc_group;
  uint32_t n_groups = (B.n_duties + G - 1) / G;
  if (g >= n_groups) return;
  const bool lead = (t & 3) == 0;
  int32_t gs = B.grp_state[g];
  if (gs != GRP_LINES) return;  // empty groups have nothing to resolve; GRP_FAIL stays failed
  uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
  for (uint32_t d = d0; d < d1; ++d) {
    if (B.dv_state[d] == RLC_COMBINED && B.h_status[B.duty_msg[d]] != 0) {
      if (lead) B.grp_state[g] = GRP_FAIL;  // resolved per duty
      return;
    }
  }
  const uint32_t* ls = B.grp_lines + (size_t)LINES_WORDS * g;
  Fp4 f = quad_one();
  int idx = 0;
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = quad_sqr(f);
    int steps = ((X_ABS >> b) & 1) ? 2 : 1;
    for (int s = 0; s < steps; ++s, ++idx) {
      f = quad_line_folded(f, ls, idx);
      for (uint32_t d = d0; d < d1; ++d) {
        if (B.dv_state[d] != RLC_COMBINED) continue;
        const G1A& P = B.dv_p[d];
        f = quad_line_at(f, B.h_lines + (size_t)LINES_WORDS * B.duty_msg[d], idx, fp_reduce(fp_neg(P.x)), P.y);
      }
    }
  }
  f = quad_final_exp(quad_conj(f));
  bool ok = quad_is_one(f);
  if (lead) B.grp_state[g] = ok ? GRP_OK : GRP_FAIL;
}

__device__ __forceinline__ void rlc_mark(const DevBatch& B, uint32_t d, int32_t st) {
  for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i)
    if (rlc_candidate(B, i)) B.partial_status[i] = st;
}
__device__ __forceinline__ void rlc_push_partials(const DevBatch& B, uint32_t d) {
  for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i)
    if (rlc_candidate(B, i)) B.part_list[atomicAdd(&B.counters[CNT_PARTIALS], 1u)] = i;
}

// After level 1 (one thread per duty): accept, split into level 2, or go to level 3.
__global__ void __launch_bounds__(64) k_rlc_resolve_groups(DevBatch B) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= B.n_duties) return;
  int32_t st = B.dv_state[d];
  if (st == RLC_NONE) return;
  if (st == RLC_EACH) { rlc_push_partials(B, d); return; }
  if (B.h_status[B.duty_msg[d]] != 0) { rlc_mark(B, d, TBG_PS_INVALID); return; }
  int32_t gs = B.grp_state[d / B.rlc_group];
  if (gs == GRP_OK) { rlc_mark(B, d, TBG_PS_VALID); return; }
  if (B.rlc_group > 1) B.dv_list[atomicAdd(&B.counters[CNT_DUTIES], 1u)] = d;
  else rlc_push_partials(B, d);
}

// Level 2 lines: one thread per listed duty.
__global__ void __launch_bounds__(64) k_rlc_duty_lines(DevBatch B) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B.counters[CNT_DUTIES]) return;
  uint32_t d = B.dv_list[k];
  G2A Sa;
  if (!jac_to_aff(B.dv_s[d], Sa)) return;  // excluded in k_rlc_combine
  Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));
  g2_lines(Sa, nx, fp_from_const(G1_NEG_Y), B.dv_lines + (size_t)LINES_WORDS * k);
}

// Level 2 check: one quad per listed duty; failures go to level 3.
__global__ void __launch_bounds__(64) k_rlc_check_duties(DevBatch B) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t k = t >> 2;
  if (k >= B.counters[CNT_DUTIES]) return;
  const bool lead = (t & 3) == 0;
  uint32_t d = B.dv_list[k];
  const G1A& P = B.dv_p[d];
  Fp nx = fp_reduce(fp_neg(P.x));
  const uint32_t* ls = B.dv_lines + (size_t)LINES_WORDS * k;
  const uint32_t* lh = B.h_lines + (size_t)LINES_WORDS * B.duty_msg[d];
  Fp4 f = quad_one();
  int idx = 0;
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = quad_sqr(f);
    int steps = ((X_ABS >> b) & 1) ? 2 : 1;
    for (int s = 0; s < steps; ++s, ++idx) {
      f = quad_line_folded(f, ls, idx);
      f = quad_line_at(f, lh, idx, nx, P.y);
    }
  }
  f = quad_final_exp(quad_conj(f));
  bool ok = quad_is_one(f);
  if (!lead) return;
  if (ok) rlc_mark(B, d, TBG_PS_VALID);
  else rlc_push_partials(B, d);
}

// Per-partial schedule (TBG_VERIFY_EACH): every candidate goes to level 3.
__global__ void __launch_bounds__(64) k_list_all_partials(DevBatch B, const int32_t* pk_status, uint32_t n_pk) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials) return;
  if (!rlc_candidate(B, i)) return;
  uint32_t pid = B.pubkey_ids[i];
  if (pid >= n_pk || pk_status[pid] != DEC_OK) {
    B.partial_status[i] = TBG_PS_ERR_PUBKEY;
    return;
  }
  B.part_list[atomicAdd(&B.counters[CNT_PARTIALS], 1u)] = i;
}

// Level 3 lines: one thread per listed partial, lines of its signature.
__global__ void __launch_bounds__(64) k_lines_sig_list(DevBatch B) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B.counters[CNT_PARTIALS]) return;
  uint32_t i = B.part_list[k];
  Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));
  g2_lines(B.sig_aff[i], nx, fp_from_const(G1_NEG_Y), B.sig_lines + (size_t)LINES_WORDS * k);
}

// Level 3 check: one quad per listed partial, the exact CoreVerify.
__global__ void __launch_bounds__(64) k_verify_list(DevBatch B, const G1A* pk_aff) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t k = t >> 2;
  if (k >= B.counters[CNT_PARTIALS]) return;
  const bool lead = (t & 3) == 0;
  uint32_t i = B.part_list[k];
  uint32_t m = B.duty_msg[B.partial_duty[i]];
  if (B.h_status[m] != 0) {
    if (lead) B.partial_status[i] = TBG_PS_INVALID;
    return;
  }
  G1A pk = pk_aff[B.pubkey_ids[i]];
  Fp nx = fp_reduce(fp_neg(pk.x));
  const uint32_t* ls = B.sig_lines + (size_t)LINES_WORDS * k;
  const uint32_t* lh = B.h_lines + (size_t)LINES_WORDS * m;
  Fp4 f = quad_one();
  int idx = 0;
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = quad_sqr(f);
    int steps = ((X_ABS >> b) & 1) ? 2 : 1;
    for (int s = 0; s < steps; ++s, ++idx) {
      f = quad_line_folded(f, ls, idx);
      f = quad_line_at(f, lh, idx, nx, pk.y);
    }
  }
  f = quad_final_exp(quad_conj(f));
  bool ok = quad_is_one(f);
  if (lead) B.partial_status[i] = ok ? TBG_PS_VALID : TBG_PS_INVALID;
}

void launch_rlc_prepare(const DevBatch& B, const G1A* pk_aff, const int32_t* pk_status, uint32_t n_pk, hipStream_t st) {
  if (!B.n_duties) return;
  if (B.rlc_group == 0) {
    if (B.n_partials) hipLaunchKernelGGL(k_list_all_partials, grid_for(B.n_partials), dim3(kBlock), 0, st, B, pk_status, n_pk);
    return;
  }
  hipLaunchKernelGGL(k_rlc_combine, grid_for(B.n_duties), dim3(kBlock), 0, st, B, pk_aff, pk_status, n_pk);
  uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
  hipLaunchKernelGGL(k_rlc_group_lines, grid_for(n_groups), dim3(kBlock), 0, st, B);
}

void launch_rlc_check(const DevBatch& B, const G1A* pk_aff, hipStream_t st) {
  if (!B.n_duties) return;
  if (B.rlc_group != 0) {
    uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
    hipLaunchKernelGGL(k_rlc_check_groups, grid_for(4 * n_groups), dim3(kBlock), 0, st, B);
    hipLaunchKernelGGL(k_rlc_resolve_groups, grid_for(B.n_duties), dim3(kBlock), 0, st, B);
    if (B.rlc_group > 1) {
      hipLaunchKernelGGL(k_rlc_duty_lines, grid_for(B.n_duties), dim3(kBlock), 0, st, B);
      hipLaunchKernelGGL(k_rlc_check_duties, grid_for(4 * B.n_duties), dim3(kBlock), 0, st, B);
    }
  }
  if (B.n_partials) {
    hipLaunchKernelGGL(k_lines_sig_list, grid_for(B.n_partials), dim3(kBlock), 0, st, B);
    hipLaunchKernelGGL(k_verify_list, grid_for(4 * B.n_partials), dim3(kBlock), 0, st, B, pk_aff);
  }
}

}  // namespace tbg
