// Batched partial-signature verification by random linear combination (RLC)
// with per-item fallback -- the engine's default schedule for the per-partial
// CoreVerify calls of tbls.Verify / tbls.VerifyAndAggregate (reference
// tbls/tss.go:153-197).
//
// Every partial i of duty d signs the duty's message m_d under its own public
// share pk_i:  e(pk_i, H(m_d)) == e(g1, s_i).  With secret 64-bit scalars r_i
// (r = 1 for the first candidate of a level-1 group) drawn after the inputs are fixed,
//
//   level 1,   group of G duties:  prod_d e(P_d, H(m_d)) * e(-g1, S) == 1,
//              P_d = sum_i r_i pk_i,  S = sum_d S_d,  S_d = sum_i r_i s_i,
//              run as C-duty chunks of P pairs + the S pair, one quad each;
//   level 1.5, a failed group's chunk c: the stored P-chunk product * e(-g1, S_c);
//   level 1.5b, a failed chunk: the exponent test finds its one bad duty;
//   level 2b,  a bad duty: the exponent test finds its one bad partial;
//   level 3,   one partial:        e(pk_i, H(m_d)) * e(-g1, s_i) == 1.
//
// A group that passes accepts all its candidates (a false accept needs the
// scalars to hit a root of a nonzero relation: probability <= 2^-64).  A
// failed group is narrowed to its failed chunks, a failed chunk to its bad
// duty, a bad duty to its bad partial; whatever the exponent tests cannot
// pin down (two or more bad members) goes to level 3, the exact per-item
// check -- so every partial's verdict is the one tbls.Verify would return.
// One lane group (a hexad: six lanes, bls_hex.h) runs each product check --
// its Miller loop, final exponentiation and exponent test -- over Miller lines
// stored in HBM: the H(m) lines are shared by all partials of a message, the
// -g1 factor is folded into the lines of S / S_c / s_i.  Work lists of the
// fallback levels are compacted on the device (atomic counters), so a clean
// batch launches them over empty lists.
// The P == Q case of the mixed addition doubles inline (bls_curve.h): no
// out-of-line call inside the kernels' point loops.
#define TBG_ADD_DBL_INLINE 1
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order (bls_field.h): keeps the tower inverse inside the hexad kernels' budget
#endif
#include "tbls_launch.h"
#include "bls_h2c.h"
#include "bls_lines.h"
#include "bls_hex.h"
#include "bls_rlc.h"
#include "bls_batchinv.h"
#include "bls_row.h"

namespace tbg {

// Candidate = decoded fine with a usable public key.  k_rlc_partial turns
// non-candidates' NOT_VERIFIED into ERR_PUBKEY concurrently, so the test reads
// the key table rather than trusting that transition to have happened.
__device__ __forceinline__ bool rlc_usable(const DevBatch& B, uint32_t i, const int32_t* pk_status, uint32_t n_pk) {
  int32_t st = B.partial_status[i];
  if (st != TBG_PS_NOT_VERIFIED && st != TBG_PS_ERR_PUBKEY) return false;
  uint32_t pid = B.pubkey_ids[i];
  return pid < n_pk && pk_status[pid] == DEC_OK;
}
__device__ __forceinline__ bool rlc_candidate(const DevBatch& B, uint32_t i) {
  return B.partial_status[i] == TBG_PS_NOT_VERIFIED;
}

// A duty that level 1.5 / 2 may combine: COMBINED and its H(m) usable.
__device__ __forceinline__ bool rlc_combinable(const DevBatch& B, uint32_t d) {
  return B.dv_state[d] == RLC_COMBINED && B.h_status[B.duty_msg[d]] == 0;
}
__device__ __forceinline__ uint32_t rlc_candidates(const DevBatch& B, uint32_t d) {
  uint32_t n = 0;
  for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i) n += rlc_candidate(B, i) ? 1u : 0u;
  return n;
}

// ------------------------------------------------------------------ level 0
// [r_i] s_i and [r_i] pk_i: k_rlc_g2_pair / k_rlc_g1 (k_pair.hip).

// One thread per duty: P_d = sum r_i pk_i (affine) and S_d = sum r_i s_i.
// Level 0 (DSUM_L0_P) forms P_d only -- its S is the batch-wide MSM -- and a
// duty it cannot combine (P_d = 0) makes level 0 fail; after a level-0
// failure DSUM_FALLBACK_S adds the S_d of the duties level 0 combined (the
// stored P-chunk products include them; S_d = 0 is just a term of the sums).
// P_d's affine conversion is batched over the workgroup (bls_batchinv.h).
template <int PHASE>
__global__ void __launch_bounds__(BINV_BLOCK) k_rlc_duty_sum(DevBatch B) {
  constexpr int phase = PHASE;
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = d < B.n_duties;
  if (phase == DSUM_FALLBACK_S) {  // (no inversion: no workgroup-wide step)
    if (!in || B.counters[CNT_L0_OK] || B.dv_state[d] != RLC_COMBINED) return;
#if TBG_GMSM
    // after the group checks: the failed groups' duties (their r_i s_i were formed)
    const int32_t gs = B.grp_state[d / B.rlc_group];
    if (gs != GRP_FAIL && gs != GRP_GID) return;
#endif
    G2J S = jac_inf<Fp2>();
    for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i)
      if (rlc_candidate(B, i)) S = jac_add(S, B.part_s[i]);
    B.dv_s[d] = S;
    return;
  }
  G1J P = jac_inf<Fp>();
  G2J S = jac_inf<Fp2>();
  int cand = 0;
  if (in) {
    for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i) {
      if (!rlc_candidate(B, i)) continue;
      // (G1 sums inline: the out-of-line form passes 3 x 2 Fp through scratch per addition)
      P = jac_add_in<Fp, true>(P, B.part_p[i]);
      if (phase == DSUM_BOTH) S = jac_add(S, B.part_s[i]);
      ++cand;
    }
  }
  G1A Pa;
  const bool aff = block_jac_to_aff<BINV_WAVES>(P, cand > 0, Pa);  // every thread of the workgroup
  if (!in) return;
  if (cand == 0) {
    B.dv_state[d] = RLC_NONE;
    return;
  }
  if (!aff || (phase == DSUM_BOTH && jac_is_inf(S))) {
    B.dv_state[d] = RLC_EACH;  // degenerate combination: check the partials one by one
    if (phase == DSUM_L0_P) B.counters[CNT_L0_BAD] = 1;  // (DSUM_P: the group levels only)
    return;
  }
  B.dv_p[d] = G1A{fp_reduce(fp_neg(Pa.x)), Pa.y};  // (-x, y): the Miller steps' evaluation operands
  if (phase == DSUM_BOTH) B.dv_s[d] = S;
  B.dv_state[d] = RLC_COMBINED;
}
inline dim3 duty_grid(const DevBatch& B) { return dim3((B.n_duties + BINV_BLOCK - 1) / BINV_BLOCK); }

// One thread per group: S = sum of the group's S_d, affine (its Miller lines,
// -g1 folded in: k_lines_fold.hip).
__global__ void TBG_LAUNCH k_rlc_group_lines(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;  // level 0 accepted the batch (k_l0_after set the groups)
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
  B.pend_pts[g] = Sa;  // lines: k_lines_fold<FOLD_GROUPS>
  B.grp_state[g] = GRP_LINES;
}

// Fp12 values in HBM in the quad layout: trio lane q's Fp4 at 4 NL words
// per lane (hex_load / hex_store, bls_hex.h).
constexpr int QUAD_WORDS = 4 * NL;

// Level 1, Miller part: one hexad per (group, chunk of rlc_chunk duties),
// plus one per group for the group's S pair alone (k_miller_hex.hip).
// Chunks share nothing but the final exponentiation, so a group's pairs are
// spread over several hexads -- and because the P pairs of a chunk are kept
// apart from S, a failed group can re-check its chunks (level 1.5) from these
// same products with only S_c's Miller loop added.

// Level 1, final part: one hexad per group multiplies its chunks' products
// (the S chunk included) and runs the one final exponentiation of the group.
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_rlc_group_final(DevBatch B) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t G = B.rlc_group, C = B.rlc_chunk;
  uint32_t n_groups = (B.n_duties + G - 1) / G;
  uint32_t nq = (G + C - 1) / C + 1;
  uint32_t g = hex_slot(t);
  if (g >= n_groups) return;
  const bool lead = hex_lead();
  if (B.grp_state[g] != GRP_LINES) return;  // empty groups have nothing to resolve; GRP_FAIL stays failed
  uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
  for (uint32_t d = d0; d < d1; ++d) {
    if (B.dv_state[d] == RLC_COMBINED && B.h_status[B.duty_msg[d]] != 0) {
      if (lead) B.grp_state[g] = GRP_FAIL;  // resolved per chunk / duty
      return;
    }
  }
  const uint32_t* base = B.chunk_f + (size_t)3 * QUAD_WORDS * nq * g;
  Fp4h f = hex_load(base);
  for (uint32_t c = 1; c < nq; ++c) f = hex_mul_ni(f, hex_load(base + (size_t)3 * QUAD_WORDS * c));
  f = hex_final_exp_in(hex_conj(f));
  bool ok = hex_is_one(f);
  if (!ok && B.gident) {
    // level 1g: the group's value A_g, and the group in the list (hexad-uniform)
    uint32_t m = 0;
    for (uint32_t d = d0; d < d1; ++d)
      if (rlc_combinable(B, d)) m += rlc_candidates(B, d);
    if (m >= 2) {
      uint32_t slot = 0;
      if (lead) slot = atomicAdd(&B.counters[CNT_GID], 1u);
      slot = (uint32_t)__shfl((int)slot, (int)hex_lead_lane());
      hex_store(B.grp_fe + (size_t)3 * QUAD_WORDS * slot, f);
      if (lead) {
        B.gid_list[slot] = g;
        B.grp_state[g] = GRP_GID;
      }
      return;
    }
  }
  if (lead) B.grp_state[g] = ok ? GRP_OK : GRP_FAIL;
}

// ------------------------------------------------------------------ level 0
// One hexad per group: the product of its P-chunk values (k_miller_hex,
// MILLER_L0); a combined duty whose H(m) is unusable makes level 0 fail.
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_l0_fold(DevBatch B) {
  TBG_URGENT();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t G = B.rlc_group, C = B.rlc_chunk;
  const uint32_t n_groups = (B.n_duties + G - 1) / G, nch = (G + C - 1) / C, nq = nch + 1;
  const uint32_t g = hex_slot(t);
  if (g >= n_groups || B.counters[CNT_L0_BAD]) return;
  const uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
  for (uint32_t d = d0; d < d1; ++d) {
    if (B.dv_state[d] == RLC_COMBINED && B.h_status[B.duty_msg[d]] != 0) {
      if (hex_lead()) B.counters[CNT_L0_BAD] = 1;
      return;
    }
  }
  const uint32_t* base = B.chunk_f + (size_t)3 * QUAD_WORDS * nq * g;
  Fp4h f = hex_load(base);
  for (uint32_t c = 1; c < nch; ++c) f = hex_mul(f, hex_load(base + (size_t)3 * QUAD_WORDS * c));
  hex_store(B.grp_f + (size_t)3 * QUAD_WORDS * g, f);
}

// Product tree, one hexad per L0_TREE_FAN values of grp_f[in .. in + n).
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_l0_tree(DevBatch B, uint32_t in, uint32_t n, uint32_t out) {
  TBG_URGENT();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t q = hex_slot(t);
  if (q == 0xFFFFFFFFu || q * L0_TREE_FAN >= n || B.counters[CNT_L0_BAD]) return;
  const uint32_t a0 = q * L0_TREE_FAN, a1 = min(a0 + L0_TREE_FAN, n);
  Fp4h f = hex_load(B.grp_f + (size_t)3 * QUAD_WORDS * (in + a0));
  for (uint32_t a = a0 + 1; a < a1; ++a) f = hex_mul(f, hex_load(B.grp_f + (size_t)3 * QUAD_WORDS * (in + a)));
  hex_store(B.grp_f + (size_t)3 * QUAD_WORDS * (out + q), f);
}

// The last <= L0_TREE_FAN values times the S pair's product, one final
// exponentiation for the whole batch -- the latency tail of every level-0
// launch -- on ROWS (bls_row.h: one Fp per 16-lane row, each Montgomery
// product limb-parallel over its row): k_l0_final forms f, k_l0_inv inverts
// it on one lane (the tower inverse; its out-of-line calls would pin the row
// kernel's 576 threads to their register budget), k_l0_fe exponentiates.
// 1.1 ms per launch against 3.3 ms on a hexad (bls_hex.h) or spread over one
// wave with one Fp product per lane (round 3; profiles/r04/rowfe/).
constexpr uint32_t L0_FINAL_THREADS = 16 * 36;  // 36 rows: a product step's Fp products
// f and f^-1 between the three kernels: two spare grp_f entries (12 x 14
// signed limbs each, the row words; grp_f_entries keeps 40 spare)
__device__ __forceinline__ int32_t* l0_f_spare(const DevBatch& B, int k) {
  const uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
  return (int32_t*)(B.grp_f + (size_t)3 * QUAD_WORDS * (grp_f_entries(n_groups) - 1 - k));
}
__global__ void __launch_bounds__(L0_FINAL_THREADS) k_l0_final(DevBatch B, uint32_t in, uint32_t n) {
  TBG_URGENT();
  if (B.counters[CNT_L0_BAD]) return;  // (workgroup-uniform)
  __shared__ RowSlots S;
  RowDevExec ex;
  const int r = threadIdx.x >> 4, j = threadIdx.x & 15;
  auto load = [&](int slot, const uint32_t* src) {
    if (r < RW_FP) row_st(S.v[slot][r], row_from_limbs(src + r * NL));
  };
  ex([&](int) { load(0, B.batch_f); });
  for (uint32_t a = 0; a < n; ++a) {
    ex([&](int) { load(1, B.grp_f + (size_t)3 * QUAD_WORDS * (in + a)); });
    row_mul_to(ex, S, 0, 0, 1);
  }
  if (r < RW_FP && j < NL) l0_f_spare(B, 0)[r * NL + j] = S.v[0][r][j];
}
__global__ void __launch_bounds__(64) k_l0_inv(DevBatch B) {
  TBG_URGENT();
  if (B.counters[CNT_L0_BAD] || threadIdx.x != 0) return;
  const int32_t* f = l0_f_spare(B, 0);
  Fp4 A[3];
  for (int q = 0; q < 3; ++q) {
    A[q].a.c0 = fp_from_signed(f + (4 * q) * NL);
    A[q].a.c1 = fp_from_signed(f + (4 * q + 1) * NL);
    A[q].b.c0 = fp_from_signed(f + (4 * q + 2) * NL);
    A[q].b.c1 = fp_from_signed(f + (4 * q + 3) * NL);
  }
  const Fp12 v = fp12_inv(quad_to_fp12(A[0], A[1], A[2]));
  int32_t* out = l0_f_spare(B, 1);
  for (int q = 0; q < 3; ++q) {
    const Fp4 c = quad_from_fp12(q, v);
    const Fp* w[4] = {&c.a.c0, &c.a.c1, &c.b.c0, &c.b.c1};
    for (int k = 0; k < 4; ++k)
      for (int i = 0; i < NL; ++i) out[(4 * q + k) * NL + i] = (int32_t)w[k]->l[i];
  }
}
__global__ void __launch_bounds__(L0_FINAL_THREADS) k_l0_fe(DevBatch B) {
  TBG_URGENT();
  if (B.counters[CNT_L0_BAD]) return;
  __shared__ RowSlots S;
  RowDevExec ex;
  const int r = threadIdx.x >> 4;
  ex([&](int) {
    if (r < RW_FP) {
      row_st(S.v[0][r], row_from_limbs((const uint32_t*)l0_f_spare(B, 0) + r * NL));
      row_st(S.v[5][r], row_from_limbs((const uint32_t*)l0_f_spare(B, 1) + r * NL));
    }
  });
  row_final_exp_inv(ex, S);
  if (threadIdx.x == 0 && row_is_one(S.v[0])) B.counters[CNT_L0_OK] = 1;
}
// Level 0's S lines (-g1 folded in) on rows: 12 rows, the six conversions of
// each finished line to HBM on row 8's first lanes (idle in the first phase
// of the next step).  On one lane pair (k_lines_fold) this was 1.4 ms of the
// launch's serial path.
constexpr uint32_t L0_LINES_THREADS = 16 * 12;
__global__ void __launch_bounds__(L0_LINES_THREADS) k_l0_lines(DevBatch B) {
  TBG_URGENT();
  if (B.counters[CNT_L0_BAD]) return;  // (workgroup-uniform)
  __shared__ RowLineSlots S;
  RowDevExec ex;
  const int r = threadIdx.x >> 4;
  ex([&](int) {
    const G2A& Q = *B.batch_pt;
    const Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X))), y = fp_from_const(G1_NEG_Y);
    const Fp* c[12] = {&Q.x.c0, &Q.x.c1, &Q.y.c0, &Q.y.c1, nullptr, nullptr, &Q.x.c0, &Q.x.c1, &Q.y.c0, &Q.y.c1, &nx, &y};
    const Fp one = fp_one(), zero = fp_zero();
    const Fp* v = r == 4 ? &one : (r == 5 ? &zero : c[r]);
    row_st(r < 10 ? S.s[r] : S.k[r - 10], row_from_limbs(v->l));
  });
  auto out6 = [&](int buf, int idx) {
    const int t = (int)threadIdx.x - 128;
    if (t >= 0 && t < 6) rl_line_out(S, buf, t, B.batch_lines + (size_t)LINE_WORDS * idx);
  };
  row_g2_lines(ex, out6, S);
}
void launch_l0_lines(const DevBatch& B, hipStream_t st) {
  TBG_KLAUNCH(k_l0_lines, dim3(1), dim3(L0_LINES_THREADS), st, B);
}

static void launch_l0_final(const DevBatch& B, uint32_t in, uint32_t n, hipStream_t st) {
  TBG_KLAUNCH(k_l0_final, dim3(1), dim3(L0_FINAL_THREADS), st, B, in, n);
  TBG_KLAUNCH(k_l0_inv, dim3(1), dim3(64), st, B);
  TBG_KLAUNCH(k_l0_fe, dim3(1), dim3(L0_FINAL_THREADS), st, B);
}

// One thread per group: after a level-0 pass every group with a combined
// duty is accepted (k_rlc_resolve_groups marks its candidates valid).
__global__ void TBG_LAUNCH k_l0_after(DevBatch B) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t G = B.rlc_group;
  if (g >= (B.n_duties + G - 1) / G || !B.counters[CNT_L0_OK]) return;
  const uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
  bool any = false;
  for (uint32_t d = d0; d < d1; ++d) any |= B.dv_state[d] == RLC_COMBINED;
  B.grp_state[g] = any ? GRP_OK : GRP_EMPTY;
}

__device__ __forceinline__ void rlc_mark(const DevBatch& B, uint32_t d, int32_t st) {
  for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i)
    if (rlc_candidate(B, i)) B.partial_status[i] = st;
}
__device__ __forceinline__ void rlc_push_partials(const DevBatch& B, uint32_t d) {
  for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i)
    if (rlc_candidate(B, i)) B.part_list[atomicAdd(&B.counters[CNT_PARTIALS], 1u)] = i;
}


// After level 1 (one thread per duty): accept, split into level 1.5 (the
// failed group's chunks), or go to level 3.
__global__ void TBG_LAUNCH k_rlc_resolve_groups(DevBatch B) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= B.n_duties) return;
  int32_t st = B.dv_state[d];
  if (st == RLC_NONE) return;
  if (st == RLC_EACH) { rlc_push_partials(B, d); return; }
  if (B.h_status[B.duty_msg[d]] != 0) { rlc_mark(B, d, TBG_PS_INVALID); return; }
  const uint32_t G = B.rlc_group, C = B.rlc_chunk;
  const uint32_t g = d / G;
  int32_t gs = B.grp_state[g];
  if (gs == GRP_OK) { rlc_mark(B, d, TBG_PS_VALID); return; }
  if (gs == GRP_GID) return;  // level 1g resolves it (or hands its chunks to level 1.5)
  if (G == 1) { rlc_push_partials(B, d); return; }
  // the chunk goes to level 1.5 once: pushed by its first combinable duty
  const uint32_t c = (d - g * G) / C, dc0 = g * G + c * C;
  for (uint32_t e = dc0; e < d; ++e)
    if (rlc_combinable(B, e)) return;
  const uint32_t nch = (G + C - 1) / C;
  B.chunk_list[atomicAdd(&B.counters[CNT_CHUNKS], 1u)] = g * nch + c;
}

// Level 1.5 lines: one thread per listed chunk: S_c = sum of its combinable
// duties' S_d, Miller lines with -g1 folded in.  A degenerate S_c (point at
// infinity) flags the list entry: its candidates go straight to level 3.
__global__ void TBG_LAUNCH k_rlc_chunk_lines(DevBatch B) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B.counters[CNT_CHUNKS]) return;
  const uint32_t G = B.rlc_group, C = B.rlc_chunk, nch = (G + C - 1) / C;
  const uint32_t qc = B.chunk_list[k], g = qc / nch, c = qc % nch;
  const uint32_t d0 = g * G + c * C, d1 = min(min(d0 + C, g * G + G), B.n_duties);
  G2J S = jac_inf<Fp2>();
  for (uint32_t d = d0; d < d1; ++d)
    if (rlc_combinable(B, d)) S = jac_add(S, B.dv_s[d]);
  G2A Sa;
  if (!jac_to_aff(S, Sa)) {
    B.chunk_list[k] = qc | CHUNK_DEGENERATE;
    return;
  }
  B.pend_pts[k] = Sa;  // lines: k_lines_fold<FOLD_CHUNKS>
}


// The fallback checks' Miller loops: f *= the step's folded lines (S-side,
// -g1 folded in) and the H(m) lines at each listed point; squarings and line
// products inline in the kernel loop (no scratch-stack call per step).
template <class F>
__device__ __forceinline__ Fp4h hex_miller(F&& step) {
  Fp4h f = hex_one();
  int idx = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; --b) {
    if (b != 62) f = hex_sqr(f);
    const int steps = ((X_ABS >> b) & 1) ? 2 : 1;
#pragma unroll 1
    for (int s = 0; s < steps; ++s, ++idx) f = step(f, idx);
  }
  return f;
}

// The exponent test's search: the w in 1..n with A^w == A' (inv_a2 = A'^-1),
// 0 if none (hexad-uniform: hex_is_one agrees on all six lanes).
__device__ __forceinline__ uint32_t hex_find_power(const Fp4h& A, const Fp4h& inv_a2, uint32_t n) {
  Fp4h Aw = A;
#pragma unroll 1
  for (uint32_t w = 1; w <= n; ++w) {
    if (hex_is_one(hex_mul_ni(Aw, inv_a2))) return w;
    Aw = hex_mul_ni(Aw, A);
  }
  return 0;
}

// ---------------------------------------------------------- identification
// The exponent test (Lee, Cheon and Hong, "Finding invalid signatures in
// pairing-based batches") finds the one bad member of a failed product with
// ONE more check instead of one per member.  For members j with values
// eps_j (1 iff member j is valid) and weights w_j = 1..m,
//   A  = prod_j eps_j^(r_j)        (the failed check's final-exponentiated value),
//   A' = prod_j eps_j^(w_j r_j)    (the same check with every member scaled by w_j).
// If exactly member b is bad, A' = A^(w_b): b is found and the others are
// valid.  A match for some w with two or more bad members needs the secret
// r_j to satisfy a fixed nonzero linear relation (probability m 2^-64, the
// RLC bound); no match falls through to the next level.
//   level 1.5b, a failed chunk (members = duties, eps = the duty's RLC product);
//   level 2b, a failed duty (members = partials, eps = the partial's pairing check).
// A duty found at level 1.5b goes straight to 2b with A = the chunk's value
// (the only bad member's product IS the chunk's).

// A failed duty with several candidates goes to level 2b with its A (every
// lane of the hexad stores its part; the lead takes the list slot).
__device__ __forceinline__ void push_ident(const DevBatch& B, uint32_t d, const Fp4h& A, bool lead) {
  uint32_t slot = 0;
  if (lead) {
    slot = atomicAdd(&B.counters[CNT_DUTIES], 1u);
    B.id_list[slot] = d;
  }
  slot = (uint32_t)__shfl((int)slot, (int)hex_lead_lane());
  hex_store(B.id_fe + (size_t)3 * QUAD_WORDS * slot, A);
}
// A duty known to be bad: one candidate -> that partial is invalid (the check
// was its own, scaled by r != 0); several -> level 2b.
__device__ __forceinline__ void resolve_bad_duty(const DevBatch& B, uint32_t d, const Fp4h& A, bool lead) {
  if (rlc_candidates(B, d) > 1) push_ident(B, d, A, lead);
  else if (lead) rlc_mark(B, d, TBG_PS_INVALID);
}

// Level 1.5 check: one hexad per listed chunk: its stored P-pair product
// times the Miller loop of S_c, one final exponentiation.  Pass -> the
// chunk's duties are valid; fail -> a lone duty is resolved at once, several
// go to level 1.5b with the chunk's value (a degenerate S_c: level 3).
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_rlc_check_chunks(DevBatch B) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t k = hex_slot(t) + B.fb_base;
  if (hex_slot(t) == 0xFFFFFFFFu || k >= B.counters[CNT_CHUNKS] || !fb_in_pass(B, k)) return;
  const bool lead = hex_lead();
  const uint32_t G = B.rlc_group, C = B.rlc_chunk, nch = (G + C - 1) / C, nq = nch + 1;
  const uint32_t entry = B.chunk_list[k], qc = entry & ~CHUNK_DEGENERATE, g = qc / nch, c = qc % nch;
  const uint32_t d0 = g * G + c * C, d1 = min(min(d0 + C, g * G + G), B.n_duties);
  if (entry & CHUNK_DEGENERATE) {
    if (lead)
      for (uint32_t d = d0; d < d1; ++d)
        if (rlc_combinable(B, d)) rlc_push_partials(B, d);
    return;
  }
  const uint32_t* ls = B.chunk_lines + fb_slot(B, k);
  Fp4h f = hex_miller([&](const Fp4h& x, int idx) { return hex_line_folded(x, ls, idx); });
  f = hex_mul_ni(f, hex_load(B.chunk_f + (size_t)3 * QUAD_WORDS * (g * nq + c)));
  f = hex_final_exp_in(hex_conj(f));
  if (hex_is_one(f)) {
    if (lead)
      for (uint32_t d = d0; d < d1; ++d)
        if (rlc_combinable(B, d)) rlc_mark(B, d, TBG_PS_VALID);
    return;
  }
  uint32_t n = 0, lone = d0;
  for (uint32_t d = d0; d < d1; ++d)
    if (rlc_combinable(B, d)) { ++n; lone = d; }
  if (n == 1) {
    resolve_bad_duty(B, lone, f, lead);
    return;
  }
  hex_store(B.chunk_fe + (size_t)3 * QUAD_WORDS * k, f);
  if (lead) B.cid_list[atomicAdd(&B.counters[CNT_CID], 1u)] = k;
}

// Level 1.5b lines, one thread per entry: S'_c = sum_d w_d S_d (suffix sums)
// and the points w_d P_d, stored as (-x, y) for the line evaluations.
__global__ void TBG_LAUNCH k_rlc_cident_lines(DevBatch B) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B.counters[CNT_CID]) return;
  const uint32_t G = B.rlc_group, C = B.rlc_chunk, nch = (G + C - 1) / C;
  const uint32_t k = B.cid_list[j], qc = B.chunk_list[k], g = qc / nch, c = qc % nch;
  const uint32_t d0 = g * G + c * C, d1 = min(min(d0 + C, g * G + G), B.n_duties);
  G2J T = jac_inf<Fp2>(), U = jac_inf<Fp2>();
  for (uint32_t d = d1; d-- > d0;) {
    if (!rlc_combinable(B, d)) continue;
    T = jac_add(T, B.dv_s[d]);
    U = jac_add(U, T);
  }
  G2A Sa;
  if (!jac_to_aff(U, Sa)) {
    B.cid_list[j] = k | ID_DEGENERATE;
    return;
  }
  uint32_t w = 0;
  for (uint32_t d = d0; d < d1; ++d) {
    if (!rlc_combinable(B, d)) continue;
    ++w;
    G1A wp = B.dv_p[d];  // (-x, y)
    if (w > 1) {
      wp.x = fp_reduce(fp_neg(wp.x));
      jac_to_aff(jac_mul_u64(jac_from_aff(wp), w), wp);  // w < r: never the identity
      wp.x = fp_reduce(fp_neg(wp.x));
    }
    B.cid_p[(size_t)C * j + (w - 1)] = wp;
  }
  B.pend_pts[j] = Sa;  // lines: k_lines_fold<FOLD_CID>
}

// Level 1.5b check: one hexad per entry computes A'_c over the chunk's duties
// and tests A_c^w == A'_c.  Found -> the other duties are valid and duty w
// is resolved with A = A_c; not found (two or more bad duties, rare) -> the
// chunk's candidates go to level 3.
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_rlc_cident_check(DevBatch B) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t j = hex_slot(t) + B.fb_base;
  if (hex_slot(t) == 0xFFFFFFFFu || j >= B.counters[CNT_CID] || !fb_in_pass(B, j)) return;
  const bool lead = hex_lead();
  const uint32_t G = B.rlc_group, C = B.rlc_chunk, nch = (G + C - 1) / C;
  const uint32_t entry = B.cid_list[j], k = entry & ~ID_DEGENERATE;
  const uint32_t qc = B.chunk_list[k], g = qc / nch, c = qc % nch;
  const uint32_t d0 = g * G + c * C, d1 = min(min(d0 + C, g * G + G), B.n_duties);
  uint32_t found = 0, n = 0;
  for (uint32_t d = d0; d < d1; ++d) n += rlc_combinable(B, d) ? 1u : 0u;
  const Fp4h A = hex_load(B.chunk_fe + (size_t)3 * QUAD_WORDS * k);
  if (!(entry & ID_DEGENERATE)) {
    const uint32_t* ls = B.cid_lines + fb_slot(B, j);
    const G1A* wp = B.cid_p + (size_t)C * j;  // (-x, y)
    const Fp4h f = hex_miller([&](Fp4h x, int idx) {
      x = hex_line_folded(x, ls, idx);
      uint32_t r = 0;
#pragma unroll 1
      for (uint32_t d = d0; d < d1; ++d) {
        if (!rlc_combinable(B, d)) continue;
        const G1A& P = wp[r++];
        x = hex_line_at(x, B.h_lines + (size_t)LINES_WORDS * B.duty_msg[d], idx, P.x, P.y);
      }
      return x;
    });
    // (A'_c)^-1: the conjugate is the inverse in GT
    found = hex_find_power(A, hex_final_exp_in(f), n);
  }
  uint32_t w = 0, bad = d0;
  for (uint32_t d = d0; d < d1; ++d) {
    if (!rlc_combinable(B, d)) continue;
    if (++w == found) bad = d;
    else if (lead) {
      if (found) rlc_mark(B, d, TBG_PS_VALID);
      else rlc_push_partials(B, d);
    }
  }
  if (found) resolve_bad_duty(B, bad, A, lead);
}

// Level 2b lines, one thread per entry: P' = sum w_i r_i pk_i (affine) and
// the lines of S' = sum w_i r_i s_i, w_i = 1..n the candidate's rank from the
// duty's start (suffix sums from its end: two additions per candidate).
__global__ void TBG_LAUNCH k_rlc_ident_lines(DevBatch B) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= B.counters[CNT_DUTIES]) return;
  const uint32_t d = B.id_list[k];
  G1J Tp = jac_inf<Fp>(), Up = jac_inf<Fp>();
  G2J Ts = jac_inf<Fp2>(), Us = jac_inf<Fp2>();
  for (uint32_t i = B.duty_first[d + 1]; i-- > B.duty_first[d];) {
    if (!rlc_candidate(B, i)) continue;
    Tp = jac_add(Tp, B.part_p[i]);
    Up = jac_add(Up, Tp);
    Ts = jac_add(Ts, B.part_s[i]);
    Us = jac_add(Us, Ts);
  }
  G1A Pa;
  G2A Sa;
  if (!jac_to_aff(Up, Pa) || !jac_to_aff(Us, Sa)) {
    B.id_list[k] = d | ID_DEGENERATE;
    return;
  }
  B.id_p[k] = Pa;
  B.pend_pts[k] = Sa;  // lines: k_lines_fold<FOLD_IDENT>
}

// Level 2b check: one hexad per entry computes A'_d and tests A_d^w == A'_d.
// Found -> partial w invalid, the others valid; not found -> level 3.
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_rlc_ident_check(DevBatch B) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (hex_slot(t) == 0xFFFFFFFFu) return;
  const bool lead = hex_lead();
  const uint32_t per = (gridDim.x * (blockDim.x / 64u) * 10u);
  fb_pass_loop(B, hex_slot(t), per, B.counters[CNT_DUTIES], [&](uint32_t k) {
  const uint32_t entry = B.id_list[k], d = entry & ~ID_DEGENERATE;
  uint32_t found = 0;
  if (!(entry & ID_DEGENERATE)) {
    const G1A P = B.id_p[k];
    Fp nx = fp_reduce(fp_neg(P.x));
    const uint32_t* ls = B.id_lines + fb_slot(B, k);
    const uint32_t* lh = B.h_lines + (size_t)LINES_WORDS * B.duty_msg[d];
    const Fp4h f = hex_miller([&](Fp4h x, int idx) { return hex_line_at(hex_line_folded(x, ls, idx), lh, idx, nx, P.y); });
    const Fp4h inv_a2 = hex_final_exp_in(f);
    found = hex_find_power(hex_load(B.id_fe + (size_t)3 * QUAD_WORDS * k), inv_a2, rlc_candidates(B, d));
  }
  if (!lead) return;
  if (!found) {
    rlc_push_partials(B, d);
    return;
  }
  uint32_t w = 0;
  for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i) {
    if (!rlc_candidate(B, i)) continue;
    B.partial_status[i] = ++w == found ? TBG_PS_INVALID : TBG_PS_VALID;
  }
  });
}

// ------------------------------------------------------------ level 1g
// The exponent test over a failed GROUP's candidates (members = partials,
// w_i = the candidate's rank in the group, A = the group's value from
// k_rlc_group_final): with exactly one bad partial -- most failed groups at
// realistic invalid rates -- it is found with ONE more check instead of the
// three levels 1.5 / 1.5b / 2b (each a final exponentiation deep).  A group
// the test cannot resolve hands its chunks to level 1.5 as before.

// G2J / G1J of lane ^ m within groups of `width` lanes
template <class P>
__device__ __forceinline__ P shfl_xor_pt(const P& a, int m, int width) {
  P r;
  const uint32_t* src = (const uint32_t*)&a;
  uint32_t* dst = (uint32_t*)&r;
#pragma unroll
  for (int j = 0; j < (int)(sizeof(P) / 4); ++j) dst[j] = (uint32_t)__shfl_xor((int)src[j], m, width);
  return r;
}

// lanes per level-1g entry: the group size rounded up to a power of two (<= 64)
__device__ __forceinline__ uint32_t gid_width(uint32_t G) { return G <= 1 ? 1u : 1u << (32 - __clz((int)(G - 1))); }

// Level 1g lines, one LANE PER DUTY of the entry's group (a power-of-two run
// of lanes): with n_d the candidates of duty d and o_d those ranked before it,
//   P'_d = [o_d] sum_(i in d) p_i + sum_j j p_j   (p_i = r_i pk_i; suffix sums),
//   S'   = sum_d ([o_d] sum_(i in d) s_i + sum_j j s_j)   (a shuffle tree),
// o_d by a prefix scan over the lanes.  P'_d is stored by the duty's position
// in the group as (-x, y); S' goes to pend_pts for its lines.
__global__ void TBG_LAUNCH k_rlc_gident_lines(DevBatch B) {
  const uint32_t G = B.rlc_group, W = gid_width(G);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, k = t / W, r = t % W;
  if (k >= B.counters[CNT_GID]) return;  // (W-lane uniform)
  const uint32_t g = B.gid_list[k], d = g * G + r;
  const bool valid = r < G && d < B.n_duties && rlc_combinable(B, d);
  G2J Xs = jac_inf<Fp2>(), Ys = jac_inf<Fp2>();
  G1J Xp = jac_inf<Fp>(), Yp = jac_inf<Fp>();
  uint32_t n = 0;
  if (valid) {
    for (uint32_t i = B.duty_first[d + 1]; i-- > B.duty_first[d];) {
      if (!rlc_candidate(B, i)) continue;
      Xs = jac_add(Xs, B.part_s[i]);
      Ys = jac_add(Ys, Xs);
      Xp = jac_add_in<Fp, true>(Xp, B.part_p[i]);
      Yp = jac_add_in<Fp, true>(Yp, Xp);
      ++n;
    }
  }
  uint32_t o = n;  // inclusive scan of n over the run, then exclusive
  for (uint32_t m = 1; m < W; m <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)o, m, W);
    if (r >= m) o += v;
  }
  o -= n;
  bool ok = true;
  if (valid) {
    if (o) {
      Yp = jac_add_in<Fp, true>(Yp, jac_mul_u64(Xp, o));
      Ys = jac_add(Ys, jac_mul_u64(Xs, o));
    }
    G1A wp;
    ok = jac_to_aff(Yp, wp);
    wp.x = fp_reduce(fp_neg(wp.x));
    B.gid_p[(size_t)G * k + r] = wp;
  }
  for (uint32_t m = 1; m < W; m <<= 1) Ys = jac_add(Ys, shfl_xor_pt(Ys, (int)m, (int)W));
  if (r == 0) {
    G2A Sa;
    if (jac_to_aff(Ys, Sa)) B.pend_pts[k] = Sa;  // lines: k_lines_fold<FOLD_GID>
    else ok = false;
  }
  if (!ok) atomicOr(&B.gid_list[k], ID_DEGENERATE);
}

// The chunks of group g with a combinable duty, to level 1.5 (as
// k_rlc_resolve_groups lists those of a group level 1g does not take).
__device__ __forceinline__ void push_group_chunks(const DevBatch& B, uint32_t g) {
  const uint32_t G = B.rlc_group, C = B.rlc_chunk, nch = (G + C - 1) / C;
  for (uint32_t c = 0; c < nch; ++c) {
    const uint32_t dc0 = g * G + c * C, dc1 = min(min(dc0 + C, g * G + G), B.n_duties);
    for (uint32_t d = dc0; d < dc1; ++d)
      if (rlc_combinable(B, d)) {
        B.chunk_list[atomicAdd(&B.counters[CNT_CHUNKS], 1u)] = g * nch + c;
        break;
      }
  }
}

// Level 1g Miller part, as level 1's: one hexad per (entry, chunk of
// rlc_chunk duties) over the duties' (P'_d, H(m_d)) pairs, and one hexad per
// entry for the S' pair (its folded lines), each product into gid_f.
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_rlc_gident_miller(DevBatch B) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t G = B.rlc_group, C = B.rlc_chunk, nch = (G + C - 1) / C, nq = nch + 1;
  const uint32_t s = hex_slot(t);
  if (s == 0xFFFFFFFFu) return;
  const uint32_t k = s / nq + B.fb_base, c = s % nq;
  if (k >= B.counters[CNT_GID] || !fb_in_pass(B, k)) return;
  const uint32_t entry = B.gid_list[k];
  if (entry & ID_DEGENERATE) return;
  const uint32_t g = entry, gd0 = g * G, gd1 = min(gd0 + G, B.n_duties);
  const uint32_t d0 = c == nch ? gd0 : min(gd0 + c * C, gd1), d1 = c == nch ? gd0 : min(d0 + C, gd1);
  const uint32_t* ls = B.gid_lines + fb_slot(B, k);
  const G1A* wp = B.gid_p + (size_t)G * k;  // (-x, y)
  const Fp4h f = hex_miller([&](Fp4h x, int idx) {
    if (c == nch) x = hex_line_folded(x, ls, idx);
#pragma unroll 1
    for (uint32_t d = d0; d < d1; ++d) {
      if (!rlc_combinable(B, d)) continue;
      const G1A& P = wp[d - gd0];
      x = hex_line_at(x, B.h_lines + (size_t)LINES_WORDS * B.duty_msg[d], idx, P.x, P.y);
    }
    return x;
  });
  hex_store(B.gid_f + (size_t)3 * QUAD_WORDS * ((size_t)k * nq + c), f);
}

// Candidates of an unresolved level-1g group up to which they all go to
// level 3 directly (more: the group's chunks go to level 1.5).
#ifndef TBG_GID_L3_MAX
#define TBG_GID_L3_MAX 40u
#endif

// Level 1g check: one hexad per entry multiplies its products into A'_g and
// tests A_g^w == A'_g.  Found -> candidate w invalid, the group's other
// candidates valid; not found (two or more bad partials) or degenerate ->
// the group's candidates go to the exact per-partial level (the levels
// between cost a final exponentiation of latency each whatever their list
// length, profiles/r03/gident/) -- or, with TBG_GIDENT=2, its chunks to
// level 1.5 as the round-2 order had them.
__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_rlc_gident_check(DevBatch B) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k = hex_slot(t) + B.fb_base;
  if (hex_slot(t) == 0xFFFFFFFFu || k >= B.counters[CNT_GID] || !fb_in_pass(B, k)) return;
  const bool lead = hex_lead();
  const uint32_t G = B.rlc_group, C = B.rlc_chunk, nq = (G + C - 1) / C + 1;
  const uint32_t entry = B.gid_list[k], g = entry & ~ID_DEGENERATE;
  const uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
  uint32_t found = 0, m = 0;
  for (uint32_t d = d0; d < d1; ++d)
    if (rlc_combinable(B, d)) m += rlc_candidates(B, d);
  if (!(entry & ID_DEGENERATE)) {
    const uint32_t* base = B.gid_f + (size_t)3 * QUAD_WORDS * ((size_t)k * nq);
    Fp4h f = hex_load(base);
    for (uint32_t c = 1; c < nq; ++c) f = hex_mul_ni(f, hex_load(base + (size_t)3 * QUAD_WORDS * c));
    const Fp4h inv_a2 = hex_final_exp_in(f);  // (A'_g)^-1
    found = hex_find_power(hex_load(B.grp_fe + (size_t)3 * QUAD_WORDS * k), inv_a2, m);
  }
  if (!lead) return;
  if (!found) {
    // a large group (many partials: 7-of-10 duties, mixed thresholds) is
    // narrowed by chunks first rather than checked partial by partial
    if (B.gident == 2 || m > TBG_GID_L3_MAX) {
      push_group_chunks(B, g);
    } else {
      for (uint32_t d = d0; d < d1; ++d)
        if (rlc_combinable(B, d)) rlc_push_partials(B, d);
    }
    return;
  }
  uint32_t w = 0;
  for (uint32_t d = d0; d < d1; ++d) {
    if (!rlc_combinable(B, d)) continue;
    for (uint32_t i = B.duty_first[d]; i < B.duty_first[d + 1]; ++i) {
      if (!rlc_candidate(B, i)) continue;
      B.partial_status[i] = ++w == found ? TBG_PS_INVALID : TBG_PS_VALID;
    }
  }
}

// Per-partial schedule (TBG_VERIFY_EACH): every candidate goes to level 3.
__global__ void TBG_LAUNCH k_list_all_partials(DevBatch B, const int32_t* pk_status, uint32_t n_pk) {
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

// Level 3 lines: one lane PAIR per listed partial (bls_pair.h, the Fp2
// coordinates split over the pair), the lines of its signature with -g1
// folded in.  (One lane per partial: 2.6 ms of latency per 16-batch launch
// at 1 % invalid against 1.4 ms, profiles/r04/merge/.)
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_lines_sig_list(DevBatch B) {
  // (pair-uniform branches; a grid smaller than the pass loops: fb_pass_loop)
  fb_pass_loop(B, (blockIdx.x * blockDim.x + threadIdx.x) >> 1, (gridDim.x * blockDim.x) >> 1,
               B.counters[CNT_PARTIALS], [&](uint32_t k) {
    const uint32_t i = B.part_list[k];
    const Fp nx = fp_reduce(fp_neg(fp_from_const(G1_X)));
    Aff<Fp2x> q = px_load(B.sig_aff[i]);
    q = {f_reduce(q.x), f_reduce(q.y)};  // decoded coordinates may be up to 16p (a negated root)
    px_g2_lines(q, nx, fp_from_const(G1_NEG_Y), B.sig_lines + fb_slot(B, k));
  });
}

// Level 3 check: one hexad per listed partial, the exact CoreVerify.
// (grid-stride over the pass: hexad slots per grid = 10 per wave)
TBG_DEV uint32_t hex_grid_slots() { return gridDim.x * (blockDim.x / 64u) * 10u; }

__global__ void TBG_LAUNCH_N(TBG_HEX_WAVES) k_verify_list(DevBatch B, const G1A* pk_aff) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (hex_slot(t) == 0xFFFFFFFFu) return;
  const bool lead = hex_lead();
  fb_pass_loop(B, hex_slot(t), hex_grid_slots(), B.counters[CNT_PARTIALS], [&](uint32_t k) {
    uint32_t i = B.part_list[k];
    uint32_t m = B.duty_msg[B.partial_duty[i]];
    if (B.h_status[m] != 0) {
      if (lead) B.partial_status[i] = TBG_PS_INVALID;
      return;
    }
    G1A pk = pk_aff[B.pubkey_ids[i]];
    Fp nx = fp_reduce(fp_neg(pk.x));
    const uint32_t* ls = B.sig_lines + fb_slot(B, k);
    const uint32_t* lh = B.h_lines + (size_t)LINES_WORDS * m;
    Fp4h f = hex_miller([&](Fp4h x, int idx) { return hex_line_at(hex_line_folded(x, ls, idx), lh, idx, nx, pk.y); });
    f = hex_final_exp_in(hex_conj(f));
    const bool ok = hex_is_one(f);
    if (lead) B.partial_status[i] = ok ? TBG_PS_VALID : TBG_PS_INVALID;
  });
}

// The fallback levels' list positions [0, max_entries) in passes of
// B.fb_window (the line buffer's capacity; 0: one pass), in stream order.
// body(P, n): n = the list positions the pass's grids cover -- all of the
// pass below B.fb_full, else FB_SMALL (the pass kernels that may run small
// loop over the rest: fb_pass_loop; the others take n = the pass).
constexpr uint32_t FB_SMALL = 640;  // 64 hexad waves, 20 pair waves
template <class F>
static void fb_passes(const DevBatch& B, uint32_t max_entries, F&& body, bool may_shrink = false) {
  const uint32_t W = B.fb_window ? B.fb_window : max_entries;
  for (uint32_t base = 0; base < max_entries; base += W) {
    DevBatch P = B;
    P.fb_base = base;
    const uint32_t n = max_entries - base < W ? max_entries - base : W;
    body(P, may_shrink && base > 0 && base >= B.fb_full && n > FB_SMALL ? FB_SMALL : n);  // (pass 0 always full)
  }
}

void launch_rlc_prepare(const DevBatch& B, const G1A* pk_aff, const G1A* xpk_aff, const G1A* pk_tab,
                        const int32_t* pk_status, uint32_t n_pk, hipStream_t st,
                        void (*after_keys)(const DevBatch&, hipStream_t)) {
  if (!B.n_duties) return;
  if (B.rlc_group == 0) {
    if (B.n_partials) TBG_KLAUNCH(k_list_all_partials, grid_for(B.n_partials), dim3(kBlock), st, B, pk_status, n_pk);
    if (after_keys) after_keys(B, st);
    return;
  }
  uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
  if (B.rlc_batch) {  // level 0: G1 products, P_d, the signature MSM and S's lines
    launch_l0_keys(B, pk_tab, pk_status, n_pk, st);
    if (after_keys) after_keys(B, st);
    launch_l0_msm(B, st);
    TBG_KLAUNCH(k_rlc_duty_sum<DSUM_L0_P>, duty_grid(B), dim3(BINV_BLOCK), st, B);
    launch_l0_lines(B, st);
    return;
  }
  if (after_keys) after_keys(B, st);
#if TBG_GMSM
  // the G1 products and P_d, then each group's S by its bucket MSM
  launch_rlc_g1(B, pk_tab, pk_aff, pk_status, n_pk, st);
  TBG_KLAUNCH(k_rlc_duty_sum<DSUM_P>, duty_grid(B), dim3(BINV_BLOCK), st, B);
  launch_gm_group_s(B, st);
#else
  launch_rlc_partials(B, pk_tab, pk_aff, pk_status, n_pk, st);
  TBG_KLAUNCH(k_rlc_duty_sum<DSUM_BOTH>, duty_grid(B), dim3(BINV_BLOCK), st, B);
  TBG_KLAUNCH(k_rlc_group_lines, grid_for(n_groups), dim3(kBlock), st, B);
#endif
  launch_lines_fold(B, FOLD_GROUPS, n_groups, st);
}

void launch_rlc_check(const DevBatch& B, const G1A* pk_aff, const G1A* xpk_aff, const int32_t* pk_status, uint32_t n_pk,
                      hipStream_t st) {
  if (!B.n_duties) return;
  if (B.rlc_group != 0) {
    uint32_t n_groups = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
    uint32_t nch = (B.rlc_group + B.rlc_chunk - 1) / B.rlc_chunk;
    // the level-0 and level-1 Miller products run on hexads (two waves per
    // SIMD, k_miller_hex.hip; the trio form measured 16.2 vs 15.2 ms, round 3)
    if (B.rlc_batch) {
      // level 0: the P chunks (kept for the group levels) and S, one product
      launch_l0_miller_hex(B, st);
      TBG_KLAUNCH(k_l0_fold, grid_for(hex_threads(n_groups)), dim3(kBlock), st, B);
      uint32_t in = 0, n = n_groups, out = n_groups;
      while (n > L0_TREE_FAN) {
        const uint32_t m = (n + L0_TREE_FAN - 1) / L0_TREE_FAN;
        TBG_KLAUNCH(k_l0_tree, grid_for(hex_threads(m)), dim3(kBlock), st, B, in, n, out);
        in = out;
        out += m;
        n = m;
      }
      launch_l0_final(B, in, n, st);
      TBG_KLAUNCH(k_l0_after, grid_for(n_groups), dim3(kBlock), st, B);
      // level 0 failed: the group levels' signature side (these kernels
      // return at once after a pass)
#if TBG_GMSM
      launch_gm_group_s(B, st);  // (G1 products, P_d and r_i: level 0's)
#else
      launch_rlc_partials(B, nullptr, pk_aff, pk_status, n_pk, st);  // (G1 products: level 0's)
      TBG_KLAUNCH(k_rlc_duty_sum<DSUM_FALLBACK_S>, duty_grid(B), dim3(BINV_BLOCK), st, B);
      TBG_KLAUNCH(k_rlc_group_lines, grid_for(n_groups), dim3(kBlock), st, B);
#endif
      launch_lines_fold(B, FOLD_GROUPS, n_groups, st);
      launch_group_s_miller_hex(B, st);
    } else {
      launch_groups_miller_hex(B, st);
    }
    TBG_KLAUNCH(k_rlc_group_final, grid_for(hex_threads(n_groups)), dim3(kBlock), st, B);
    TBG_KLAUNCH(k_rlc_resolve_groups, grid_for(B.n_duties), dim3(kBlock), st, B);
#if TBG_GMSM
    // the failed groups' r_i s_i and S_d, which every deeper level reads
    launch_gm_failed_partials(B, pk_aff, st);
    TBG_KLAUNCH(k_rlc_duty_sum<DSUM_FALLBACK_S>, duty_grid(B), dim3(BINV_BLOCK), st, B);
#endif
    if (B.rlc_group > 1) {
      // level 1g before the chunks: its unresolved groups add to the chunk list
      uint32_t W = 1;
      while (W < B.rlc_group) W <<= 1;
      TBG_KLAUNCH(k_rlc_gident_lines, grid_for(n_groups * W), dim3(kBlock), st, B);
      fb_passes(B, n_groups, [&](const DevBatch& P, uint32_t n) {
        launch_lines_fold(P, FOLD_GID, n, st);
        TBG_KLAUNCH(k_rlc_gident_miller, grid_for(hex_threads(n * (nch + 1))), dim3(kBlock), st, P);
        TBG_KLAUNCH(k_rlc_gident_check, grid_for(hex_threads(n)), dim3(kBlock), st, P);
      });
      TBG_KLAUNCH(k_rlc_chunk_lines, grid_for(n_groups * nch), dim3(kBlock), st, B);
      fb_passes(B, n_groups * nch, [&](const DevBatch& P, uint32_t n) {
        launch_lines_fold(P, FOLD_CHUNKS, n, st);
        TBG_KLAUNCH(k_rlc_check_chunks, grid_for(hex_threads(n)), dim3(kBlock), st, P);
      });
      TBG_KLAUNCH(k_rlc_cident_lines, grid_for(n_groups * nch), dim3(kBlock), st, B);
      fb_passes(B, n_groups * nch, [&](const DevBatch& P, uint32_t n) {
        launch_lines_fold(P, FOLD_CID, n, st);
        TBG_KLAUNCH(k_rlc_cident_check, grid_for(hex_threads(n)), dim3(kBlock), st, P);
      });
      TBG_KLAUNCH(k_rlc_ident_lines, grid_for(B.n_duties), dim3(kBlock), st, B);
      fb_passes(B, B.n_duties, [&](const DevBatch& P, uint32_t n) {
        launch_lines_fold(P, FOLD_IDENT, n, st);
        TBG_KLAUNCH(k_rlc_ident_check, grid_for(hex_threads(n)), dim3(kBlock), st, P);
      }, true);
    }
  }
  if (B.n_partials) {
    fb_passes(B, B.n_partials, [&](const DevBatch& P, uint32_t n) {
      TBG_KLAUNCH(k_lines_sig_list, grid_for(2 * n), dim3(kBlock), st, P);
      TBG_KLAUNCH(k_verify_list, grid_for(hex_threads(n)), dim3(kBlock), st, P, pk_aff);
    }, true);
  }
}

}  // namespace tbg
