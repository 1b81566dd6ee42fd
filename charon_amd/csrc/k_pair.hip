// Level-0 RLC products [r_i] s_i (G2) and [r_i] pk_i (G1), one lane per
// partial for the Fp-level work and one lane PAIR for the G2 point work
// (bls_pair.h: halves the G2 state per lane so the kernel fits two waves per
// SIMD, which on gfx950 issue the multiply-adds ~1.7x faster than one).
//
//   phase 1, lane L owns partial L: the G1 product from the key's pair
//            table, the G2 table's slope inversion batched over the workgroup;
//   phase 2, lanes (2k, 2k+1) run the G2 table and its 15 doublings + 31
//            additions for partial 2k, then for 2k+1, with the Fp2
//            coordinates split over the pair and the owner's inverse and
//            digits handed over by DPP.
//
// Measured and rejected: separate G1 / pair-G2 kernels with inversion-free
// Jacobian tables (bls_rlc.h *_j) -- 446 spilled VGPRs in the pair kernel,
// 3.19 ms against 2.85 ms for the fused single-lane kernel.
#define TBG_ADD_DBL_INLINE 1
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernel in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_rlc.h"
#include "bls_pair.h"
#include "bls_batchinv.h"

namespace tbg {

__device__ __forceinline__ bool rlc_usable_pk(const DevBatch& B, uint32_t i, const int32_t* pk_status, uint32_t n_pk) {
  int32_t st = B.partial_status[i];
  if (st != TBG_PS_NOT_VERIFIED && st != TBG_PS_ERR_PUBKEY) return false;
  uint32_t pid = B.pubkey_ids[i];
  return pid < n_pk && pk_status[pid] == DEC_OK;
}

// Only the first usable candidate of the whole level-1 GROUP takes r = 1 (a
// fixed coefficient per duty would let two invalid partials of different
// duties in one group cancel; k_rlc.hip).  Both kernels decide it the same way
// whichever of them has already marked bad-key partials ERR_PUBKEY.
__device__ __forceinline__ bool rlc_group_lead(const DevBatch& B, uint32_t i, const int32_t* pk_status, uint32_t n_pk) {
  if (B.rlc_batch) return false;  // level 0 drew every r_i at random (k_msm.hip); the groups reuse them
  const uint32_t d = B.partial_duty[i];
  const uint32_t d0 = (d / B.rlc_group) * B.rlc_group;
  for (uint32_t j = B.duty_first[d0]; j < i; ++j)
    if (rlc_usable_pk(B, j, pk_status, n_pk)) return false;
  return true;
}

// The pair-owner's Fp2 value (owner = the lane of parity j) in pair form:
// every lane sends the component its partner needs, the owner keeps its own.
__device__ __forceinline__ Fp2x px_from_owner(const Fp2& own, uint32_t j) {
  const uint32_t par = pair_par();
  const Fp recv = pair_xch(par ? own.c0 : own.c1);  // the partner's value, component par
  return {par == j ? (par ? own.c1 : own.c0) : recv};
}
__device__ __forceinline__ uint32_t u32_from_owner(uint32_t own, uint32_t j) {
  const uint32_t recv = pair_u32(own);
  return pair_par() == j ? own : recv;
}

// The G1 product comes from the key's pair table (k_pubkey_tables, computed
// once per key) -- or was already formed by level 0 (k_rlc_g1_l0, same r_i)
// when this runs after a level-0 failure; the G2 table's slope inversion is
// batched over the workgroup (bls_batchinv.h).
__global__ void __launch_bounds__(BINV_BLOCK, TBG_PAIR_WAVES) k_rlc_partial2(DevBatch B, const G1A* pk_tab,
                                                                             const G1A* pk_aff,
                                                                             const int32_t* pk_status, uint32_t n_pk) {
  // No early return: both lanes of every pair must reach the DPP exchanges and
  // every thread the workgroup's batched inversion (the level-0 pass below is
  // grid-uniform).
  if (B.counters[CNT_L0_OK]) return;  // level 0 accepted the batch: no group levels
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  bool active = i < B.n_partials && B.partial_status[i] == TBG_PS_NOT_VERIFIED;
  uint32_t pid = 0;
  if (active) {
    pid = B.pubkey_ids[i];
    if (pid >= n_pk || pk_status[pid] != DEC_OK) {
      B.partial_status[i] = TBG_PS_ERR_PUBKEY;
      active = false;
    }
  }
  const bool lead = active && rlc_group_lead(B, i, pk_status, n_pk);
  const bool work = active && !lead;
  uint32_t a[4] = {0, 0, 0, 0};
  Fp2 dx2 = fp2_one();
  if (lead) {
    B.part_s[i] = jac_from_aff(B.sig_aff[i]);
    B.part_p[i] = jac_from_aff(pk_aff[pid]);
  } else if (work) {
    rlc_digits(rlc_scalar(B.rlc_seed, i), a);
    const G2A s = B.sig_aff[i];
    dx2 = fp2_reduce(fp2_sub(fp2_mul(fp2_conj(s.x), fp2_from_const(PSI_X)), s.x));  // psi(s).x - s.x
    if (!B.rlc_batch) B.part_p[i] = rlc_mul_key(pk_tab + (size_t)PK_TAB * pid, a);
  }
  const Fp2 inv2 = block_batch_inv2<BINV_WAVES>(dx2, work);  // every thread of the workgroup
  for (uint32_t j = 0; j < 2; ++j) {
    if (!u32_from_owner(work ? 1u : 0u, j)) continue;  // pair-uniform
    const uint32_t owner = (i & ~1u) | j;
    const Fp2x ix = px_from_owner(inv2, j);
    uint32_t u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = u32_from_owner(a[k], j);
    const Aff<Fp2x> s = px_load(B.sig_aff[owner]);
    const Aff<Fp2x> ps{f_mulc(f_conj(s.x), PSI_X), f_mulc(f_conj(s.y), PSI_Y)};  // psi(s) = [x] s
    Aff<Fp2x> ap, am;
    rlc_pair_from_inv(s, ps, ix, ap, am);
    px_store(B.part_s[owner], rlc_mul_table(ap, am, fp_from_const(PSI2_X), u));
  }
}

// List mode (k_gmsm.hip): r_i s_i for the candidates of failed groups only
// (gm_list, CNT_LAZY entries), after the group checks; the G1 products and
// the key marks are made, the group's lead is gm_lead.  Lane L owns list
// entry base + L (its slope denominator in the workgroup's batched
// inversion), the lane pair runs the G2 products of its two entries, as
// k_rlc_partial2 does (one entry per pair measured 4.7 vs 4.2 ms at 1 %
// invalid: the inversion amortised over half the partials).  Grid-stride
// over the list with a workgroup-uniform trip count.
__global__ void __launch_bounds__(BINV_BLOCK, TBG_PAIR_WAVES) k_rlc_partial2_list(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  const uint32_t nl = B.counters[CNT_LAZY];
#pragma unroll 1
  for (uint32_t base = blockIdx.x * blockDim.x; base < nl; base += gridDim.x * blockDim.x) {
    const uint32_t t = base + threadIdx.x;
    const bool active = t < nl;
    const uint32_t i = active ? B.gm_list[t] : 0u;
    const bool lead = active && B.gm_lead[B.partial_duty[i] / B.rlc_group] == i;
    const bool work = active && !lead;
    uint32_t a[4] = {0, 0, 0, 0};
    Fp2 dx2 = fp2_one();
    if (lead) {
      B.part_s[i] = jac_from_aff(B.sig_aff[i]);
    } else if (work) {
      rlc_digits(rlc_scalar(B.rlc_seed, i), a);
      const G2A s = B.sig_aff[i];
      dx2 = fp2_reduce(fp2_sub(fp2_mul(fp2_conj(s.x), fp2_from_const(PSI_X)), s.x));  // psi(s).x - s.x
    }
    const Fp2 inv2 = block_batch_inv2<BINV_WAVES>(dx2, work);  // every thread of the workgroup
    for (uint32_t j = 0; j < 2; ++j) {
      if (!u32_from_owner(work ? 1u : 0u, j)) continue;  // pair-uniform
      const uint32_t owner = u32_from_owner(i, j);  // the listed partial of the pair's lane j
      const Fp2x ix = px_from_owner(inv2, j);
      uint32_t u[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) u[k] = u32_from_owner(a[k], j);
      const Aff<Fp2x> s = px_load(B.sig_aff[owner]);
      const Aff<Fp2x> ps{f_mulc(f_conj(s.x), PSI_X), f_mulc(f_conj(s.y), PSI_Y)};  // psi(s) = [x] s
      Aff<Fp2x> ap, am;
      rlc_pair_from_inv(s, ps, ix, ap, am);
      px_store(B.part_s[owner], rlc_mul_table(ap, am, fp_from_const(PSI2_X), u));
    }
  }
}

void launch_rlc_partials_list(const DevBatch& B, const G1A* pk_aff, hipStream_t st) {
  (void)pk_aff;
  uint32_t blocks = (B.n_partials + BINV_BLOCK - 1) / BINV_BLOCK;
  if (blocks > 4096) blocks = 4096;
  if (blocks) TBG_KLAUNCH(k_rlc_partial2_list, dim3(blocks), dim3(BINV_BLOCK), st, B);
}

void launch_rlc_partials(const DevBatch& B, const G1A* pk_tab, const G1A* pk_aff, const int32_t* pk_status,
                         uint32_t n_pk, hipStream_t st) {
  if (!B.n_partials) return;
  TBG_KLAUNCH(k_rlc_partial2, dim3((B.n_partials + BINV_BLOCK - 1) / BINV_BLOCK), dim3(BINV_BLOCK), st, B, pk_tab,
              pk_aff, pk_status, n_pk);
}

}  // namespace tbg
