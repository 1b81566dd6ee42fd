// Level 0 of the RLC schedule: the whole device batch (every caller batch
// packed into one launch) as ONE product check
//   prod_d e(P_d, H(m_d)) * e(-g1, S) == 1,  P_d = sum_i r_i pk_i,  S = sum_i r_i s_i,
// before any group check (reference: the per-partial CoreVerify calls of
// tbls.Verify / VerifyAndAggregate, tbls/tss.go:153-197, all of which a pass
// accepts; any failure falls through to the group levels of k_rlc.hip, so
// every verdict stays the exact per-item one).
//
// The signature side is the bucket MSM of bls_msm.h: 4 mixed additions per
// partial instead of a 64-bit G2 scalar multiplication (15 doublings, 31
// additions and a field inversion per partial at the group levels); the key
// side uses per-key pair tables A+- = pk +- [x]pk computed once when the key
// table is loaded, so P_d needs no inversion per partial either.
//
//   k_rlc_g1_l0      one lane per partial: r_i, [r_i] pk_i, bucket sizes
//   k_msm_scan       bucket offsets (one workgroup)
//   k_msm_scatter    bucket entries
//   k_msm_bucket_part  one lane PAIR per quarter of a bucket: its sum
//   k_msm_bucket     one lane PAIR per bucket: the quarters' sum times (2j + 1)
//   k_msm_tree, k_msm_tree_final  the sum of the scaled buckets (LDS trees), S affine
#define TBG_ADD_DBL_INLINE 1
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernels in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_msm.h"
#include "bls_pair.h"
#include "bls_batchinv.h"

namespace tbg {

// Table of every usable key (k_rlc_g1_l0, k_rlc_partial2): the window table
// of bls_rlc.h (TBG_PK_W2: e0 pk + e1 [x]pk, e0 in {1, 3}, e1 in {+-1, +-3})
// or the pair table A+ = pk + [x]pk, A- = pk - [x]pk, each entry's affine
// conversion batched over the workgroup (bls_batchinv.h).
__global__ void __launch_bounds__(BINV_BLOCK) k_pubkey_tables(const G1A* pk, const G1A* xpk, const int32_t* status,
                                                              uint32_t n, G1A* tab) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n;
  const bool ok = in && status[i] == DEC_OK;
  G1A p0{fp_zero(), fp_zero()}, x0 = p0;
  if (ok) {
    p0 = pk[i];
    x0 = xpk[i];
  }
#if TBG_PK_W2
  // e0 pk + e1 [x]pk is never the identity for a prime-order key (it would
  // need x = -e0 / e1 mod r); every thread runs every batched conversion
#pragma unroll 1
  for (int k = 0; k < (int)PK_TAB; ++k) {
    const G1J e = ok ? rlc_key_table_w2_entry(p0, x0, k) : jac_inf<Fp>();
    G1A a{fp_zero(), fp_zero()};
    const bool got = block_jac_to_aff<BINV_WAVES>(e, ok, a);
    if (in) tab[(size_t)PK_TAB * i + k] = got ? a : G1A{fp_zero(), fp_zero()};
  }
#else
  // x0.x != p0.x for a prime-order key ([x]pk = +-pk would need x = +-1 mod r)
  const Fp t = block_batch_inv<BINV_WAVES>(fp_reduce(fp_sub(x0.x, p0.x)), ok);  // every thread of the workgroup
  if (!in) return;
  G1A ap{fp_zero(), fp_zero()}, am = ap;
  if (ok) rlc_pair_from_inv(p0, x0, t, ap, am);
  tab[2ull * i] = ap;
  tab[2ull * i + 1] = am;
#endif
}

// Level-0 G1 side, one lane per partial: unusable keys are marked, every
// candidate's r_i is drawn (no group lead: at level 0 two r = 1 partials of
// different groups could cancel) and [r_i] pk_i computed from the key's pair
// table; the four digits count into their buckets.
__global__ void TBG_LAUNCH k_rlc_g1_l0(DevBatch B, const G1A* tab, const int32_t* pk_status, uint32_t n_pk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials || B.partial_status[i] != TBG_PS_NOT_VERIFIED) return;
  const uint32_t pid = B.pubkey_ids[i];
  if (pid >= n_pk || pk_status[pid] != DEC_OK) {
    B.partial_status[i] = TBG_PS_ERR_PUBKEY;
    return;
  }
  const uint64_t r = rlc_scalar(B.rlc_seed, i);
  uint32_t u[4];
  rlc_digits(r, u);
  B.msm_r[i] = r;
  B.part_p[i] = rlc_mul_key(tab + (size_t)PK_TAB * pid, u);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    bool neg;
    atomicAdd(&B.msm_off[msm_bucket(u[k], neg)], 1u);
  }
}

// Exclusive scan of the bucket sizes into offsets (msm_off) and cursors
// (msm_cur): one workgroup of 1024 lanes, 32 buckets per lane.
constexpr int kScanBlock = 1024;
__global__ void __launch_bounds__(kScanBlock) k_msm_scan(DevBatch B) {
  TBG_URGENT();
  __shared__ uint32_t part[kScanBlock];
  constexpr uint32_t per = MSM_BUCKETS / kScanBlock;
  const uint32_t t = threadIdx.x, j0 = t * per;
  uint32_t sum = 0;
  for (uint32_t j = 0; j < per; ++j) sum += B.msm_off[j0 + j];
  part[t] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < kScanBlock; d <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t j = 0; j < per; ++j) {
    const uint32_t c = B.msm_off[j0 + j];
    B.msm_off[j0 + j] = run;
    B.msm_cur[j0 + j] = run;
    run += c;
  }
  if (t == kScanBlock - 1) B.msm_off[MSM_BUCKETS] = run;
}

__global__ void TBG_LAUNCH k_msm_scatter(DevBatch B) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials || B.partial_status[i] != TBG_PS_NOT_VERIFIED) return;
  uint32_t u[4];
  rlc_digits(B.msm_r[i], u);
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    bool neg;
    const uint32_t j = msm_bucket(u[k], neg);
    B.msm_ent[atomicAdd(&B.msm_cur[j], 1u)] = msm_entry(i, k, neg);
  }
}

// psi^k(s) (bls_msm.h) with the Fp2 coordinates split over the lane pair.
__device__ __forceinline__ Aff<Fp2x> px_psi_k(const G2A& s, uint32_t k, bool neg) {
  Aff<Fp2x> p = px_load(s);
  p.y = f_reduce(p.y);  // decoded coordinates may be up to 16p (a negated root)
  if (k & 1) p = Aff<Fp2x>{f_mulc(f_conj(p.x), PSI_X), f_mulc(f_conj(p.y), PSI_Y)};
  const bool ny = ((k & 2) != 0) != neg;
  if (k & 2) p.x = f_mulfp(p.x, fp_from_const(PSI2_X));
  if (ny) p.y = f_reduce(f_neg(p.y));
  return p;
}

// Bucket sums in two kernels so that no lane pair runs a long chain: a pair
// per (bucket j, slice of its entries) adds its slice (~20 mixed additions),
// then a pair per bucket adds the MSM_SPLIT slice sums and multiplies by
// (2j + 1) (one pair per bucket running all ~80 additions and the scaling
// took 5.0 ms per 160k-DV launch, latency-bound on 1,024 waves).
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_msm_bucket_part(DevBatch B) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // both lanes of a pair take the same branches
  if (w >= MSM_BUCKETS * MSM_SPLIT) return;
  if (B.counters[CNT_L0_BAD]) return;
  const uint32_t j = w / MSM_SPLIT, sl = w % MSM_SPLIT;
  const uint32_t o0 = B.msm_off[j], n = B.msm_off[j + 1] - o0;
  const uint32_t e0 = o0 + (n * sl) / MSM_SPLIT, e1 = o0 + (n * (sl + 1)) / MSM_SPLIT;
  Jac<Fp2x> acc = jac_inf<Fp2x>();
#pragma unroll 1
  for (uint32_t e = e0; e < e1; ++e) {
    const uint32_t v = B.msm_ent[e];
    acc = jac_add_aff_in(acc, px_psi_k(B.sig_aff[v >> 3], (v >> 1) & 3u, (v & 1u) != 0));
  }
  px_store(B.msm_part[w], acc);
}

// [2j + 1] (sum of bucket j's slices): FAST = the additions without the
// doubling branch (`exc` set when one needed it), else the complete formulas
// (out-of-line calls)
template <bool FAST>
__device__ __forceinline__ Jac<Fp2x> msm_bucket_scaled(const DevBatch& B, uint32_t j, bool& exc) {
  Jac<Fp2x> acc = px_load(B.msm_part[MSM_SPLIT * j]);
#pragma unroll 1
  for (uint32_t sl = 1; sl < MSM_SPLIT; ++sl) {
    const Jac<Fp2x> q = px_load(B.msm_part[MSM_SPLIT * j + sl]);
    acc = FAST ? jac_add_x(acc, q, exc) : jac_add(acc, q);
  }
  const uint32_t m = 2 * j + 1;
  if (m > 1 && !jac_is_inf(acc)) {
    // the base waits in the output slot, read where it is added (held in
    // registers across the ladder it spilled ~40 words per step)
    px_store(B.msm_bkt[j], acc);
    const int top = 31 - __builtin_clz(m);
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; --bit) {
      acc = jac_dbl_in(acc);
      if ((m >> bit) & 1u) {
        __asm__ __volatile__("" ::: "memory");
        const Jac<Fp2x> b = px_load(B.msm_bkt[j]);
        acc = FAST ? jac_add_x(acc, b, exc) : jac_add(acc, b);
      }
    }
  }
  return acc;
}
#ifndef TBG_MSM_BUCKET_X
#define TBG_MSM_BUCKET_X 1  // 0: the complete additions inline (139 spilled VGPRs)
#endif
// the doubling case of an addition (equal slice sums: crafted signatures
// only) redone with the complete formulas, out of line
__device__ __noinline__ Jac<Fp2x> msm_bucket_complete(const DevBatch& B, uint32_t j) {
  bool unused = false;
  return msm_bucket_scaled<false>(B, j, unused);
}

// (the additions without the doubling branch: the complete formulas inline
// spilled 139 VGPRs on this latency-bound tail kernel)
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_msm_bucket(DevBatch B) {
  TBG_URGENT();
  const uint32_t j = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (j >= MSM_BUCKETS) return;
  if (B.counters[CNT_L0_BAD]) return;
#if TBG_MSM_BUCKET_X
  bool exc = false;
  Jac<Fp2x> acc = msm_bucket_scaled<true>(B, j, exc);
  if (!pair_all(!exc)) acc = msm_bucket_complete(B, j);  // (pair-uniform)
#else
  Jac<Fp2x> acc = px_load(B.msm_part[MSM_SPLIT * j]);
#pragma unroll 1
  for (uint32_t sl = 1; sl < MSM_SPLIT; ++sl) acc = jac_add_in<Fp2x, true>(acc, px_load(B.msm_part[MSM_SPLIT * j + sl]));
  const uint32_t m = 2 * j + 1;
  if (m > 1 && !jac_is_inf(acc)) {
    const Jac<Fp2x> b = acc;
    const int top = 31 - __builtin_clz(m);
#pragma unroll 1
    for (int bit = top - 1; bit >= 0; --bit) {
      acc = jac_dbl_in(acc);
      if ((m >> bit) & 1u) acc = jac_add_in<Fp2x, true>(acc, b);
    }
  }
#endif
  px_store(B.msm_bkt[j], acc);
}

// Tree sum of the scaled buckets in TWO kernels (four passes of 16-point
// chains took 60 dependent additions, ~1.8 ms of a launch's critical path):
// a lane pair adds MSM_TREE_PER points, then the workgroup halves its pairs
// through LDS (log2 levels); the first kernel leaves one point per
// workgroup, the second sums those the same way and writes S in affine form
// (or flags level 0 when S is the point at infinity): 3 + 7 + 1 + 5 = 16
// dependent additions.
constexpr uint32_t MSM_TREE_PAIRS = 128;  // lane pairs per workgroup of the first kernel
constexpr uint32_t MSM_TREE_PER = 4;      // points per pair in the first kernel
constexpr uint32_t MSM_TREE_WG = MSM_BUCKETS / (MSM_TREE_PAIRS * MSM_TREE_PER);  // 64 partial sums
static_assert(MSM_TREE_WG <= 2 * 64 && MSM_TREE_WG <= MSM_SUM_ENTRIES, "second tree kernel: one workgroup");

// acc summed over the workgroup's PAIRS lane pairs (every thread calls it;
// pair 0 ends with the total)
template <uint32_t PAIRS>
__device__ __forceinline__ Jac<Fp2x> pair_tree_sum(Jac<Fp2x> acc, Jac<Fp2x>* lds) {
  const uint32_t t = threadIdx.x, pr = t >> 1;
#pragma unroll 1
  for (uint32_t s = 1; s < PAIRS; s <<= 1) {
    lds[t] = acc;
    __syncthreads();
    if ((pr & (2 * s - 1)) == 0 && pr + s < PAIRS) acc = jac_add_in<Fp2x, true>(acc, lds[t + 2 * s]);
    __syncthreads();
  }
  return acc;
}

__global__ void __launch_bounds__(2 * MSM_TREE_PAIRS) k_msm_tree(DevBatch B) {
  TBG_URGENT();
  __shared__ Jac<Fp2x> lds[2 * MSM_TREE_PAIRS];
  if (B.counters[CNT_L0_BAD]) return;  // (grid-uniform)
  const uint32_t pr = threadIdx.x >> 1;
  const uint32_t a0 = (blockIdx.x * MSM_TREE_PAIRS + pr) * MSM_TREE_PER;
  Jac<Fp2x> acc = px_load(B.msm_bkt[a0]);
#pragma unroll 1
  for (uint32_t a = a0 + 1; a < a0 + MSM_TREE_PER; ++a) acc = jac_add_in<Fp2x, true>(acc, px_load(B.msm_bkt[a]));
  acc = pair_tree_sum<MSM_TREE_PAIRS>(acc, lds);
  if (pr == 0) px_store(B.msm_sum[blockIdx.x], acc);
}

__global__ void __launch_bounds__(MSM_TREE_WG) k_msm_tree_final(DevBatch B) {
  TBG_URGENT();
  constexpr uint32_t PAIRS = MSM_TREE_WG / 2;
  __shared__ Jac<Fp2x> lds[2 * PAIRS];
  if (B.counters[CNT_L0_BAD]) return;
  const uint32_t pr = threadIdx.x >> 1;
  Jac<Fp2x> acc = jac_add_in<Fp2x, true>(px_load(B.msm_sum[2 * pr]), px_load(B.msm_sum[2 * pr + 1]));
  acc = pair_tree_sum<PAIRS>(acc, lds);
  if (pr != 0) return;
  if (jac_is_inf(acc)) {
    if (pair_par() == 0) B.counters[CNT_L0_BAD] = 1;  // S = 0: no lines; the group levels decide
    return;
  }
  const Fp2x zi = f_inv(acc.Z);
  const Fp2x zi2 = f_sqr(zi);
  px_store(*B.batch_pt, Aff<Fp2x>{f_mul(acc.X, zi2), f_mul(acc.Y, f_mul(zi2, zi))});
}

void launch_pubkey_tables(const G1A* pk, const G1A* xpk, const int32_t* status, uint32_t n, G1A* tab, hipStream_t st) {
  if (n) TBG_KLAUNCH(k_pubkey_tables, dim3((n + BINV_BLOCK - 1) / BINV_BLOCK), dim3(BINV_BLOCK), st, pk, xpk, status, n,
                     tab);
}

// Level 0's key side: G1 products, bucket sizes, and the ERR_PUBKEY marks
// (after it the candidates are final: the speculative aggregation may run).
void launch_l0_keys(const DevBatch& B, const G1A* pk_tab, const int32_t* pk_status, uint32_t n_pk, hipStream_t st) {
  // (msm_off was zeroed by k_decode_sigs, the chain's first kernel)
  if (B.n_partials) TBG_KLAUNCH(k_rlc_g1_l0, grid_for(B.n_partials), dim3(kBlock), st, B, pk_tab, pk_status, n_pk);
}

// Level 0's signature side: the bucket MSM up to S (affine).
void launch_l0_msm(const DevBatch& B, hipStream_t st) {
  TBG_KLAUNCH(k_msm_scan, dim3(1), dim3(kScanBlock), st, B);
  if (B.n_partials) TBG_KLAUNCH(k_msm_scatter, grid_for(B.n_partials), dim3(kBlock), st, B);
  TBG_KLAUNCH(k_msm_bucket_part, grid_for(2 * MSM_BUCKETS * MSM_SPLIT), dim3(kBlock), st, B);
  TBG_KLAUNCH(k_msm_bucket, grid_for(2 * MSM_BUCKETS), dim3(kBlock), st, B);
  TBG_KLAUNCH(k_msm_tree, dim3(MSM_TREE_WG), dim3(2 * MSM_TREE_PAIRS), st, B);
  TBG_KLAUNCH(k_msm_tree_final, dim3(1), dim3(MSM_TREE_WG), st, B);
}

}  // namespace tbg
