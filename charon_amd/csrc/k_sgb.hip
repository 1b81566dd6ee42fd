// Batched subgroup test of the decoded signatures: the
// per-signature check psi(s) == [x] s (k_subgroup_sigs: 63 doublings + 5
// additions per signature) runs only for the members of groups whose
// random combinations fail.  Reference: tblsconv.SigFromCore's subgroup
// check (tblsconv/tblsconv.go:125-132) -- every partial still gets the exact
// per-item verdict.
//
// E2(Fp2) = G2 x H with |H| the G2 cofactor h2, whose smallest prime factor
// is 13.  Write s_i = g_i + t_i (t_i in H).  For a group of SGB_M consecutive
// partials and SGB_K combinations
//   Q_k = sum_i c_ik s_i,   c_ik uniform in {-6, ..., 6} (distinct mod 13),
// Q_k is in G2 iff sum_i c_ik t_i = 0.  If some t_j != 0, fix every other
// coefficient: c t_j takes 13 distinct values (ord t_j has no prime factor
// below 13), so at most one value of c_jk cancels -- probability <= 1/13 per
// combination, 13^-18 < 2^-66 for all 18.  The coefficients come from the
// batch's secret seed (sgb_digits, bls_rlc.h), so a submitter cannot aim at
// them.  Each Q_k is a bucket sum: bucket (k, v) adds +-s_i over the members
// with |c_ik| = v, and Q_k = sum_v v B_(k,v) by running sums -- ~16.6 mixed
// additions per signature instead of ~68 group operations, plus 18 tests per
// group of 1,024.
//
//   k_sgb_sort    one workgroup per group: digits, bucket counts and entries in LDS
//   k_sgb_bucket  one lane PAIR per (group, bucket, slice): the slice's sum
//   k_sgb_combine one lane PAIR per (group, combination): Q_k from its buckets
//   k_sgb_test    one lane PAIR per (group, combination): psi(Q_k) == [x] Q_k
// then k_subgroup_sigs tests the members of failed groups one by one.
#define TBG_ADD_DBL_INLINE 1
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernels in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_rlc.h"
#include "bls_pair.h"

namespace tbg {

#ifndef TBG_SGB_SORT_BLOCK
#define TBG_SGB_SORT_BLOCK 256
#endif
constexpr uint32_t kSgbSortBlock = TBG_SGB_SORT_BLOCK;  // threads per group's sort

__global__ void __launch_bounds__(kSgbSortBlock) k_sgb_sort(DevBatch B) {
  __shared__ uint32_t cnt[SGB_BUCKETS];
  __shared__ uint32_t off[SGB_BUCKETS + 1];
  __shared__ int8_t dig[SGB_M * SGB_K];  // (the largest group)
  const uint32_t g = blockIdx.x, t = threadIdx.x, m = B.sgb_m;
  const uint32_t i0 = g * m;
  const uint32_t n = min(m, B.n_partials - i0);
  for (uint32_t b = t; b < SGB_BUCKETS; b += kSgbSortBlock) cnt[b] = 0;
  if (t == 0) B.sgb_bad[g] = 0;
  __syncthreads();
  for (uint32_t li = t; li < n; li += kSgbSortBlock) {
    const bool ok = B.partial_status[i0 + li] == TBG_PS_NOT_VERIFIED;
    int32_t c[SGB_K];
    sgb_digits(B.sgb_seed, i0 + li, c);
#pragma unroll
    for (uint32_t k = 0; k < SGB_K; ++k) {
      const int32_t d = ok ? c[k] : 0;
      dig[li * SGB_K + k] = (int8_t)d;
      if (d) atomicAdd(&cnt[k * SGB_V + (uint32_t)(d < 0 ? -d : d) - 1], 1u);
    }
  }
  __syncthreads();
  if (t == 0) {
    uint32_t run = 0;
    for (uint32_t b = 0; b < SGB_BUCKETS; ++b) {
      off[b] = run;
      run += cnt[b];
    }
    off[SGB_BUCKETS] = run;
  }
  __syncthreads();
  uint32_t* goff = B.sgb_off + (size_t)(SGB_BUCKETS + 1) * g;
  for (uint32_t b = t; b <= SGB_BUCKETS; b += kSgbSortBlock) {
    goff[b] = off[b];
    if (b < SGB_BUCKETS) cnt[b] = off[b];  // scatter cursors
  }
  __syncthreads();
  uint32_t* ent = B.sgb_ent + (size_t)m * SGB_K * g;
  for (uint32_t li = t; li < n; li += kSgbSortBlock) {
#pragma unroll 1
    for (uint32_t k = 0; k < SGB_K; ++k) {
      const int32_t d = dig[li * SGB_K + k];
      if (!d) continue;
      const uint32_t pos = atomicAdd(&cnt[k * SGB_V + (uint32_t)(d < 0 ? -d : d) - 1], 1u);
      ent[pos] = (li << 1) | (d < 0 ? 1u : 0u);
    }
  }
}

// one lane pair per (group, bucket, slice)
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_sgb_bucket(DevBatch B, uint32_t n_sg) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // both lanes of a pair take the same branches
  const uint32_t S = B.sgb_split, m = B.sgb_m;
  if (w >= n_sg * SGB_BUCKETS * S) return;
  const uint32_t g = w / (SGB_BUCKETS * S), b = (w / S) % SGB_BUCKETS, sl = w % S;
  const uint32_t* goff = B.sgb_off + (size_t)(SGB_BUCKETS + 1) * g;
  const uint32_t o0 = goff[b], n = goff[b + 1] - o0;
  const uint32_t e0 = o0 + (n * sl) / S, e1 = o0 + (n * (sl + 1)) / S;
  const uint32_t* ent = B.sgb_ent + (size_t)m * SGB_K * g;
  const G2A* sig = B.sig_aff + (size_t)m * g;
  Jac<Fp2x> acc = jac_inf<Fp2x>();
#pragma unroll 1
  for (uint32_t e = e0; e < e1; ++e) {
    const uint32_t v = ent[e];
    Aff<Fp2x> p = px_load(sig[v >> 1]);
    p.y = f_reduce(p.y);  // decoded coordinates may be up to 16p (a negated root)
    if (v & 1u) p.y = f_reduce(f_neg(p.y));
    acc = jac_add_aff_in(acc, p);
  }
  px_store(B.sgb_part[w], acc);
}

// one lane pair per (group, bucket): the bucket's SGB_SPLIT slice sums into
// its first slice, so the running sums below are 2 x SGB_V additions deep
// instead of (SGB_SPLIT + 1) x SGB_V (a latency-bound kernel: few waves,
// each one serial chain).  The additions skip the doubling case (bls_pair.h
// jac_add_x: fewer live values than the complete formulas): two equal
// partial sums -- which random digits make negligible -- fail the group,
// whose members are then tested one by one.
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_sgb_fold(DevBatch B, uint32_t n_sg) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // both lanes of a pair take the same branches
  if (w >= n_sg * SGB_BUCKETS) return;
  const uint32_t S = B.sgb_split;
  G2J* part = B.sgb_part + (size_t)w * S;
  Jac<Fp2x> acc = px_load(part[0]);
  bool exc = false;
#pragma unroll 1
  for (uint32_t sl = 1; sl < S; ++sl) acc = jac_add_x(acc, px_load(part[sl]), exc);
  if (pair_all(!exc)) px_store(part[0], acc);
  else if (pair_par() == 0) B.sgb_bad[w / SGB_BUCKETS] = 1u;
}

// one lane pair per (group, combination): Q_k = sum_v v B_v by running sums
// from v = 6 down over the folded buckets, stored over the combination's
// first bucket (only this pair reads those buckets)
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_sgb_combine(DevBatch B, uint32_t n_sg) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // both lanes of a pair take the same branches
  if (w >= n_sg * SGB_K) return;
  const uint32_t g = w / SGB_K, k = w % SGB_K, S = B.sgb_split;
  G2J* part = B.sgb_part + ((size_t)SGB_BUCKETS * g + (size_t)SGB_V * k) * S;
  Jac<Fp2x> run = jac_inf<Fp2x>(), q = run;
  bool exc = false;
#pragma unroll 1
  for (int v = (int)SGB_V; v >= 1; --v) {
    run = jac_add_x(run, px_load(part[(size_t)(v - 1) * S]), exc);
    q = jac_add_x(q, run, exc);
  }
  if (pair_all(!exc)) px_store(part[0], q);
  else if (pair_par() == 0) B.sgb_bad[g] = 1u;
}

// one lane pair per (group, combination): psi(Q) == [x] Q; a failure (or the
// doubling case in the [|x|] chain, which only points of tiny order reach)
// fails the group
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_sgb_test(DevBatch B, uint32_t n_sg) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (w >= n_sg * SGB_K) return;
  const uint32_t g = w / SGB_K, k = w % SGB_K;
  const G2J& slot = B.sgb_part[((size_t)SGB_BUCKETS * g + (size_t)SGB_V * k) * B.sgb_split];
  bool ok = true;
  if (!jac_is_inf(px_load(slot))) {
    // [|x|] Q with Q re-read from its slot where it is added (held across the
    // doublings it went through scratch every step)
    bool exc = false;
    Jac<Fp2x> m = px_load(slot);
#pragma unroll 1
    for (int i = 62; i >= 0; --i) {
      m = jac_dbl_lo(m);
      if ((X_ABS >> i) & 1) {
        __asm__ __volatile__("" ::: "memory");
        m = jac_add_x(m, px_load(slot), exc);
      }
    }  // psi(Q) == [x] Q == -m
    if (exc || jac_is_inf(m)) {
      ok = false;
    } else {
      __asm__ __volatile__("" ::: "memory");
      const Jac<Fp2x> ps = g2_psi_g(px_load(slot));
      const Fp2x z1 = f_sqr(ps.Z), z2 = f_sqr(m.Z);
      ok = f_eq(f_mul(ps.X, z2), f_mul(m.X, z1)) &&
           f_eq(f_mul(f_mul(ps.Y, m.Z), z2), f_reduce(f_neg(f_mul(f_mul(m.Y, ps.Z), z1))));
    }
  }
  if (!ok && pair_par() == 0) B.sgb_bad[g] = 1u;
}

void launch_subgroup_batch(const DevBatch& B, hipStream_t st) {
  if (!B.sgb) return;
  const uint32_t n_sg = sgb_groups(B.n_partials, B.sgb_m);
  if (!n_sg) return;
  TBG_KLAUNCH(k_sgb_sort, dim3(n_sg), dim3(kSgbSortBlock), st, B);
  TBG_KLAUNCH(k_sgb_bucket, grid_for(2 * n_sg * SGB_BUCKETS * B.sgb_split), dim3(kBlock), st, B, n_sg);
  if (B.sgb_split > 1) TBG_KLAUNCH(k_sgb_fold, grid_for(2 * n_sg * SGB_BUCKETS), dim3(kBlock), st, B, n_sg);
  TBG_KLAUNCH(k_sgb_combine, grid_for(2 * n_sg * SGB_K), dim3(kBlock), st, B, n_sg);
  TBG_KLAUNCH(k_sgb_test, grid_for(2 * n_sg * SGB_K), dim3(kBlock), st, B, n_sg);
}

}  // namespace tbg
