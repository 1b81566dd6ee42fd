// Level 1's group sums S_g = sum_i r_i s_i as one bucket MSM per group
// (VERDICT r05 item 2), in place of a 64-bit G2 scalar multiplication per
// partial (k_rlc_partial2: 15 doublings, 31 additions and a batched field
// inversion each).  Reference: the per-partial CoreVerify calls of
// tbls.Verify / VerifyAndAggregate (tbls/tss.go:163-197), batched per
// k_rlc.hip's header; every verdict stays the exact per-item one.
//
// r_i = sum_k a_k x^k with 16-bit signed-binary digits a_k (bls_rlc.h), and
// [r_i] s_i = sum_k a_k psi^k(s_i) on G2.  Each a_k is four 4-bit windows
// v_w = 2 nibble - 15 (odd, |v| <= 15), so
//   S_g = sum_w 16^w sum_b (2b + 1) B_(w, b),
//   B_(w, b) = sum of +-psi^k(s_i) over the (i, k) whose window w has |v| = 2b + 1
// (bls_msm.h gm_bucket / gm_reference): 16 mixed additions per partial into
// the group's 32 buckets, 4 x 15 running-sum additions and 12 doublings per
// group -- ~2x fewer group operations than the per-partial products at a
// 3-of-4 group of 8 duties, more at larger groups.
//
//   k_rlc_g1      one lane per partial: key marks, the group lead, [r_i] pk_i (no level 0)
//   k_gm_sort     one wave per group: the group's 16 n entries sorted into its 32 buckets
//   k_gm_bucket   one lane PAIR per (group, bucket): the bucket's sum
//   k_gm_window   one lane PAIR per (group, window): T_w = sum_b (2b + 1) B_(w, b)
//   k_gm_combine  one lane PAIR per group: S_g = sum_w 16^w T_w, affine, grp_state
// After the group checks (k_rlc_group_final), k_gm_failed_list lists the
// candidates of FAILED groups; k_rlc_partial2 (list mode) forms their r_i s_i
// and k_rlc_duty_sum<DSUM_FALLBACK_S> their S_d, which the chunk / duty /
// partial levels use as before -- at 1 % invalid partials ~12 % of the groups.
//
// Every kernel returns at once when level 0 accepted the batch (after a
// level-0 pass they are launched over nothing), and runs a grid-stride loop
// over a capped grid, so the empty launches of a clean batch cost few waves.
#define TBG_ADD_DBL_INLINE 1
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernels in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_msm.h"
#include "bls_pair.h"

namespace tbg {

constexpr uint32_t kGmSortBlock = 64;   // one wave per group
constexpr uint32_t kGmMaxBlocks = 2048;  // two waves per SIMD of the grid-stride kernels

inline dim3 gm_grid(uint64_t threads, uint32_t block) {
  const uint64_t b = (threads + block - 1) / block;
  return dim3((uint32_t)(b < kGmMaxBlocks ? (b ? b : 1) : kGmMaxBlocks));
}

__device__ __forceinline__ uint32_t gm_groups(const DevBatch& B) { return (B.n_duties + B.rlc_group - 1) / B.rlc_group; }

// partial i enters its group's S: a candidate of a duty the P side combined
__device__ __forceinline__ bool gm_member(const DevBatch& B, uint32_t i) {
  return B.partial_status[i] == TBG_PS_NOT_VERIFIED && B.dv_state[B.partial_duty[i]] == RLC_COMBINED;
}

// Level 1's G1 side without level 0 (one lane per partial): unusable keys are
// marked ERR_PUBKEY, the group's first usable candidate takes r = 1 (a fixed
// coefficient per duty would let invalid partials of two duties cancel), the
// others [r_i] pk_i from the key's window table.
__global__ void TBG_LAUNCH k_rlc_g1(DevBatch B, const G1A* tab, const G1A* pk_aff, const int32_t* pk_status,
                                   uint32_t n_pk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B.n_partials || B.partial_status[i] != TBG_PS_NOT_VERIFIED) return;
  const uint32_t pid = B.pubkey_ids[i];
  if (pid >= n_pk || pk_status[pid] != DEC_OK) {
    B.partial_status[i] = TBG_PS_ERR_PUBKEY;
    return;
  }
  // the lead: no usable candidate before i in the group (the usability test
  // reads the key table, so it holds whichever marks are already made)
  const uint32_t d = B.partial_duty[i];
  const uint32_t d0 = (d / B.rlc_group) * B.rlc_group;
  bool lead = true;
  for (uint32_t j = B.duty_first[d0]; j < i && lead; ++j) {
    const int32_t st = B.partial_status[j];
    const uint32_t q = B.pubkey_ids[j];
    lead = !((st == TBG_PS_NOT_VERIFIED || st == TBG_PS_ERR_PUBKEY) && q < n_pk && pk_status[q] == DEC_OK);
  }
  if (lead) {
    B.part_p[i] = jac_from_aff(pk_aff[pid]);
    return;
  }
  uint32_t u[4];
  rlc_digits(rlc_scalar(B.rlc_seed, i), u);
  B.part_p[i] = rlc_mul_key(tab + (size_t)PK_TAB * pid, u);
}

// One wave per group (grid-stride): the lead, the 32 bucket sizes, offsets
// and the entries (order within a bucket is immaterial: its sum is a group
// element).  Group g's entries occupy [16 p0, 16 p1) of gm_ent.
__global__ void __launch_bounds__(kGmSortBlock) k_gm_sort(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  __shared__ uint32_t cnt[GM_BUCKETS];
  __shared__ uint32_t lead;
  const uint32_t t = threadIdx.x, G = B.rlc_group, ng = gm_groups(B);
#pragma unroll 1
  for (uint32_t g = blockIdx.x; g < ng; g += gridDim.x) {
    const uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
    const uint32_t p0 = B.duty_first[d0], p1 = B.duty_first[d1];
    if (t < GM_BUCKETS) cnt[t] = 0;
    if (t == 0) lead = 0xFFFFFFFFu;
    if (g == blockIdx.x)  // (the size histogram of k_gm_hist, zeroed before it runs)
      for (uint32_t k = t; k < 256u && blockIdx.x == 0; k += kGmSortBlock) B.gm_hist[k] = 0;
    __syncthreads();
    // level 0 drew every r_i at random (no lead); otherwise the group's first
    // candidate (k_rlc_g1 gave it r = 1 on the key side)
    if (!B.rlc_batch)
      for (uint32_t i = p0 + t; i < p1; i += kGmSortBlock)
        if (B.partial_status[i] == TBG_PS_NOT_VERIFIED) atomicMin(&lead, i);
    __syncthreads();
    const uint32_t ld = lead;
    for (uint32_t i = p0 + t; i < p1; i += kGmSortBlock) {
      if (!gm_member(B, i)) continue;
      if (i == ld) {
        atomicAdd(&cnt[0], 1u);
        continue;
      }
      uint32_t u[4];
      rlc_digits(rlc_scalar(B.rlc_seed, i), u);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k)
#pragma unroll
        for (uint32_t w = 0; w < GM_W; ++w) {
          bool neg;
          atomicAdd(&cnt[gm_bucket(u[k], w, neg)], 1u);
        }
    }
    __syncthreads();
    uint32_t* off = B.gm_off + (size_t)(GM_BUCKETS + 1) * g;
    if (t == 0) {
      uint32_t run = 0;
      for (uint32_t b = 0; b < GM_BUCKETS; ++b) {
        const uint32_t c = cnt[b];
        off[b] = run;
        cnt[b] = run;  // scatter cursors
        run += c;
      }
      off[GM_BUCKETS] = run;
      B.gm_lead[g] = ld;
    }
    __syncthreads();
    uint32_t* ent = B.gm_ent + 16ull * p0;
    for (uint32_t i = p0 + t; i < p1; i += kGmSortBlock) {
      if (!gm_member(B, i)) continue;
      if (i == ld) {
        ent[atomicAdd(&cnt[0], 1u)] = msm_entry(i, 0, false);
        continue;
      }
      uint32_t u[4];
      rlc_digits(rlc_scalar(B.rlc_seed, i), u);
#pragma unroll 1
      for (uint32_t k = 0; k < 4; ++k)
#pragma unroll
        for (uint32_t w = 0; w < GM_W; ++w) {
          bool neg;
          const uint32_t b = gm_bucket(u[k], w, neg);
          ent[atomicAdd(&cnt[b], 1u)] = msm_entry(i, k, neg);
        }
    }
    __syncthreads();
  }
}

// psi^k(s), negated on request, with the Fp2 coordinates split over the pair
__device__ __forceinline__ Aff<Fp2x> gm_point(const G2A& s, uint32_t k, bool neg) {
  Aff<Fp2x> p = px_load(s);
  p.y = f_reduce(p.y);  // decoded coordinates may be up to 16p (a negated root)
  if (k & 1) p = Aff<Fp2x>{f_mulc(f_conj(p.x), PSI_X), f_mulc(f_conj(p.y), PSI_Y)};
  const bool ny = ((k & 2) != 0) != neg;
  if (k & 2) p.x = f_mulfp(p.x, fp_from_const(PSI2_X));
  if (ny) p.y = f_reduce(f_neg(p.y));
  return p;
}

// The buckets in order of decreasing size (a counting sort of their sizes):
// a wave runs as long as its longest bucket, and the 32 buckets of one group
// differ by ~1.5x between the mean and the largest (~16 entries each for a
// 3-of-4 group of 8 duties), so the bucket kernel takes them size-matched.
constexpr uint32_t GM_SIZES = 256;  // size classes (larger buckets share the last)
__global__ void TBG_LAUNCH k_gm_hist(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  __shared__ uint32_t h[GM_SIZES];
  for (uint32_t k = threadIdx.x; k < GM_SIZES; k += blockDim.x) h[k] = 0;
  __syncthreads();
  const uint32_t n = gm_groups(B) * GM_BUCKETS;
  for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
    const uint32_t* off = B.gm_off + (size_t)(GM_BUCKETS + 1) * (x / GM_BUCKETS) + x % GM_BUCKETS;
    atomicAdd(&h[min(off[1] - off[0], GM_SIZES - 1)], 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < GM_SIZES; k += blockDim.x)
    if (h[k]) atomicAdd(&B.gm_hist[k], h[k]);
}
// exclusive scan from the largest size class down: the cursors of the scatter
__global__ void __launch_bounds__(64) k_gm_hist_scan(DevBatch B) {
  if (B.counters[CNT_L0_OK] || threadIdx.x) return;
  uint32_t run = 0;
  for (int k = (int)GM_SIZES - 1; k >= 0; --k) {
    const uint32_t c = B.gm_hist[k];
    B.gm_hist[k] = run;
    run += c;
  }
}
// The scatter: each workgroup takes a contiguous range of buckets, counts
// its size classes in LDS, reserves one range per class with ONE global
// atomic, and places its buckets from LDS cursors (global atomics per bucket
// on the few class cursors serialised: 1.9 ms per 16-batch launch).
__global__ void TBG_LAUNCH k_gm_order(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  __shared__ uint32_t h[GM_SIZES];
  const uint32_t n = gm_groups(B) * GM_BUCKETS;
  const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
  const uint32_t x0 = min(n, blockIdx.x * per), x1 = min(n, x0 + per);
  for (uint32_t k = threadIdx.x; k < GM_SIZES; k += blockDim.x) h[k] = 0;
  __syncthreads();
  auto cls = [&](uint32_t x) {
    const uint32_t* off = B.gm_off + (size_t)(GM_BUCKETS + 1) * (x / GM_BUCKETS) + x % GM_BUCKETS;
    return min(off[1] - off[0], GM_SIZES - 1);
  };
  for (uint32_t x = x0 + threadIdx.x; x < x1; x += blockDim.x) atomicAdd(&h[cls(x)], 1u);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < GM_SIZES; k += blockDim.x)
    if (h[k]) h[k] = atomicAdd(&B.gm_hist[k], h[k]);
  __syncthreads();
  for (uint32_t x = x0 + threadIdx.x; x < x1; x += blockDim.x) B.gm_order[atomicAdd(&h[cls(x)], 1u)] = x;
}

// one lane pair per (group, bucket), grid-stride over the size order
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_gm_bucket(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  const uint32_t n = gm_groups(B) * GM_BUCKETS;
  const uint32_t stride = (gridDim.x * blockDim.x) >> 1;
#pragma unroll 1
  for (uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) >> 1; x < n; x += stride) {  // pair-uniform
    const uint32_t w = B.gm_order[x];
    const uint32_t g = w / GM_BUCKETS, b = w % GM_BUCKETS;
    const uint32_t* off = B.gm_off + (size_t)(GM_BUCKETS + 1) * g;
    const uint32_t* ent = B.gm_ent + 16ull * B.duty_first[g * B.rlc_group];
    const uint32_t e1 = off[b + 1];
    Jac<Fp2x> acc = jac_inf<Fp2x>();
#pragma unroll 1
    for (uint32_t e = off[b]; e < e1; ++e) {
      const uint32_t v = ent[e];
      acc = jac_add_aff_in(acc, gm_point(B.sig_aff[v >> 3], (v >> 1) & 3u, (v & 1u) != 0));
    }
    px_store(B.gm_part[w], acc);
  }
}

// one lane pair per (group, window): T_w = sum_b (2b + 1) B_b = 2 sum_b b B_b
// + sum_b B_b by running sums from b = 7 down, stored over bucket (w, 0)
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_gm_window(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  const uint32_t n = gm_groups(B) * GM_W;
  const uint32_t stride = (gridDim.x * blockDim.x) >> 1;
#pragma unroll 1
  for (uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) >> 1; x < n; x += stride) {  // pair-uniform
    G2J* part = B.gm_part + (size_t)GM_V * x;  // (group, window) x's eight buckets
    Jac<Fp2x> run = jac_inf<Fp2x>(), acc = run;
#pragma unroll 1
    for (int b = (int)GM_V - 1; b >= 1; --b) {
      run = jac_add_in<Fp2x, true>(run, px_load(part[b]));
      acc = jac_add_in<Fp2x, true>(acc, run);
    }
    run = jac_add_in<Fp2x, true>(run, px_load(part[0]));
    px_store(part[0], jac_add_in<Fp2x, true>(jac_dbl_in(acc), run));
  }
}

// one lane pair per group: S_g = sum_w 16^w T_w, then what k_rlc_group_lines
// does with it: no combined duty -> GRP_EMPTY, S_g = 0 -> GRP_FAIL (its
// chunks decide), else S_g affine for its lines (k_lines_fold<FOLD_GROUPS>)
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_gm_combine(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  const uint32_t ng = gm_groups(B), G = B.rlc_group;
  const uint32_t stride = (gridDim.x * blockDim.x) >> 1;
#pragma unroll 1
  for (uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 1; g < ng; g += stride) {  // pair-uniform
    const uint32_t d0 = g * G, d1 = min(d0 + G, B.n_duties);
    uint32_t n = 0;
    for (uint32_t d = d0; d < d1; ++d) n += B.dv_state[d] == RLC_COMBINED ? 1u : 0u;
    if (n == 0) {
      if (pair_par() == 0) B.grp_state[g] = GRP_EMPTY;
      continue;
    }
    const G2J* part = B.gm_part + (size_t)GM_BUCKETS * g;
    Jac<Fp2x> S = px_load(part[GM_V * (GM_W - 1)]);
#pragma unroll 1
    for (int w = (int)GM_W - 2; w >= 0; --w) {
      S = jac_dbl_in(jac_dbl_in(jac_dbl_in(jac_dbl_in(S))));
      S = jac_add_in<Fp2x, true>(S, px_load(part[GM_V * w]));
    }
    if (jac_is_inf(S)) {
      if (pair_par() == 0) B.grp_state[g] = GRP_FAIL;
      continue;
    }
    const Fp2x zi = f_inv(S.Z);
    const Fp2x zi2 = f_sqr(zi);
    px_store(B.pend_pts[g], Aff<Fp2x>{f_mul(S.X, zi2), f_mul(S.Y, f_mul(zi2, zi))});
    if (pair_par() == 0) B.grp_state[g] = GRP_LINES;
  }
}

// After the group checks: the candidates of failed groups (level 1g's too)
// whose duties were combined -- the only partials whose r_i s_i the chunk,
// duty and partial levels read.
__global__ void TBG_LAUNCH k_gm_failed_list(DevBatch B) {
  if (B.counters[CNT_L0_OK]) return;
  const uint32_t stride = gridDim.x * blockDim.x;
#pragma unroll 1
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < B.n_partials; i += stride) {
    if (!gm_member(B, i)) continue;
    const int32_t gs = B.grp_state[B.partial_duty[i] / B.rlc_group];
    if (gs == GRP_FAIL || gs == GRP_GID) B.gm_list[atomicAdd(&B.counters[CNT_LAZY], 1u)] = i;
  }
}

void launch_rlc_g1(const DevBatch& B, const G1A* pk_tab, const G1A* pk_aff, const int32_t* pk_status, uint32_t n_pk,
                   hipStream_t st) {
  if (B.n_partials) TBG_KLAUNCH(k_rlc_g1, grid_for(B.n_partials), dim3(kBlock), st, B, pk_tab, pk_aff, pk_status, n_pk);
}

void launch_gm_group_s(const DevBatch& B, hipStream_t st) {
  const uint32_t ng = (B.n_duties + B.rlc_group - 1) / B.rlc_group;
  if (!ng) return;
  TBG_KLAUNCH(k_gm_sort, gm_grid(64ull * ng, kGmSortBlock), dim3(kGmSortBlock), st, B);
  TBG_KLAUNCH(k_gm_hist, gm_grid((uint64_t)ng * GM_BUCKETS, kBlock), dim3(kBlock), st, B);
  TBG_KLAUNCH(k_gm_hist_scan, dim3(1), dim3(64), st, B);
  TBG_KLAUNCH(k_gm_order, gm_grid((uint64_t)ng * GM_BUCKETS, kBlock), dim3(kBlock), st, B);
  TBG_KLAUNCH(k_gm_bucket, gm_grid(2ull * ng * GM_BUCKETS, kBlock), dim3(kBlock), st, B);
  TBG_KLAUNCH(k_gm_window, gm_grid(2ull * ng * GM_W, kBlock), dim3(kBlock), st, B);
  TBG_KLAUNCH(k_gm_combine, gm_grid(2ull * ng, kBlock), dim3(kBlock), st, B);
}

void launch_gm_failed_partials(const DevBatch& B, const G1A* pk_aff, hipStream_t st) {
  if (!B.n_partials) return;
  TBG_KLAUNCH(k_gm_failed_list, gm_grid(B.n_partials, kBlock), dim3(kBlock), st, B);
  launch_rlc_partials_list(B, pk_aff, st);
}

}  // namespace tbg
