// Threshold recombination (CombineSignatures, tss.go:142-149 / :181): Lagrange
// coefficients, G2 combination, affine conversion and 96-byte compression.
#include "tbls_launch.h"
#include "bls_tss.h"
#include "bls_batchinv.h"
#include "bls_pair.h"

namespace tbg {

// The speculative pass (SPEC: the candidates taken as valid, run as soon as
// they are final while level 0 is on) and the regular pass after the checks,
// which returns at once after a level-0 pass and otherwise aggregates every
// duty again.  With TBG_SPEC_ALWAYS (tbls_launch.h; measured slower) every
// VERIFY_AGGREGATE chain speculates and the regular pass redoes only the
// duties whose participant set the checks changed (spec_redo): a duty none
// of whose partials turned out INVALID keeps the speculative aggregate.
__device__ __forceinline__ bool spec_skip(const DevBatch& B, bool spec) {
  if (spec) return TBG_SPEC_ALWAYS ? false : B.counters[CNT_L0_BAD] != 0;
  return B.op == TBG_OP_VERIFY_AGGREGATE && B.counters[CNT_L0_OK] != 0;
}
// (an ERR_PUBKEY mark made after the speculative pass -- the group levels'
// k_rlc_partial2 -- changes the set too)
__device__ __forceinline__ bool spec_redo(const DevBatch& B, uint32_t d) {
  if (!TBG_SPEC_ALWAYS || B.op != TBG_OP_VERIFY_AGGREGATE) return true;
  for (uint32_t j = B.duty_first[d]; j < B.duty_first[d + 1]; ++j) {
    const int32_t st = B.partial_status[j];
    if (st == TBG_PS_INVALID || st == TBG_PS_ERR_PUBKEY) return true;
  }
  return false;
}

template <bool SPEC>
__global__ void TBG_LAUNCH k_lagrange(DevBatch B) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (spec_skip(B, SPEC)) return;
  if (i == 0) B.counters[CNT_AGG] = 0;  // (k_aggregate appends after this grid)
  if (i >= B.n_partials) return;
  if (!SPEC && !spec_redo(B, B.partial_duty[i])) return;  // the speculative coefficients stand
  uint32_t* w = B.lam + 8ull * i;
  for (int j = 0; j < 8; ++j) w[j] = 0;
  if (!participates<SPEC>(B.op, B.partial_status[i])) return;
  uint32_t d = B.partial_duty[i];
  uint32_t first = B.duty_first[d], last = B.duty_first[d + 1];
  uint8_t ids[256];
  int k = 0, me = -1;
  for (uint32_t j = first; j < last; ++j) {
    if (!participates<SPEC>(B.op, B.partial_status[j])) continue;
    if (j == i) me = k;
    ids[k++] = B.identifiers[j];
  }
  uint32_t lw[8];
  if (!lagrange_encode(ids, k, me, lw)) return;  // duplicate ids: duty kernel reports it
  for (int j = 0; j < 8; ++j) w[j] = lw[j];
}

// 96-byte compressed encoding of an affine point straight into the output
// as 24 big-endian-packed words (the byte image of g2_compress, written with
// word stores instead of a 96-byte stack array and byte stores).
__device__ __forceinline__ void agg_store_compressed(const DevBatch& B, uint32_t d, const G2A& a) {
  const Fp x0 = fp_from_mont(a.x.c0), x1 = fp_from_mont(a.x.c1);
  const uint32_t flags = 0x80u | (fp2_lex_largest(a.y) ? 0x20u : 0u);
  uint32_t* out = (uint32_t*)(B.agg + 96ull * d);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const Fp& x = h == 0 ? x1 : x0;
#pragma unroll
    for (int w = 0; w < 12; ++w) {
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // byte 4w + j of this half: bits 8 (47 - 4w - j)
        const int bit = 8 * (47 - 4 * w - j);
        const int li = bit / 28, off = bit % 28;
        uint32_t b = x.l[li] >> off;
        if (off > 20 && li + 1 < NL) b |= x.l[li + 1] << (28 - off);
        v |= (b & 0xffu) << (8 * j);  // little-endian word of big-endian bytes
      }
      if (h == 0 && w == 0) v |= flags;
      out[12 * h + w] = v;
    }
  }
}
__device__ __forceinline__ void agg_store_zero(const DevBatch& B, uint32_t d) {
  uint32_t* out = (uint32_t*)(B.agg + 96ull * d);
#pragma unroll
  for (int w = 0; w < 24; ++w) out[w] = 0;
}

// Affine conversion, compression and status of a finished sum.
__device__ void agg_emit(const DevBatch& B, uint32_t d, const G2J& acc) {
  G2A a;
  if (!jac_to_aff(acc, a)) {
    agg_store_zero(B, d);
    B.duty_status[d] = TBG_DS_AGG_IDENTITY;
    return;
  }
  agg_store_compressed(B, d, a);
  B.duty_status[d] = TBG_DS_OK;
}

constexpr uint32_t AGG_EXC = 0x80000000u;  // agg_list flag: the [1/D] ladder met the doubling case
constexpr uint32_t AGG_REF = 0x40000000u;  // agg_list flag: the whole combination on the reference path

// A duty's aggregation status before any curve work (kryptology's checks in
// CombineSignatures' order; reference tbls/tss.go:142-149, :181): TBG_DS_OK
// when a combination is due.  Lane `writer` zeroes the output first.
// pmask: the participants among the first 32 partials; fast: the integer
// coefficient form of at most 32 partials (combine_int_pair) applies.
template <bool SPEC>
__device__ int32_t agg_status(const DevBatch& B, uint32_t d, bool writer, uint32_t& pmask, bool& fast) {
  pmask = 0;
  fast = false;
  if (writer) agg_store_zero(B, d);
  const uint32_t first = B.duty_first[d], last = B.duty_first[d + 1];
  const uint32_t n = last - first;
  if (B.op == TBG_OP_VERIFY) return TBG_DS_NOT_AGGREGATED;
  int k = 0;
  bool decode_err = false, identity = false;
  for (uint32_t j = first; j < last; ++j) {
    int32_t st = B.partial_status[j];
    if (participates<SPEC>(B.op, st)) ++k;
    if (st == TBG_PS_ERR_IDENTITY) identity = true;
    else if (st < 0 && st != TBG_PS_ERR_PUBKEY) decode_err = true;
  }
  if (B.op == TBG_OP_VERIFY_AGGREGATE) {
    uint32_t t = B.duty_threshold[d];
    if (n < t) return TBG_DS_INSUFFICIENT;
    if ((uint32_t)k < t) return TBG_DS_INSUFFICIENT_VALID;
  } else {
    if (decode_err) return TBG_DS_DECODE;
    if (identity) return TBG_DS_AGG_IDENTITY;
  }
  if (k < 2) return TBG_DS_AGG_TOO_FEW;
  // duplicate identifiers among participants
  for (uint32_t a = first; a < last; ++a) {
    if (!participates<SPEC>(B.op, B.partial_status[a])) continue;
    for (uint32_t b = a + 1; b < last; ++b) {
      if (participates<SPEC>(B.op, B.partial_status[b]) && B.identifiers[a] == B.identifiers[b])
        return TBG_DS_AGG_DUPLICATE_ID;
    }
  }
  for (uint32_t j = first; j < last && j - first < 32; ++j)
    if (participates<SPEC>(B.op, B.partial_status[j])) pmask |= 1u << (j - first);
  fast = n <= 32 && (B.lam[8ull * (first + (uint32_t)__builtin_ctz(pmask)) + 7] & LAM_INT_FLAG);
  return TBG_DS_OK;
}

// The integer-form combination sum_j N_j P_j on a lane pair (bls_pair.h: one
// Fp2 component per lane): double-and-add over the few bits of |N_j|
// (3-of-4: 2 bits) with the branch-free group law; a doubling case sets exc
// (the duty then takes the reference path).
template <bool SPEC>
__device__ __forceinline__ Jac<Fp2x> combine_int_pair(const DevBatch& B, uint32_t first, uint32_t n, uint32_t pmask,
                                                     uint64_t& D, bool& exc) {
  int nbits = 0;
  for (uint32_t j = 0; j < n; ++j) {
    if (!((pmask >> j) & 1u)) continue;
    const uint32_t* w = B.lam + 8ull * (first + j);
    const int b = bitlen_u64((uint64_t)w[0] | ((uint64_t)w[1] << 32));
    nbits = nbits > b ? nbits : b;
  }
  Jac<Fp2x> acc = jac_inf<Fp2x>();
  for (int bit = nbits - 1; bit >= 0; --bit) {
    acc = jac_dbl_lo(acc);
    for (uint32_t j = 0; j < n; ++j) {
      if (!((pmask >> j) & 1u)) continue;
      const uint32_t* w = B.lam + 8ull * (first + j);
      const uint64_t mag = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
      if (!((mag >> bit) & 1)) continue;
      Aff<Fp2x> p = px_load(B.sig_aff[first + j]);
      if (w[7] & 1) p.y = f_reduce(f_neg(p.y));
      acc = jac_add_aff_x(acc, p, exc);
    }
  }
  const uint32_t* w0 = B.lam + 8ull * (first + (uint32_t)__builtin_ctz(pmask));
  D = (uint64_t)w0[2] | ((uint64_t)w0[3] << 32);
  return acc;
}

// The reference form of one duty's aggregation (single lane, any coefficient
// form, [1/D] inline): for the duties the pair kernels hand over.
template <bool SPEC>
__device__ void agg_reference(const DevBatch& B, uint32_t d) {
  uint32_t pmask;
  bool fast;
  const int32_t st = agg_status<SPEC>(B, d, true, pmask, fast);
  if (st != TBG_DS_OK) {
    B.duty_status[d] = st;
    return;
  }
  const uint32_t first = B.duty_first[d], n = B.duty_first[d + 1] - first;
  uint8_t mask[256];
  for (uint32_t j = 0; j < n; ++j) mask[j] = participates<SPEC>(B.op, B.partial_status[first + j]) ? 1 : 0;
  uint64_t D = 1;
  G2J acc = tss_combine(B.sig_aff + first, B.lam + 8ull * first, mask, (int)n, &D);
  if (D > 1) acc = tss_div_den(acc, D);
  agg_emit(B, d, acc);
}

// One lane PAIR per duty: the status checks, the integer-form combination in
// pair form (two waves per SIMD; the single-lane kernel held 766 registers at
// one wave), then the affine conversion with the Fp norms' inversion batched
// over the workgroup and the 96-byte compression.  D > 1 sums go to
// k_aggregate_finish; other coefficient forms and doubling cases to the
// reference path (k_aggregate_exc).
template <bool SPEC>
__global__ void __launch_bounds__(BINV_BLOCK, TBG_PAIR_WAVES) k_aggregate(DevBatch B) {
  if (spec_skip(B, SPEC)) return;  // (grid-uniform)
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, d = t >> 1;
  const bool lead = pair_par() == 0;
  // (a duty the regular pass leaves keeps the speculative output; it still
  // takes part in the workgroup's batched inversion below)
  const bool in = d < B.n_duties && (SPEC || spec_redo(B, d));
  uint32_t pmask = 0;
  bool fast = false;
  const int32_t st = in ? agg_status<SPEC>(B, d, lead, pmask, fast) : TBG_DS_OK;
  bool want = in && st == TBG_DS_OK;
  if (want && !fast) {
    if (lead) B.agg_list[atomicAdd(&B.counters[CNT_AGG], 1u)] = d | AGG_REF;
    want = false;
  }
  Jac<Fp2x> acc = jac_inf<Fp2x>();
  if (want) {
    uint64_t D = 1;
    bool exc = false;
    const uint32_t first = B.duty_first[d];
    acc = combine_int_pair<SPEC>(B, first, B.duty_first[d + 1] - first, pmask, D, exc);
    if (exc || D > 1) {
      if (!exc) px_store(B.agg_acc[d], acc);
      if (lead) B.agg_list[atomicAdd(&B.counters[CNT_AGG], 1u)] = exc ? (d | AGG_REF) : d;
      want = false;
    }
  }
  const bool present = want && !jac_is_inf(acc);
  const Fp Zp = pair_xch(acc.Z.v);
  const Fp ni = block_batch_inv<BINV_WAVES>(fp_mul2(acc.Z.v, acc.Z.v, Zp, Zp), present);  // every thread
  if (!in) return;
  if (st != TBG_DS_OK) {
    if (lead) B.duty_status[d] = st;
    return;
  }
  if (!want) return;  // k_aggregate_finish / k_aggregate_exc set it
  if (!present) {
    if (lead) B.duty_status[d] = TBG_DS_AGG_IDENTITY;
    return;
  }
  const Fp2x zi = f_mulfp(px_conj(acc.Z), ni);  // 1 / Z = conj(Z) / N(Z)
  const Fp2x zi2 = f_sqr(zi);
  const G2A a = {px_gather(f_mul(acc.X, zi2)), px_gather(f_mul(acc.Y, f_mul(zi2, zi)))};
  if (lead) {
    agg_store_compressed(B, d, a);
    B.duty_status[d] = TBG_DS_OK;
  }
}

// this lane's component of the same pair-form point on lane ^ m
__device__ __forceinline__ Jac<Fp2x> shfl_xor_px(const Jac<Fp2x>& a, int m) {
  Jac<Fp2x> r;
  const Fp* src[3] = {&a.X.v, &a.Y.v, &a.Z.v};
  Fp* dst[3] = {&r.X.v, &r.Y.v, &r.Z.v};
  for (int k = 0; k < 3; ++k)
    for (int j = 0; j < NL; ++j) dst[k]->l[j] = __shfl_xor(src[k]->l[j], m, 8);
  return r;
}

// [1/D] acc as the 4-way base-|x| MSM of bls_tss.h: EIGHT lanes per listed
// duty, digit q = (lane >> 1) & 3 on a lane pair (bls_pair.h: each lane holds
// one component of every Fp2, so the G2 loop fits two waves per SIMD -- the
// single-lane form needed 768 registers and spilled 454), 64 doublings per
// pair, summed over the four pairs.
template <bool SPEC>
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_aggregate_finish(DevBatch B) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t k = t >> 3;
  const int q = (int)((t >> 1) & 3);
  if (spec_skip(B, SPEC)) return;
  if (k >= B.counters[CNT_AGG] || (B.agg_list[k] & AGG_REF)) return;  // 8-lane uniform
  const uint32_t d = B.agg_list[k];
  uint32_t first = B.duty_first[d], last = B.duty_first[d + 1];
  uint32_t j = first;
  while (j < last && !participates<SPEC>(B.op, B.partial_status[j])) ++j;
  const uint32_t* w = B.lam + 8ull * j;  // listed duties have a participant (k >= 2)
  uint64_t D = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  uint64_t dg[4];
  inv_den_digits(D, dg);
  const uint64_t e = q == 0 ? dg[0] : q == 1 ? dg[1] : q == 2 ? dg[2] : dg[3];
  const Jac<Fp2x> p = px_load(base_x_point(B.agg_acc[d], q));
  // additions without the doubling branch (bls_pair.h jac_add_x): a case that
  // needs it (probability ~2^-250 per step) sets `exc` and the duty is
  // finished on the single-lane reference path instead
  bool exc = false;
  Jac<Fp2x> acc = jac_inf<Fp2x>();
  for (int b = 63; b >= 0; --b) {
    acc = jac_dbl_lo(acc);
    if ((e >> b) & 1) acc = jac_add_x(acc, p, exc);
  }
  acc = jac_add_x(acc, shfl_xor_px(acc, 2), exc);
  acc = jac_add_x(acc, shfl_xor_px(acc, 4), exc);
  exc = __any(exc);  // (wave-wide: rare; the 8-lane group decides together)
  if (q != 0) return;
  if (exc) {
    if (pair_par() == 0) B.agg_list[k] = d | AGG_EXC;  // k_aggregate_exc finishes it
    return;
  }
  const G2J full = {px_gather(acc.X), px_gather(acc.Y), px_gather(acc.Z)};
  if (pair_par() == 0) agg_emit(B, d, full);
}

// The listed duties whose pair-form ladder met the doubling case: the
// single-lane reference form (one thread per list entry).
template <bool SPEC>
__global__ void TBG_LAUNCH_N(2) k_aggregate_exc(DevBatch B) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (spec_skip(B, SPEC) || k >= B.counters[CNT_AGG]) return;
  const uint32_t entry = B.agg_list[k];
  if (entry & AGG_REF) {
    agg_reference<SPEC>(B, entry & ~AGG_REF);
    return;
  }
  if (!(entry & AGG_EXC)) return;
  const uint32_t d = entry & ~AGG_EXC;
  uint32_t j = B.duty_first[d];
  while (j < B.duty_first[d + 1] && !participates<SPEC>(B.op, B.partial_status[j])) ++j;
  const uint32_t* w = B.lam + 8ull * j;
  agg_emit(B, d, tss_div_den(B.agg_acc[d], (uint64_t)w[2] | ((uint64_t)w[3] << 32)));
}

void launch_lagrange(const DevBatch& B, hipStream_t st, bool spec) {
  if (!B.n_partials) return;
  if (spec) TBG_KLAUNCH(k_lagrange<true>, grid_for(B.n_partials), dim3(kBlock), st, B);
  else TBG_KLAUNCH(k_lagrange<false>, grid_for(B.n_partials), dim3(kBlock), st, B);
}
void launch_aggregate(const DevBatch& B, hipStream_t st, bool spec) {
  if (!B.n_duties) return;
  const dim3 grid((2 * B.n_duties + BINV_BLOCK - 1) / BINV_BLOCK);  // a lane pair per duty
  if (spec) TBG_KLAUNCH(k_aggregate<true>, grid, dim3(BINV_BLOCK), st, B);
  else TBG_KLAUNCH(k_aggregate<false>, grid, dim3(BINV_BLOCK), st, B);
}
void launch_aggregate_finish(const DevBatch& B, hipStream_t st, bool spec) {
  if (!B.n_duties) return;
  if (spec) {
    TBG_KLAUNCH(k_aggregate_finish<true>, grid_for(8 * B.n_duties), dim3(kBlock), st, B);
    TBG_KLAUNCH(k_aggregate_exc<true>, grid_for(B.n_duties), dim3(kBlock), st, B);
  } else {
    TBG_KLAUNCH(k_aggregate_finish<false>, grid_for(8 * B.n_duties), dim3(kBlock), st, B);
    TBG_KLAUNCH(k_aggregate_exc<false>, grid_for(B.n_duties), dim3(kBlock), st, B);
  }
}

}  // namespace tbg
