// BLS12-381 base field Fp for gfx950: 14 limbs of 28 bits in 32-bit VGPRs,
// Montgomery form with R = 2^392.
//
// Why radix 2^28: a 28x28-bit product is 56 bits, so a whole Montgomery
// column (14 a*b products + 14 m*p products + carry) fits in one 64-bit
// accumulator and every partial product is a single v_mad_u64_u32 with no
// carry instructions (measured 64 G Fp-mul/s on MI355X vs 45 G for a 12x32
// CIOS with addc chains, tools/microbench/fp_mul_bench.hip).
//
// Value-bound conventions (all limbs are always normalised to < 2^28, the
// value is tracked in multiples of p):
//   fp_mul / fp_sqr / fp_mul2   inputs < 32p (one may be < 64p), output < 2p
//   fp_add                      output bound = sum of input bounds
//   fp_sub(a, b)                a + 16p - b, requires b < 16p
//   fp_reduce                   any value < 2^390 -> < 2p
//   fp_canon                    -> canonical [0, p)
// Define TBG_BOUNDS_CHECK in a host build to assert these at run time.
#pragma once
#include <cstdint>
#include "bls_constants.h"

#if defined(__HIP__)
#define TBG_HD __host__ __device__ __forceinline__
// Out-of-line on the device: shared code for the big tower/curve routines
// keeps kernels within the instruction cache and compile times sane.
// Out-of-line device functions.  Calls pass the large point / tower structs
// through the scratch stack, but inlining whole call trees into the kernels
// (-DTBG_INLINE_ALL=1) costs 15+ min of compile time, drops every kernel to
// one wave per SIMD (AGPR spill space) and spills thousands of VGPRs in the
// final exponentiation; and inlining only the point / quad primitives
// (TBG_INLINE_PT=1) must not be combined with an out-of-line caller whose
// loop body then exceeds the branch range: this compiler expands such long
// branches through s[30:31], the caller's return address (a hang on gfx950).
#if defined(TBG_INLINE_ALL) && TBG_INLINE_ALL
#define TBG_NI __host__ __device__ __forceinline__
#else
#define TBG_NI __host__ __device__ __noinline__ inline
#endif
// Point / line / quad primitives: out of line unless TBG_INLINE_PT=1 or
// TBG_INLINE_ALL=1 (see above).
#ifndef TBG_INLINE_PT
#if defined(TBG_INLINE_ALL) && TBG_INLINE_ALL
#define TBG_INLINE_PT 1
#else
#define TBG_INLINE_PT 0
#endif
#endif
#if TBG_INLINE_PT
#define TBG_PT __host__ __device__ __forceinline__
#else
#define TBG_PT __host__ __device__ __noinline__ inline
#endif
#else
#define TBG_HD inline
#define TBG_NI inline
#define TBG_PT inline
#endif

#if defined(TBG_BOUNDS_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
#include <cstdio>
#include <cstdlib>
#define TBG_BOUND(cond, what) do { if (!(cond)) { fprintf(stderr, "bound violated: %s at %s:%d\n", what, __FILE__, __LINE__); abort(); } } while (0)
#else
#define TBG_BOUND(cond, what) do { } while (0)
#endif

// Work accounting (host counting build only): u32 multiply-adds issued by the
// field layer, used to freeze the algorithmic work model (tools/count_work.py).
#if defined(TBG_COUNT_OPS) && !defined(__HIP_DEVICE_COMPILE__)
extern "C" unsigned long long tbg_mad_count;
#define TBG_COUNT(n) (tbg_mad_count += (unsigned long long)(n))
#else
#define TBG_COUNT(n) ((void)0)
#endif

namespace tbg {

struct Fp { uint32_t l[NL]; };

// Limbs: normalised values (every product, reduction and normalised sum)
// have limbs < 2^28.  The LAZY sum / difference (fp_add_l, fp_sub_l) skip the
// carry normalisation (39 of a normalised sum's 53 instructions) and leave
// limbs < 2^31; such a value may feed fp_mul / fp_mul2 / fp_sqr (whose 64-bit
// columns take the larger limbs, checked below), fp_reduce, fp_add_l, the
// first operand of fp_sub(_l), fp_mul_small and limb-wise moves -- never the
// second operand of a subtraction, fp_neg or a store that another kernel
// reads as normalised.
TBG_HD uint32_t fp_max_limb(const Fp& a) {
  uint32_t m = 0;
  for (int i = 0; i < NL; ++i) m = a.l[i] > m ? a.l[i] : m;
  return m;
}

TBG_HD Fp fp_from_const(const uint32_t (&c)[NL]) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = c[i];
  return r;
}
TBG_HD Fp fp_zero() {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = 0;
  return r;
}
TBG_HD Fp fp_one() { return fp_from_const(ONE_M); }

// Approximate value / p from the top limbs (host bound checks only).
TBG_HD double fp_ratio_p(const Fp& a) {
  double v = 0;
  for (int i = NL - 1; i >= NL - 3; --i) v = v * 268435456.0 + (double)a.l[i];
  double p = 0;
  for (int i = NL - 1; i >= NL - 3; --i) p = p * 268435456.0 + (double)P_L[i];
  return v / p;
}

TBG_HD void fp_normalize(Fp& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    a.l[i + 1] += a.l[i] >> 28;
    a.l[i] &= LMASK;
  }
}

TBG_HD Fp fp_add(const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] + b.l[i];
  fp_normalize(r);
  return r;
}

TBG_HD Fp fp_dbl(const Fp& a) { return fp_add(a, a); }

// a + 16p - b (b < 16p). SUB16P_L is 16p with every limb but the top one
// >= 2^28 - 1, so no limb difference goes negative before normalisation.
TBG_HD Fp fp_sub(const Fp& a, const Fp& b) {
  TBG_BOUND(fp_ratio_p(b) <= 16.0, "fp_sub b <= 16p");
  TBG_BOUND(fp_max_limb(b) < (1u << 28), "fp_sub b normalised");
  TBG_BOUND(fp_max_limb(a) < (1u << 31), "fp_sub a limbs < 2^31");
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] + SUB16P_L[i] - b.l[i];
  fp_normalize(r);
  return r;
}

TBG_HD Fp fp_neg(const Fp& a) {
  TBG_BOUND(fp_ratio_p(a) <= 16.0, "fp_neg a <= 16p");
  TBG_BOUND(fp_max_limb(a) < (1u << 28), "fp_neg a normalised");
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = SUB16P_L[i] - a.l[i];
  fp_normalize(r);
  return r;
}

// Lazy a + b and a + 16p - b (b normalised): the limbs are left unnormalised
// (< 2^31, see the note at the top); value bounds as fp_add / fp_sub.
TBG_HD Fp fp_add_l(const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] + b.l[i];
  TBG_BOUND(fp_max_limb(r) < (1u << 31), "fp_add_l limbs < 2^31");
  return r;
}
TBG_HD Fp fp_sub_l(const Fp& a, const Fp& b) {
  TBG_BOUND(fp_ratio_p(b) <= 16.0, "fp_sub_l b <= 16p");
  TBG_BOUND(fp_max_limb(b) < (1u << 28), "fp_sub_l b normalised");
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = a.l[i] + SUB16P_L[i] - b.l[i];
  TBG_BOUND(fp_max_limb(r) < (1u << 31), "fp_sub_l limbs < 2^31");
  return r;
}
// Lazy 16p - a (a normalised): limbs < 2^29, unnormalised -- for a product
// operand only (fp_mul_sum's column check covers it)
TBG_HD Fp fp_neg_l(const Fp& a) {
  TBG_BOUND(fp_ratio_p(a) <= 16.0, "fp_neg_l a <= 16p");
  TBG_BOUND(fp_max_limb(a) < (1u << 28), "fp_neg_l a normalised");
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = SUB16P_L[i] - a.l[i];
  return r;
}
// normalise the limbs of a lazy value (same value)
TBG_HD Fp fp_norm(const Fp& a) {
  Fp r = a;
  fp_normalize(r);
  return r;
}

// a - q p for q = floor(a/p) or floor(a/p) - 1: result in [0, 2p).
// Valid for a < 2^390 with limbs < 2^31 (lazy sums included: the quotient
// estimate ADDS the top limbs, so unpropagated carries still count).
TBG_HD Fp fp_reduce(const Fp& a) {
  TBG_BOUND(a.l[NL - 1] < (1u << 26), "fp_reduce a < 2^390");
  TBG_BOUND(fp_max_limb(a) < (1u << 31), "fp_reduce limbs < 2^31");
  TBG_COUNT(14);
  // top 60 bits: a >> 330  (limb 13 holds bits 364.., limb 12 bits 336.., limb 11 bits 308..)
  uint64_t t = ((uint64_t)a.l[13] << 34) + ((uint64_t)a.l[12] << 6) + (uint64_t)(a.l[11] >> 22);
  double q = (double)t * INV_PT - 1e-9;
  int32_t qi = q < 0.0 ? 0 : (int32_t)q;
  Fp r;
  int64_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    int64_t s = (int64_t)a.l[i] + carry - (int64_t)qi * (int64_t)P_L[i];
    r.l[i] = (uint32_t)s & LMASK;
    carry = s >> 28;  // arithmetic shift
  }
  // the true result is in [0, 2p): the final carry is zero
  return r;
}

// Conditional subtract of p: input < 2p -> [0, p).
TBG_HD Fp fp_csub_p(const Fp& a) {
  Fp d;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)a.l[i] - (int32_t)P_L[i] + borrow;
    d.l[i] = (uint32_t)s & LMASK;
    borrow = s >> 28;
  }
  // borrow == -1 -> a < p, keep a
  bool keep = borrow < 0;
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = keep ? a.l[i] : d.l[i];
  return r;
}

TBG_HD Fp fp_canon(const Fp& a) { return fp_csub_p(fp_reduce(a)); }

// Montgomery product REDC(sum_k a_k * b_k), product scanning, 28-bit limbs.
// Column bound: 14 (K + 1) products of < 2^56 each, so K <= 16 fits 64 bits.
// The a*b products of a column are spread round-robin over four independent
// 64-bit accumulators and the m*p products over two, so consecutive
// v_mad_u64_u32 never depend on each other; only the m_k / carry chain is
// serial from column to column.
#ifndef TBG_ACC_AB
#define TBG_ACC_AB 4  // independent 64-bit accumulators for the a*b products of a column
#endif
#ifndef TBG_ACC_MP
#define TBG_ACC_MP 2  // ... and for the m*p products
#endif
static_assert(TBG_ACC_AB == 1 || TBG_ACC_AB == 2 || TBG_ACC_AB == 4, "TBG_ACC_AB");
static_assert(TBG_ACC_MP == 1 || TBG_ACC_MP == 2, "TBG_ACC_MP");

// TBG_SCHED_FENCE=1 (set per translation unit before the includes): a
// scheduling barrier around every Montgomery product, so the machine
// scheduler does not interleave independent products for ILP -- each product
// already has six independent accumulator chains, and interleaving two of
// them is what pushes the point kernels past 256 VGPRs (two waves per SIMD,
// which hide latency better than the interleaving does).
#if defined(__HIP_DEVICE_COMPILE__) && defined(TBG_SCHED_FENCE) && TBG_SCHED_FENCE
#define TBG_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define TBG_FENCE() ((void)0)
#endif

template <int N>
TBG_HD uint64_t acc_total(const uint64_t (&s)[N]) {
  if constexpr (N == 4) return (s[0] + s[1]) + (s[2] + s[3]);
  else if constexpr (N == 2) return s[0] + s[1];
  else return s[0];
}

// Host checks: the largest column, sum_k a_i b_j over 14 K products, plus
// the 14 m p products and the carry, must fit the 64-bit accumulator.
TBG_HD bool fp_columns_fit(double ab_products) {
  return ab_products + 14.0 * 268435456.0 * 268435456.0 + 68719476736.0 < 18446744073709551616.0;
}

template <int K>
TBG_HD Fp fp_mul_sum(const Fp* const (&a)[K], const Fp* const (&b)[K]) {
  TBG_COUNT(196 * (K + 1));
#if defined(TBG_BOUNDS_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
  {
    double col = 0;
    for (int n = 0; n < K; ++n) col += 14.0 * (double)fp_max_limb(*a[n]) * (double)fp_max_limb(*b[n]);
    TBG_BOUND(fp_columns_fit(col), "fp_mul_sum columns fit 64 bits");
  }
#endif
  TBG_FENCE();
  uint32_t m[NL];
  Fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; ++k) {
    uint64_t s[TBG_ACC_AB] = {};
    uint64_t t[TBG_ACC_MP] = {};
    int c = 0;
    const int lo = k < NL ? 0 : k - NL + 1;
    const int hi = k < NL ? k : NL - 1;
#pragma unroll
    for (int i = lo; i <= hi; ++i) {
#pragma unroll
      for (int n = 0; n < K; ++n) {
        s[c % TBG_ACC_AB] += (uint64_t)a[n]->l[i] * b[n]->l[k - i];
        ++c;
      }
    }
    const int mhi = k < NL ? k - 1 : NL - 1;
#pragma unroll
    for (int i = lo; i <= mhi; ++i) t[i % TBG_ACC_MP] += (uint64_t)m[i] * P_L[k - i];
    uint64_t sum = acc_total(s) + (acc_total(t) + acc);
    if (k < NL) {
      m[k] = ((uint32_t)sum * NINV) & LMASK;
      sum += (uint64_t)m[k] * P_L[0];
    } else {
      r.l[k - NL] = (uint32_t)sum & LMASK;
    }
    acc = sum >> 28;
  }
  r.l[NL - 1] = (uint32_t)acc;
  TBG_FENCE();
  return r;
}

TBG_HD Fp fp_mul(const Fp& a, const Fp& b) {
  TBG_BOUND(fp_ratio_p(a) * fp_ratio_p(b) < 2048.0, "fp_mul a*b < 2^11 p^2");
  const Fp* const A[1] = {&a};
  const Fp* const B[1] = {&b};
  return fp_mul_sum<1>(A, B);
}

// REDC(a*b + c*d)
TBG_HD Fp fp_mul2(const Fp& a, const Fp& b, const Fp& c, const Fp& d) {
  TBG_BOUND(fp_ratio_p(a) * fp_ratio_p(b) + fp_ratio_p(c) * fp_ratio_p(d) < 2048.0, "fp_mul2 bound");
  const Fp* const A[2] = {&a, &c};
  const Fp* const B[2] = {&b, &d};
  return fp_mul_sum<2>(A, B);
}

// Squaring: off-diagonal products once against a doubled copy; accumulators
// split as in fp_mul_sum.
TBG_HD Fp fp_sqr(const Fp& a) {
  TBG_BOUND(fp_ratio_p(a) * fp_ratio_p(a) < 2048.0, "fp_sqr bound");
  TBG_BOUND(fp_max_limb(a) < (1u << 31), "fp_sqr limbs < 2^31");
  TBG_BOUND(fp_columns_fit(8.0 * 2.0 * (double)fp_max_limb(a) * (double)fp_max_limb(a)), "fp_sqr columns fit");
  TBG_COUNT(301);
  TBG_FENCE();
  uint32_t a2[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) a2[i] = a.l[i] << 1;
  uint32_t m[NL];
  Fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; ++k) {
    uint64_t s[TBG_ACC_AB] = {};
    uint64_t t[TBG_ACC_MP] = {};
    int c = 0;
    const int lo = k < NL ? 0 : k - NL + 1;
#pragma unroll
    for (int i = lo; 2 * i < k; ++i) {
      s[c % TBG_ACC_AB] += (uint64_t)a.l[i] * a2[k - i];
      ++c;
    }
    if ((k & 1) == 0) s[c % TBG_ACC_AB] += (uint64_t)a.l[k / 2] * a.l[k / 2];
    const int mhi = k < NL ? k - 1 : NL - 1;
#pragma unroll
    for (int i = lo; i <= mhi; ++i) t[i % TBG_ACC_MP] += (uint64_t)m[i] * P_L[k - i];
    uint64_t sum = acc_total(s) + (acc_total(t) + acc);
    if (k < NL) {
      m[k] = ((uint32_t)sum * NINV) & LMASK;
      sum += (uint64_t)m[k] * P_L[0];
    } else {
      r.l[k - NL] = (uint32_t)sum & LMASK;
    }
    acc = sum >> 28;
  }
  r.l[NL - 1] = (uint32_t)acc;
  TBG_FENCE();
  return r;
}

// a * k for a small constant k (k * 2^28 * 16 fits): normalised, no reduction.
TBG_HD Fp fp_mul_small(const Fp& a, uint32_t k) {
  Fp r;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    uint64_t s = (uint64_t)a.l[i] * k + carry;
    r.l[i] = (uint32_t)s & LMASK;
    carry = s >> 28;
  }
  r.l[NL - 1] = (uint32_t)((uint64_t)a.l[NL - 1] * k + carry);
  return r;
}

TBG_HD bool fp_is_zero(const Fp& a) {
  Fp c = fp_canon(a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) o |= c.l[i];
  return o == 0;
}

TBG_HD bool fp_eq(const Fp& a, const Fp& b) {
  Fp ca = fp_canon(a), cb = fp_canon(b);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) o |= ca.l[i] ^ cb.l[i];
  return o == 0;
}

TBG_HD Fp fp_select(bool c, const Fp& a, const Fp& b) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// Montgomery -> canonical integer limbs.
TBG_HD Fp fp_from_mont(const Fp& a) {
  Fp one = fp_zero();
  one.l[0] = 1;
  return fp_canon(fp_mul(a, one));
}

// Canonical integer limbs (< 2^384) -> Montgomery form.
TBG_HD Fp fp_to_mont(const Fp& a) {
  Fp r2 = fp_from_const(R2_M);
  return fp_mul(a, r2);
}

// Exponentiation by a fixed public exponent: MSB-first sliding window of
// width WIN over the odd powers a, a^3, ... (about 378 squarings + 98
// products at width 3, + 83 at width 4, for the 380-bit exponents of p,
// against 378 + 228 for square and multiply).  The exponent is a template
// argument (a constant array), so every bit test is a scalar load and the
// window scan uniform control flow.  Width 4's eight table entries cost
// registers: k_hash_map's square roots take it (7.2 -> 6.8 ms per 16-batch
// launch), k_decode_sigs lost 13 % with it and keeps width 3
// (profiles/r04/pow/).
// (_in: the inline body, for kernels that keep the whole chain in registers
// -- k_hash_sswu; fp_pow_const: out of line.)
template <int NBITS, const uint32_t (&WD)[12], int WIN = 3>
TBG_HD Fp fp_pow_const_in(const Fp& a) {
  static_assert(WIN == 3 || WIN == 4, "window width");
  const Fp a2 = fp_sqr(a);
  const Fp t1 = a, t3 = fp_mul(t1, a2), t5 = fp_mul(t3, a2), t7 = fp_mul(t5, a2);
  Fp t9 = t7, t11 = t7, t13 = t7, t15 = t7;
  if (WIN == 4) {
    t9 = fp_mul(t7, a2);
    t11 = fp_mul(t9, a2);
    t13 = fp_mul(t11, a2);
    t15 = fp_mul(t13, a2);
  }
  auto bit = [&](int i) -> uint32_t { return (WD[i >> 5] >> (i & 31)) & 1u; };
  Fp r = t1;
  bool started = false;
  int i = NBITS - 1;  // top bit is 1
  while (i >= 0) {
    if (!bit(i)) {
      r = fp_sqr(r);
      --i;
      continue;
    }
    int L = i + 1 < WIN ? i + 1 : WIN;
    while (!bit(i - L + 1)) --L;
    uint32_t v = 0;
    for (int k = 0; k < L; ++k) v = (v << 1) | bit(i - k);
    Fp tv;
    if (WIN == 3) tv = fp_select(v == 1, t1, fp_select(v == 3, t3, fp_select(v == 5, t5, t7)));
    else if (v < 9) tv = v < 5 ? (v == 1 ? t1 : t3) : (v == 5 ? t5 : t7);
    else tv = v < 13 ? (v == 9 ? t9 : t11) : (v == 13 ? t13 : t15);
    if (started) {
      for (int k = 0; k < L; ++k) r = fp_sqr(r);
      r = fp_mul(r, tv);
    } else {
      r = tv;
      started = true;
    }
    i -= L;
  }
  return r;
}
template <int NBITS, const uint32_t (&WD)[12], int WIN = 3>
TBG_NI Fp fp_pow_const(const Fp& a) {
  return fp_pow_const_in<NBITS, WD, WIN>(a);
}

// Fermat: a^(p-2), ~380 squarings + ~95 products in one dependent chain
// (0.44 ms on a lone lane, profiles/r03/wide_fe.txt).
TBG_HD Fp fp_inv_fermat(const Fp& a) { return fp_pow_const<EXP_INV_BITS, EXP_INV_WORDS>(a); }

// ---- plain-integer limb helpers for the binary inversion (values < 2^392,
// limbs normalised to 28 bits)
TBG_HD bool li_is_one(const Fp& a) {
  uint32_t o = a.l[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < NL; ++i) o |= a.l[i];
  return o == 0;
}
TBG_HD void li_shr1(Fp& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) a.l[i] = (a.l[i] >> 1) | ((a.l[i + 1] & 1u) << 27);
  a.l[NL - 1] >>= 1;
}
// a >= b
TBG_HD bool li_geq(const Fp& a, const Fp& b) {
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) borrow = ((int32_t)a.l[i] - (int32_t)b.l[i] + borrow) >> 28;
  return borrow == 0;
}
// a - b (a >= b)
TBG_HD Fp li_sub(const Fp& a, const Fp& b) {
  Fp r;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int32_t v = (int32_t)a.l[i] - (int32_t)b.l[i] + borrow;
    r.l[i] = (uint32_t)v & LMASK;
    borrow = v >> 28;
  }
  return r;
}
// x / 2 mod p for x in [0, p)
TBG_HD Fp li_half_mod(const Fp& x) {
  Fp r = x;
  if (x.l[0] & 1u) {
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const uint32_t v = r.l[i] + P_L[i] + carry;
      r.l[i] = v & LMASK;
      carry = v >> 28;
    }
  }
  li_shr1(r);
  return r;
}
// x - y mod p for x, y in [0, p)
TBG_HD Fp li_sub_mod(const Fp& x, const Fp& y) {
  if (li_geq(x, y)) return li_sub(x, y);
  uint32_t carry = 0;
  Fp t;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t v = x.l[i] + P_L[i] + carry;
    t.l[i] = v & LMASK;
    carry = v >> 28;
  }
  return li_sub(t, y);
}

// 1 / a by the binary extended Euclidean algorithm on the plain integer
// a = xR mod p (then one product by R^3 gives the Montgomery form of 1/x):
// ~760 shift / subtract steps of 14-limb integers instead of Fermat's ~475
// dependent Montgomery products -- several times less latency for the lone
// lanes that run it (each workgroup of the batched to-affine conversions,
// the final exponentiations' Fp12 inverse).  VARIABLE TIME: its trip count
// depends on the value; every inverted value here is public (key, signature
// and message points, the pairing products) or a combination whose scalars
// are fresh per batch and no longer secret once its checks have run.
// fp_inv(0) = 0 as Fermat's.
TBG_HD Fp fp_inv_vartime(const Fp& a) {
  Fp u = fp_canon(a), v = fp_from_const(P_L), x1 = fp_zero(), x2 = fp_zero();
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) nz |= u.l[i];
  if (nz == 0) return fp_zero();
  x1.l[0] = 1;
  while (!li_is_one(u) && !li_is_one(v)) {
    while (!(u.l[0] & 1u)) {
      li_shr1(u);
      x1 = li_half_mod(x1);
    }
    while (!(v.l[0] & 1u)) {
      li_shr1(v);
      x2 = li_half_mod(x2);
    }
    if (li_geq(u, v)) {
      u = li_sub(u, v);
      x1 = li_sub_mod(x1, x2);
    } else {
      v = li_sub(v, u);
      x2 = li_sub_mod(x2, x1);
    }
  }
  return fp_mul(fp_select(li_is_one(u), x1, x2), fp_from_const(R3_L));
}

// ---- Bernstein-Yang inversion ("Fast constant-time gcd computation and
// modular inversion", 2019), variable-time form: divsteps on the low 62 bits
// of f, g build a 2x2 transition matrix (entries <= 2^62), applied to the
// full f, g (exact / 2^62) and to the cofactors d, e (/ 2^62 mod p, a
// Montgomery-style multiple of p making the division exact) -- ~12 batches of
// 62 steps for 381-bit values instead of ~760 full-width shift / subtract
// steps.  Integers as seven signed 62-bit limbs (limbs 0..5 in [0, 2^62)).
struct S62 {
  int64_t v[7];
};
constexpr uint64_t M62 = (1ull << 62) - 1;
TBG_HD S62 s62_from_fp(const Fp& a) {  // a: normalised limbs, value < 2^392
  S62 r = {{0, 0, 0, 0, 0, 0, 0}};
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int pos = 28 * i, w = pos / 62, off = pos % 62;
    const uint64_t x = a.l[i];
    r.v[w] += (int64_t)((x << off) & M62);
    if (off + 28 > 62) r.v[w + 1] += (int64_t)(x >> (62 - off));
  }
  return r;
}
// x >= 0 with normalised limbs -> 14 x 28-bit limbs
TBG_HD Fp fp_from_s62(const S62& x) {
  Fp r;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int pos = 28 * i, w = pos / 62, off = pos % 62;
    uint64_t bits = (uint64_t)x.v[w] >> off;
    if (off + 28 > 62 && w + 1 < 7) bits |= (uint64_t)x.v[w + 1] << (62 - off);
    r.l[i] = (uint32_t)(bits & LMASK);
  }
  return r;
}
// 62 divsteps (delta, f, g) on the low bits; [f_62; g_62] 2^62 = [u v; q r] [f; g]
TBG_HD int64_t divsteps62(int64_t delta, uint64_t f0, uint64_t g0, int64_t& u, int64_t& v, int64_t& q, int64_t& r) {
  u = 1;
  v = 0;
  q = 0;
  r = 1;
#pragma unroll 2
  for (int i = 0; i < 62; ++i) {
    const bool godd = (g0 & 1u) != 0, swap = delta > 0 && godd;
    const uint64_t nf = swap ? g0 : f0;
    const uint64_t ng = swap ? g0 - f0 : (godd ? g0 + f0 : g0);
    const int64_t nu = swap ? q : u, nv = swap ? r : v;
    const int64_t nq = swap ? q - u : (godd ? q + u : q), nr = swap ? r - v : (godd ? r + v : r);
    f0 = nf;
    g0 = ng >> 1;
    u = 2 * nu;
    v = 2 * nv;
    q = nq;
    r = nr;
    delta = swap ? 1 - delta : 1 + delta;
  }
  return delta;
}
// (a, b) <- ([m00 m01; m10 m11] (a, b) + (k0, k1) P) / 2^62, exact; P = null: no multiple
TBG_HD void s62_update(S62& a, S62& b, int64_t m00, int64_t m01, int64_t m10, int64_t m11, const S62* P,
                       uint64_t pinv) {
  int64_t k0 = 0, k1 = 0;
  if (P) {
    const uint64_t l0 = (uint64_t)m00 * (uint64_t)a.v[0] + (uint64_t)m01 * (uint64_t)b.v[0];
    const uint64_t l1 = (uint64_t)m10 * (uint64_t)a.v[0] + (uint64_t)m11 * (uint64_t)b.v[0];
    k0 = (int64_t)((0 - l0 * pinv) & M62);
    k1 = (int64_t)((0 - l1 * pinv) & M62);
  }
  __int128 c0 = (__int128)m00 * a.v[0] + (__int128)m01 * b.v[0];
  __int128 c1 = (__int128)m10 * a.v[0] + (__int128)m11 * b.v[0];
  if (P) {
    c0 += (__int128)k0 * P->v[0];
    c1 += (__int128)k1 * P->v[0];
  }
  c0 >>= 62;  // (the low 62 bits are zero)
  c1 >>= 62;
#pragma unroll
  for (int i = 1; i < 7; ++i) {
    c0 += (__int128)m00 * a.v[i] + (__int128)m01 * b.v[i];
    c1 += (__int128)m10 * a.v[i] + (__int128)m11 * b.v[i];
    if (P) {
      c0 += (__int128)k0 * P->v[i];
      c1 += (__int128)k1 * P->v[i];
    }
    a.v[i - 1] = (int64_t)((uint64_t)c0 & M62);
    b.v[i - 1] = (int64_t)((uint64_t)c1 & M62);
    c0 >>= 62;
    c1 >>= 62;
  }
  a.v[6] = (int64_t)c0;
  b.v[6] = (int64_t)c1;
}
// 1 / a in Montgomery form (a = xR -> 1/x R), VARIABLE TIME (see
// fp_inv_vartime); fp_inv(0) = 0
TBG_HD Fp fp_inv_bgcd(const Fp& a) {
  const Fp x = fp_canon(a);
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) nz |= x.l[i];
  if (nz == 0) return fp_zero();
  const S62 P = s62_from_fp(fp_from_const(P_L));
  uint64_t pinv = (uint64_t)P.v[0];  // p^-1 mod 2^64 by Newton (p odd)
#pragma unroll
  for (int i = 0; i < 5; ++i) pinv *= 2 - (uint64_t)P.v[0] * pinv;
  S62 f = P, g = s62_from_fp(x), d = {{0, 0, 0, 0, 0, 0, 0}}, e = {{1, 0, 0, 0, 0, 0, 0}};
  int64_t delta = 1, gz = 1;
  for (int it = 0; it < 40 && gz != 0; ++it) {  // <= ~18 batches for 381-bit values
    int64_t u, v, q, r;
    delta = divsteps62(delta, (uint64_t)f.v[0], (uint64_t)g.v[0], u, v, q, r);
    s62_update(f, g, u, v, q, r, nullptr, 0);
    s62_update(d, e, u, v, q, r, &P, pinv);
    gz = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) gz |= g.v[i];
  }
  // convergence (host bound checks): g reached 0 and f = +-1 --
  // a change to delta, the batch width or the limb form that broke the
  // iteration bound would otherwise return a wrong value in [0, 2p)
  TBG_BOUND(gz == 0, "fp_inv_bgcd: g reached 0 within 40 batches");
  TBG_BOUND((f.v[0] == 1 && (f.v[1] | f.v[2] | f.v[3] | f.v[4] | f.v[5] | f.v[6]) == 0) ||
                ((f.v[0] & f.v[1] & f.v[2] & f.v[3] & f.v[4] & f.v[5]) == (int64_t)M62 && f.v[6] == -1),
            "fp_inv_bgcd: f = +-1");
  // f = +-1 = d x (mod p): 1/x = sign(f) d; |d| < 41 p, shifted by 64 p into (23 p, 105 p)
  const bool neg = f.v[6] < 0;
  S62 y;
  __int128 c = 0;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    c += (__int128)(neg ? -d.v[i] : d.v[i]) + (__int128)64 * P.v[i];
    y.v[i] = i < 6 ? (int64_t)((uint64_t)c & M62) : (int64_t)c;
    c >>= 62;
  }
  return fp_mul(fp_reduce(fp_from_s62(y)), fp_from_const(R3_L));
}

// The inversion of every public value (see fp_inv_vartime).  Values that
// depend on a secret key call fp_inv_fermat directly (k_gen.hip).
TBG_HD Fp fp_inv(const Fp& a) { return fp_inv_bgcd(a); }

// Big-endian bytes (48) -> integer limbs; also reports whether value < p.
TBG_HD Fp fp_limbs_from_be48(const uint8_t* b, bool* lt_p) {
  Fp r = fp_zero();
  // bit position of byte j (from the end): 8 * (47 - j)
#pragma unroll
  for (int j = 0; j < 48; ++j) {
    int bit = 8 * (47 - j);
    uint32_t v = b[j];
    int li = bit / 28, off = bit % 28;
    r.l[li] |= (v << off) & LMASK;
    if (off > 20 && li + 1 < NL) r.l[li + 1] |= v >> (28 - off);
  }
  if (lt_p) {
    int32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      int32_t s = (int32_t)r.l[i] - (int32_t)P_L[i] + borrow;
      borrow = s >> 28;
    }
    *lt_p = borrow < 0;
  }
  return r;
}

// Canonical integer limbs -> 48 big-endian bytes.
TBG_HD void fp_limbs_to_be48(const Fp& a, uint8_t* b) {
#pragma unroll
  for (int j = 0; j < 48; ++j) {
    int bit = 8 * (47 - j);
    int li = bit / 28, off = bit % 28;
    uint32_t v = a.l[li] >> off;
    if (off > 20 && li + 1 < NL) v |= a.l[li + 1] << (28 - off);
    b[j] = (uint8_t)v;
  }
}

// lexicographically largest (ZCash): canonical value > (p-1)/2
TBG_HD bool fp_lex_largest_canon(const Fp& c) {
  // compare 2c > p - 1  <=>  2c >= p  (c < p)
  Fp d = fp_add(c, c);
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    int32_t s = (int32_t)d.l[i] - (int32_t)P_L[i] + borrow;
    borrow = s >> 28;
  }
  return borrow == 0;
}

TBG_HD uint32_t fp_parity_canon(const Fp& c) { return c.l[0] & 1; }

}  // namespace tbg
