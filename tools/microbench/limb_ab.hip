// Limb-choice A/B: the engine's Montgomery product on
// 14 x 28-bit limbs (bls_field.h fp_mul / fp_mul2: 196 + 196 = 392 mul-adds,
// every column of <= 28 products of 56 bits in ONE 64-bit accumulator, no
// carry instructions) against 13 x 30-bit limbs (169 + 169 = 338 mul-adds,
// but a column of 13 products of 60 bits nearly fills 64 bits, so the a*b
// and m*p halves keep separate accumulators and the column sum is split at
// 30 bits before it is combined: extra shifts / masks / adds per column, and
// no headroom for lazy (unnormalised) operands, which the engine's hexad and
// lane-pair formulas use throughout).  Same harness as fp_chain_bench: C
// independent chains per lane, 1 or 2 waves per SIMD; the 30-bit product is
// checked against the 28-bit one (both map a Montgomery-form value x R to
// x y R, different R: compared through a host big-integer check).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/microbench/limb_ab.hip -o /tmp/limb_ab && /tmp/limb_ab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define TBG_SCHED_FENCE 1
#include "../../charon_amd/csrc/bls_field.h"
using namespace tbg;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

constexpr int NL30 = 13;
constexpr uint32_t M30 = (1u << 30) - 1;
__device__ constexpr uint32_t P30[13] = {0x3fffaaabu, 0x27fbffffu, 0x153ffffbu, 0x2affffacu, 0x30f6241eu, 0x34a83dau,
                                         0x112bf673u, 0x12e13ce1u, 0x2cd76477u, 0x1ed90d2eu, 0x29a4b1bau, 0x3a8e5ff9u,
                                         0x1a0111u};
constexpr uint32_t NINV30 = 0x3ffcfffdu;
struct Fp30 { uint32_t l[NL30]; };

// REDC(sum_n a_n b_n), product scanning, normalised (< 2^30) limbs: per
// column the a*b products in two accumulators, the m*p products in one, each
// split at 30 bits before the column sum (13 products of < 2^60 fit 64 bits
// alone, not together with the other half).
template <int K>
__device__ __forceinline__ Fp30 fp30_mul_sum(const Fp30* const (&a)[K], const Fp30* const (&b)[K]) {
  __builtin_amdgcn_sched_barrier(0);
  uint32_t m[NL30];
  Fp30 r;
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL30 - 1; ++k) {
    uint64_t s0 = 0, s1 = 0, t = 0;
    int c = 0;
    const int lo = k < NL30 ? 0 : k - NL30 + 1;
    const int hi = k < NL30 ? k : NL30 - 1;
#pragma unroll
    for (int i = lo; i <= hi; ++i)
#pragma unroll
      for (int n = 0; n < K; ++n) {
        if (c++ & 1) s1 += (uint64_t)a[n]->l[i] * b[n]->l[k - i];
        else s0 += (uint64_t)a[n]->l[i] * b[n]->l[k - i];
      }
    const int mhi = k < NL30 ? k - 1 : NL30 - 1;
#pragma unroll
    for (int i = lo; i <= mhi; ++i) t += (uint64_t)m[i] * P30[k - i];
    // split at 30 bits: the low parts and the carry-in sum to < 2^33, the high parts to < 2^36
    uint64_t low = (s0 & M30) + (s1 & M30) + (t & M30) + (carry & M30);
    uint64_t high = (s0 >> 30) + (s1 >> 30) + (t >> 30) + (carry >> 30);
    if (k < NL30) {
      m[k] = ((uint32_t)low * NINV30) & M30;
      low += (uint64_t)m[k] * P30[0];
    } else {
      r.l[k - NL30] = (uint32_t)low & M30;
    }
    carry = high + (low >> 30);
  }
  r.l[NL30 - 1] = (uint32_t)carry;
  __builtin_amdgcn_sched_barrier(0);
  return r;
}
__device__ __forceinline__ Fp30 fp30_mul(const Fp30& a, const Fp30& b) {
  const Fp30* const A[1] = {&a};
  const Fp30* const B[1] = {&b};
  return fp30_mul_sum<1>(A, B);
}
__device__ __forceinline__ Fp30 fp30_mul2(const Fp30& a, const Fp30& b, const Fp30& c, const Fp30& d) {
  const Fp30* const A[2] = {&a, &c};
  const Fp30* const B[2] = {&b, &d};
  return fp30_mul_sum<2>(A, B);
}

template <int C, int K>
__global__ void __launch_bounds__(256) chain28(const uint32_t* in, uint32_t* out, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  Fp x[C], y;
  for (int j = 0; j < NL; ++j) y.l[j] = in[(tid * 8) % 4096 + j] & LMASK;
  y.l[NL - 1] &= 0xffff;
#pragma unroll
  for (int c = 0; c < C; ++c) { x[c] = y; x[c].l[0] ^= c; }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = K == 1 ? fp_mul(x[c], y) : fp_mul2(x[c], y, y, x[c]);
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) for (int j = 0; j < NL; ++j) acc ^= x[c].l[j];
  out[tid] = acc;
}

// (the 30-bit product's output < 2p feeds the next one unreduced: 2p < 2^382,
// products < 2^764 < R p = 2^390 p -- the chain stays in range like the engine's)
template <int C, int K>
__global__ void __launch_bounds__(256) chain30(const uint32_t* in, uint32_t* out, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  Fp30 x[C], y;
  for (int j = 0; j < NL30; ++j) y.l[j] = in[(tid * 8) % 4096 + j] & M30;
  y.l[NL30 - 1] &= 0xffff;
#pragma unroll
  for (int c = 0; c < C; ++c) { x[c] = y; x[c].l[0] ^= c; }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = K == 1 ? fp30_mul(x[c], y) : fp30_mul2(x[c], y, y, x[c]);
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) for (int j = 0; j < NL30; ++j) acc ^= x[c].l[j];
  out[tid] = acc;
}

// correctness: REDC30(a b) for fixed inputs, printed for the host check
__global__ void check30(const uint32_t* ab, uint32_t* out) {
  if (threadIdx.x) return;
  Fp30 a, b;
  for (int j = 0; j < NL30; ++j) { a.l[j] = ab[j]; b.l[j] = ab[NL30 + j]; }
  const Fp30 r = fp30_mul(a, b), r2 = fp30_mul2(a, b, b, a);
  for (int j = 0; j < NL30; ++j) { out[j] = r.l[j]; out[NL30 + j] = r2.l[j]; }
}

template <class Kern>
double run(Kern k, uint32_t* din, uint32_t* dout, int cus, int bpc, int iters, int chains) {
  const int blocks = cus * bpc;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, din, dout, 2);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, din, dout, iters);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  return (double)blocks * 256 * iters * chains / (ms * 1e-3) / 1e9;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t *din, *dout;
  CHK(hipMalloc(&din, 4096 * 4 + 64));
  CHK(hipMalloc(&dout, cus * 4 * 256 * 4));
  uint32_t h[4096 + 16];
  uint64_t s = 88172645463325252ull;
  for (auto& v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (uint32_t)s; }
  CHK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
  // correctness inputs: a = 3^200 mod p-ish limbs from the host stream (< p: top limb masked)
  uint32_t ab[2 * NL30], outv[2 * NL30];
  for (int j = 0; j < 2 * NL30; ++j) ab[j] = h[100 + j] & M30;
  ab[NL30 - 1] &= 0xffff;
  ab[2 * NL30 - 1] &= 0xffff;
  CHK(hipMemcpy(din, ab, sizeof(ab), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(check30, dim3(1), dim3(64), 0, 0, din, dout);
  CHK(hipMemcpy(outv, dout, sizeof(outv), hipMemcpyDeviceToHost));
  printf("check a");
  for (int j = 0; j < NL30; ++j) printf(" %x", ab[j]);
  printf(" b");
  for (int j = 0; j < NL30; ++j) printf(" %x", ab[NL30 + j]);
  printf(" r");
  for (int j = 0; j < NL30; ++j) printf(" %x", outv[j]);
  printf(" r2");
  for (int j = 0; j < NL30; ++j) printf(" %x", outv[NL30 + j]);
  printf("\n");
  CHK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
  for (int bpc : {1, 2}) {
    const double a1 = run(chain28<2, 1>, din, dout, cus, bpc, 400, 2), b1 = run(chain30<2, 1>, din, dout, cus, bpc, 400, 2);
    const double a2 = run(chain28<2, 2>, din, dout, cus, bpc, 200, 2), b2 = run(chain30<2, 2>, din, dout, cus, bpc, 200, 2);
    printf("waves/SIMD=%d  fp_mul: 14x28 %.2f G/s, 13x30 %.2f G/s (%.3fx)   fp_mul2: 14x28 %.2f G/s, 13x30 %.2f G/s (%.3fx)\n",
           bpc, a1, b1, b1 / a1, a2, b2, b2 / a2);
  }
  return 0;
}
