// Does the compiler's merging of fp_mul_sum's independent column
// accumulators into one dependent v_mad_u64_u32 chain cost latency /
// throughput on gfx950?  fp_mul (charon_amd/csrc/bls_field.h, the compiler
// reassociates the four a*b accumulators into one chain) against the same
// product with every multiply-add an opaque asm statement, so the four a*b
// chains and two m*p chains of a column stay independent.
//   latency:    one lane, 400 dependent products
//   throughput: every SIMD, 1 or 2 waves, 2 independent chains per thread
//
// Build: hipcc --offload-arch=gfx950 -O3 -I charon_amd/csrc fp_acc_bench.hip -o fp_acc_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "bls_field.h"
using namespace tbg;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mad_opaque(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r;
  uint64_t dummy;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(dummy) : "v"(a), "v"(b), "v"(c));
  return r;
}

template <int K, int NA, int NM>
__device__ __forceinline__ Fp fp_mul_sum_asm(const Fp* const (&a)[K], const Fp* const (&b)[K]) {
  uint32_t m[NL];
  Fp r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; ++k) {
    uint64_t s[NA] = {};
    uint64_t t[NM] = {};
    int c = 0;
    const int lo = k < NL ? 0 : k - NL + 1;
    const int hi = k < NL ? k : NL - 1;
#pragma unroll
    for (int i = lo; i <= hi; ++i) {
#pragma unroll
      for (int n = 0; n < K; ++n) {
        s[c % NA] = mad_opaque(a[n]->l[i], b[n]->l[k - i], s[c % NA]);
        ++c;
      }
    }
    const int mhi = k < NL ? k - 1 : NL - 1;
#pragma unroll
    for (int i = lo; i <= mhi; ++i) t[i % NM] = mad_opaque(m[i], P_L[k - i], t[i % NM]);
    uint64_t sum = acc;
#pragma unroll
    for (int j = 0; j < NA; ++j) sum += s[j];
#pragma unroll
    for (int j = 0; j < NM; ++j) sum += t[j];
    if (k < NL) {
      m[k] = ((uint32_t)sum * NINV) & LMASK;
      sum = mad_opaque(m[k], P_L[0], sum);
    } else {
      r.l[k - NL] = (uint32_t)sum & LMASK;
    }
    acc = sum >> 28;
  }
  r.l[NL - 1] = (uint32_t)acc;
  return r;
}
template <int NA, int NM>
__device__ __forceinline__ Fp fp_mul_asm(const Fp& a, const Fp& b) {
  const Fp* const A[1] = {&a};
  const Fp* const B[1] = {&b};
  return fp_mul_sum_asm<1, NA, NM>(A, B);
}

template <int V>
__device__ __forceinline__ Fp mulv(const Fp& a, const Fp& b) {
  if constexpr (V == 0) return fp_mul(a, b);
  else if constexpr (V == 1) return fp_mul_asm<4, 2>(a, b);
  else if constexpr (V == 2) return fp_mul_asm<2, 1>(a, b);
  else return fp_mul_asm<1, 1>(a, b);
}

__device__ Fp load_fp(const uint32_t* in, int t) {
  Fp y;
  for (int j = 0; j < NL; ++j) y.l[j] = in[(t * 8 + j) % 4096] & LMASK;
  y.l[NL - 1] &= 0xffff;
  return y;
}

template <int V>
__global__ void __launch_bounds__(64) k_lat(const uint32_t* in, uint32_t* out, int iters) {
  Fp x = load_fp(in, threadIdx.x), y = load_fp(in, threadIdx.x + 7);
  if (threadIdx.x == 0)
    for (int i = 0; i < iters; ++i) x = mulv<V>(x, y);
  uint32_t acc = 0;
  for (int j = 0; j < NL; ++j) acc ^= x.l[j];
  out[threadIdx.x] = acc;
}

template <int V>
__global__ void __launch_bounds__(256) k_thr(const uint32_t* in, uint32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  Fp x0 = load_fp(in, t), x1 = load_fp(in, t + 3), y = load_fp(in, t + 7);
  for (int i = 0; i < iters; ++i) {
    x0 = mulv<V>(x0, y);
    x1 = mulv<V>(x1, y);
  }
  uint32_t acc = 0;
  for (int j = 0; j < NL; ++j) acc ^= x0.l[j] ^ x1.l[j];
  out[t] = acc;
}

template <int V>
void run(const char* name, const uint32_t* din, uint32_t* dout, int cus) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float ms;
  hipLaunchKernelGGL(k_lat<V>, dim3(1), dim3(64), 0, 0, din, dout, 4);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_lat<V>, dim3(1), dim3(64), 0, 0, din, dout, 400);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  CHK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-22s latency %.3f us/mul", name, ms * 1e3 / 400);
  for (int w = 1; w <= 2; ++w) {
    const int blocks = cus * w;
    hipLaunchKernelGGL(k_thr<V>, dim3(blocks), dim3(256), 0, 0, din, dout, 2);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_thr<V>, dim3(blocks), dim3(256), 0, 0, din, dout, 200);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double muls = (double)blocks * 256 * 200 * 2;
    printf("  %dw: %.1f G Fp-mul/s (%.1f T mad/s)", w, muls / (ms * 1e-3) / 1e9, muls * 392 / (ms * 1e-3) / 1e12);
  }
  printf("\n");
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t *din, *dout;
  CHK(hipMalloc(&din, 4096 * 4));
  CHK(hipMalloc(&dout, cus * 2 * 256 * 4));
  uint32_t h[4096];
  uint64_t s = 88172645463325252ull;
  for (auto& v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (uint32_t)s; }
  CHK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
  run<0>("fp_mul (compiler)", din, dout, cus);
  run<1>("asm acc 4+2", din, dout, cus);
  run<2>("asm acc 2+1", din, dout, cus);
  run<3>("asm acc 1+1", din, dout, cus);
  return 0;
}
