// Fp (BLS12-381 base field) Montgomery multiply throughput on gfx950:
//   A: 12 x 32-bit limbs, CIOS, independent mads + one addc chain per row
//   B: 14 x 28-bit limbs, product scanning, 64-bit column accumulators (no
//      carry instructions: 28 products of 56 bits fit in 64 bits)
// Both are checked against each other (canonical results) on every thread.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

#define HD __host__ __device__ __forceinline__

// p = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
__constant__ static const uint32_t dPA[12] = {0xffffaaab, 0xb9feffff, 0xb153ffff, 0x1eabfffe, 0xf6b0f624, 0x6730d2a0,
  0xf38512bf, 0x64774b84, 0x434bacd7, 0x4b1ba7b6, 0x397fe69a, 0x1a0111ea};
static const uint32_t hPA[12] = {0xffffaaab, 0xb9feffff, 0xb153ffff, 0x1eabfffe, 0xf6b0f624, 0x6730d2a0,
  0xf38512bf, 0x64774b84, 0x434bacd7, 0x4b1ba7b6, 0x397fe69a, 0x1a0111ea};
constexpr uint32_t NINV32 = 0xfffcfffdu;

struct FpA { uint32_t l[12]; };
struct FpB { uint32_t l[14]; };

template <int N> struct PB_ { uint32_t v[14]; };

// --------------------------- variant A ---------------------------------
__device__ __forceinline__ FpA mulA(const FpA& a, const FpA& b) {
  uint32_t t[13];
#pragma unroll
  for (int j = 0; j < 13; ++j) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    uint64_t X[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) X[j] = (uint64_t)a.l[j] * b.l[i] + t[j];
    uint32_t c = 0;
    t[0] = (uint32_t)X[0];
#pragma unroll
    for (int j = 1; j < 12; ++j) t[j] = __builtin_addc((uint32_t)X[j], (uint32_t)(X[j - 1] >> 32), c, &c);
    uint32_t t13;
    t[12] = __builtin_addc(t[12], (uint32_t)(X[11] >> 32), c, &t13);
    uint32_t m = t[0] * NINV32;
    uint64_t Y[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) Y[j] = (uint64_t)m * dPA[j] + t[j];
    c = 0;
#pragma unroll
    for (int j = 1; j < 12; ++j) t[j - 1] = __builtin_addc((uint32_t)Y[j], (uint32_t)(Y[j - 1] >> 32), c, &c);
    t[11] = __builtin_addc(t[12], (uint32_t)(Y[11] >> 32), c, &c);
    t[12] = t13 + c;
  }
  FpA r;
#pragma unroll
  for (int j = 0; j < 12; ++j) r.l[j] = t[j];
  return r;  // in [0, 2p) for inputs in [0, 2p)
}

// --------------------------- variant B ---------------------------------
constexpr uint32_t MASK28 = 0x0fffffffu;
__constant__ static uint32_t dPB[14];
static uint32_t hPB[14];
static uint32_t NINV28;
__constant__ static uint32_t dNINV28;

__device__ __forceinline__ FpB mulB(const FpB& a, const FpB& b) {
  uint32_t m[14];
  FpB r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
    uint64_t s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i <= k; ++i) s0 += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
    for (int i = 0; i < k; ++i) s1 += (uint64_t)m[i] * dPB[k - i];
    acc += s0 + s1;
    m[k] = ((uint32_t)acc * dNINV28) & MASK28;
    acc += (uint64_t)m[k] * dPB[0];
    acc >>= 28;
  }
#pragma unroll
  for (int k = 14; k < 27; ++k) {
    uint64_t s0 = 0, s1 = 0;
#pragma unroll
    for (int i = k - 13; i < 14; ++i) { s0 += (uint64_t)a.l[i] * b.l[k - i]; s1 += (uint64_t)m[i] * dPB[k - i]; }
    acc += s0 + s1;
    r.l[k - 14] = (uint32_t)acc & MASK28;
    acc >>= 28;
  }
  r.l[13] = (uint32_t)acc;
  return r;
}

// ------------------------------------------------------------------------
template <int V>
__global__ void __launch_bounds__(256) bench(const uint32_t* in, uint32_t* out, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (V == 0) {
    FpA x, y, z;
    for (int j = 0; j < 12; ++j) { x.l[j] = in[tid * 40 + j]; y.l[j] = in[tid * 40 + 12 + j]; z.l[j] = in[tid * 40 + 24 + j]; }
    x.l[11] &= 0x0fffffff; y.l[11] &= 0x0fffffff; z.l[11] &= 0x0fffffff;
    for (int it = 0; it < iters; ++it) { x = mulA(x, y); z = mulA(z, y); }
    for (int j = 0; j < 12; ++j) { out[tid * 28 + j] = x.l[j]; out[tid * 28 + 12 + j] = z.l[j]; }
  } else {
    FpB x, y, z;
    for (int j = 0; j < 14; ++j) { x.l[j] = in[tid * 42 + j] & MASK28; y.l[j] = in[tid * 42 + 14 + j] & MASK28; z.l[j] = in[tid * 42 + 28 + j] & MASK28; }
    x.l[13] &= 0xffff; y.l[13] &= 0xffff; z.l[13] &= 0xffff;
    for (int it = 0; it < iters; ++it) { x = mulB(x, y); z = mulB(z, y); }
    for (int j = 0; j < 14; ++j) { out[tid * 28 + j] = x.l[j]; out[tid * 28 + 14 + j] = z.l[j]; }
  }
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 200;
  // 28-bit limbs of p and -p^-1 mod 2^28
  {
    // p as bits from hPA
    for (int k = 0; k < 14; ++k) {
      uint32_t v = 0;
      for (int b = 0; b < 28; ++b) {
        int bit = k * 28 + b;
        if (bit < 384 && ((hPA[bit / 32] >> (bit % 32)) & 1)) v |= 1u << b;
      }
      hPB[k] = v;
    }
    uint32_t p0 = hPB[0], inv = 1;
    for (int i = 0; i < 6; ++i) inv *= 2 - p0 * inv;  // inverse mod 2^32
    NINV28 = (0u - inv) & MASK28;
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(dPB), hPB, sizeof(hPB)));
    CHK(hipMemcpyToSymbol(HIP_SYMBOL(dNINV28), &NINV28, 4));
  }
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  for (int bpc : {1, 2, 4}) {
    int blocks = cus * bpc, threads = blocks * 256;
    uint32_t *din, *dout;
    size_t nin = (size_t)threads * 42;
    uint32_t* hin = (uint32_t*)malloc(nin * 4);
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < nin; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; hin[i] = (uint32_t)s; }
    CHK(hipMalloc(&din, nin * 4)); CHK(hipMalloc(&dout, (size_t)threads * 28 * 4));
    CHK(hipMemcpy(din, hin, nin * 4, hipMemcpyHostToDevice));
    for (int v = 0; v < 2; ++v) {
      hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
      if (v == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(256), 0, 0, din, dout, 2);
      else hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(256), 0, 0, din, dout, 2);
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(256), 0, 0, din, dout, iters);
      else hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(256), 0, 0, din, dout, iters);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      double muls = (double)threads * iters * 2;
      printf("variant %c  %d blocks/CU: %.2f G Fp-mul/s  (%.3f ms)\n", v == 0 ? 'A' : 'B', bpc, muls / (ms * 1e-3) / 1e9, ms);
    }
    CHK(hipFree(din)); CHK(hipFree(dout)); free(hin);
  }
  return 0;
}
