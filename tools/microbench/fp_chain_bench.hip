// Latency vs throughput of the engine's Fp multiply (charon_amd/csrc/bls_field.h)
// on gfx950: C independent dependent-chains per thread, 1 or 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../charon_amd/csrc/bls_field.h"
using namespace tbg;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

template <int C>
__global__ void __launch_bounds__(256) chain(const uint32_t* in, uint32_t* out, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  Fp x[C], y;
  for (int j = 0; j < NL; ++j) y.l[j] = in[(tid * 8) % 4096 + j] & LMASK;
  y.l[NL - 1] &= 0xffff;
#pragma unroll
  for (int c = 0; c < C; ++c) { x[c] = y; x[c].l[0] ^= c; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = fp_mul(x[c], y);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) for (int j = 0; j < NL; ++j) acc ^= x[c].l[j];
  out[tid] = acc;
}

// Same dependent chain, body unrolled U times: U * ~500 instructions of
// straight-line code (I-cache pressure test).
template <int U>
__global__ void __launch_bounds__(256) chain_unrolled(const uint32_t* in, uint32_t* out, int iters) {
  int tid = blockIdx.x * blockDim.x + threadIdx.x;
  Fp x, y;
  for (int j = 0; j < NL; ++j) y.l[j] = in[(tid * 8) % 4096 + j] & LMASK;
  y.l[NL - 1] &= 0xffff;
  x = y;
  for (int it = 0; it < iters; it += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) { x = fp_mul(x, y); y.l[u % NL] ^= 1; }
  }
  uint32_t acc = 0;
  for (int j = 0; j < NL; ++j) acc ^= x.l[j];
  out[tid] = acc;
}

template <int U>
void run_unrolled(uint32_t* din, uint32_t* dout, int cus, int iters) {
  int blocks = cus;
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chain_unrolled<U>, dim3(blocks), dim3(256), 0, 0, din, dout, U);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(chain_unrolled<U>, dim3(blocks), dim3(256), 0, 0, din, dout, iters);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  printf("unroll=%d: per-lane latency %.3f us per mul\n", U, ms * 1e3 / iters);
}

template <int C>
void run(uint32_t* din, uint32_t* dout, int cus, int bpc, int iters) {
  int blocks = cus * bpc;
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chain<C>, dim3(blocks), dim3(256), 0, 0, din, dout, 2);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(chain<C>, dim3(blocks), dim3(256), 0, 0, din, dout, iters);
  CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double muls = (double)blocks * 256 * iters * C;
  printf("chains=%d waves/SIMD=%d: %.2f G Fp-mul/s, per-lane latency %.3f us per mul\n", C, bpc,
         muls / (ms * 1e-3) / 1e9, ms * 1e3 / iters);
}

int main() {
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  uint32_t *din, *dout;
  CHK(hipMalloc(&din, 4096 * 4 + 64)); CHK(hipMalloc(&dout, cus * 4 * 256 * 4));
  uint32_t h[4096 + 16]; uint64_t s = 88172645463325252ull;
  for (auto& v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (uint32_t)s; }
  CHK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
  run_unrolled<1>(din, dout, cus, 384);
  run_unrolled<8>(din, dout, cus, 384);
  run_unrolled<32>(din, dout, cus, 384);
  run_unrolled<128>(din, dout, cus, 384);
  for (int bpc : {1, 2}) { run<1>(din, dout, cus, bpc, 400); run<2>(din, dout, cus, bpc, 400); run<4>(din, dout, cus, bpc, 200); }
  return 0;
}
