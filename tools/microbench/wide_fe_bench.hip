// Latency of the level-0 tail's pieces on one wave (k_l0_final's form,
// charon_amd/csrc/bls_wide.h): the whole wide final exponentiation, its
// one-lane Fp12 inversion, 63 wide cyclotomic squarings, 16 wide products,
// and a one-lane chain of 400 dependent Fp products.
//
// Build: hipcc --offload-arch=gfx950 -O3 -I charon_amd/csrc wide_fe_bench.hip -o wide_fe_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "bls_wide.h"
using namespace tbg;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

struct Exec {
  template <class Fn>
  __device__ void operator()(Fn&& fn) {
    fn((int)threadIdx.x);
    __syncthreads();
  }
};

__device__ void load_in(WideSlots& S, const uint32_t* in) {
  const int l = threadIdx.x;
  if (l < WIDE_FP)
    for (int j = 0; j < NL; ++j) S.v[0][l].l[j] = in[l * NL + j] & (j == NL - 1 ? 0xffffu : LMASK);
  __syncthreads();
}
__device__ void store_out(WideSlots& S, uint32_t* out) {
  const int l = threadIdx.x;
  if (l < WIDE_FP)
    for (int j = 0; j < NL; ++j) out[l * NL + j] = S.v[0][l].l[j];
}

template <int WHAT>
__global__ void __launch_bounds__(64) k_bench(const uint32_t* in, uint32_t* out) {
  __shared__ WideSlots S;
  Exec ex;
  load_in(S, in);
  if (WHAT == 0) wide_final_exp(ex, S);
  if (WHAT == 1) ex([&](int l) { wide_inv(l, S.v[1], S.v[0]); });
  if (WHAT == 2)
    for (int i = 0; i < 63; ++i) wide_cyc_sqr(ex, S, 0);
  if (WHAT == 3) {
    ex([&](int l) { wide_copy(l, S.v[1], S.v[0]); });
    for (int i = 0; i < 16; ++i) wide_mul_to(ex, S, 0, 0, 1);
  }
  if (WHAT == 4 && threadIdx.x == 0) {
    Fp x = S.v[0][0], y = S.v[0][1];
    for (int i = 0; i < 400; ++i) x = fp_mul(x, y);
    S.v[0][0] = x;
  }
  if (WHAT == 5 && threadIdx.x == 0) S.v[0][0] = fp_inv(S.v[0][0]);
  __syncthreads();
  store_out(S, out);
}

template <int WHAT>
float run(const uint32_t* in, uint32_t* out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_bench<WHAT>, dim3(1), dim3(64), 0, 0, in, out);
  CHK(hipDeviceSynchronize());
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(k_bench<WHAT>, dim3(1), dim3(64), 0, 0, in, out);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  uint32_t *in, *out;
  CHK(hipMalloc(&in, 4096 * 4));
  CHK(hipMalloc(&out, 4096 * 4));
  uint32_t h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (uint32_t)(i * 2654435761u + 12345u);
  CHK(hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice));
  printf("wide final exponentiation        %8.3f ms\n", run<0>(in, out));
  printf("wide_inv (one lane, fp12_inv)    %8.3f ms\n", run<1>(in, out));
  printf("63 wide cyclotomic squarings     %8.3f ms\n", run<2>(in, out));
  printf("16 wide products                 %8.3f ms\n", run<3>(in, out));
  printf("400 dependent fp_mul, one lane   %8.3f ms\n", run<4>(in, out));
  printf("fp_inv, one lane                 %8.3f ms\n", run<5>(in, out));
  return 0;
}
