// Single-wave issue rate of v_mad_u64_u32 (gfx950) by carry-out SGPR choice
// and chain count: is the one-wave cap (19 T lane-ops/s in valu_rates) set by
// the dead carry-out SGPR the compiler reuses, or by the chains' latency?
//   same8   8 chains, every mad writes its dead carry to s[20:21]
//   dist8   8 chains, chain i writes s[20 + 2i : 21 + 2i]
//   same16  16 chains, s[20:21]
// at 1 and 2 waves per SIMD (256 CU x 4 SIMD x w waves of 64 lanes).
//
// Build: hipcc --offload-arch=gfx950 -O3 mad_issue.hip -o mad_issue
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

#define MAD_S(i, s) asm volatile("v_mad_u64_u32 %0, " s ", %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b) : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", "s34", "s35")

template <int MODE>
__global__ void __launch_bounds__(64) bench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  constexpr int N = MODE == 2 ? 16 : 8;
  uint64_t x[N];
  for (int i = 0; i < N; ++i) x[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (MODE == 0) {
        MAD_S(0, "s[20:21]"); MAD_S(1, "s[20:21]"); MAD_S(2, "s[20:21]"); MAD_S(3, "s[20:21]");
        MAD_S(4, "s[20:21]"); MAD_S(5, "s[20:21]"); MAD_S(6, "s[20:21]"); MAD_S(7, "s[20:21]");
      } else if constexpr (MODE == 1) {
        MAD_S(0, "s[20:21]"); MAD_S(1, "s[22:23]"); MAD_S(2, "s[24:25]"); MAD_S(3, "s[26:27]");
        MAD_S(4, "s[28:29]"); MAD_S(5, "s[30:31]"); MAD_S(6, "s[32:33]"); MAD_S(7, "s[34:35]");
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) MAD_S(i, "s[20:21]");
      }
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < N; ++i) acc ^= (uint32_t)x[i] ^ (uint32_t)(x[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
double run(uint32_t* out, int waves_per_simd, int iters) {
  const int blocks = 256 * 4 * waves_per_simd;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(64), 0, 0, out, 2, 1u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(64), 0, 0, out, iters, 1u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = (double)blocks * 64 * iters * 8 * (MODE == 2 ? 16 : 8);
  return ops / (ms * 1e-3) / 1e12;
}

int main() {
  uint32_t* out;
  CHK(hipMalloc(&out, 256 * 4 * 8 * 64 * 4));
  const char* names[3] = {"same8 ", "dist8 ", "same16"};
  for (int w = 1; w <= 2; ++w) {
    printf("waves/SIMD %d: %s %.2f T  %s %.2f T  %s %.2f T\n", w, names[0], run<0>(out, w, 4000), names[1],
           run<1>(out, w, 4000), names[2], run<2>(out, w, 2000));
  }
  return 0;
}
