// VALU issue-rate microbenchmark for the integer instructions a 381-bit
// Montgomery multiply is built from (gfx950).  Each thread runs 8 independent
// chains of one instruction; the rate is reported in lane-ops per second so
// it can be compared directly with the 256 CU x 64 lane x 2.4 GHz full rate.
//
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

enum Op { MAD_U64_U32, MUL_LO_U32, MUL_HI_U32, MAD_U32_U24, MUL_HI_U32_U24,
          ADD_CO_U32, ADDC_CO_U32, ADD_U32, FMA_F64, ADD3_U32, NOPS };
static const char* kNames[NOPS] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
  "v_mad_u32_u24", "v_mul_hi_u32_u24", "v_add_co_u32", "v_addc_co_u32", "v_add_u32",
  "v_fma_f64", "v_add3_u32"};

constexpr int UNROLL = 16;

template <int OP>
__global__ void __launch_bounds__(256) bench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  uint64_t x[8];
  uint32_t y[8];
  double d[8];
  uint64_t c[8];
  for (int i = 0; i < 8; ++i) { x[i] = a + i; y[i] = b + 3 * i; d[i] = 1.0 + i * 1e-3; c[i] = 0; }
  double da = 0.999999, db = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == MAD_U64_U32) {
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x[i]), "=s"(c[i]) : "v"(a), "v"(b));
        } else if constexpr (OP == MUL_LO_U32) {
          asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(y[i]) : "v"(b));
        } else if constexpr (OP == MUL_HI_U32) {
          asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(y[i]) : "v"(b));
        } else if constexpr (OP == MAD_U32_U24) {
          asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(y[i]) : "v"(a), "v"(b));
        } else if constexpr (OP == MUL_HI_U32_U24) {
          asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(y[i]) : "v"(b));
        } else if constexpr (OP == ADD_CO_U32) {
          asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(y[i]), "=s"(c[i]) : "v"(b));
        } else if constexpr (OP == ADDC_CO_U32) {
          asm volatile("v_addc_co_u32 %0, %1, %0, %2, %1" : "+v"(y[i]), "+s"(c[i]) : "v"(b));
        } else if constexpr (OP == ADD_U32) {
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(y[i]) : "v"(b));
        } else if constexpr (OP == FMA_F64) {
          asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[i]) : "v"(da), "v"(db));
        } else if constexpr (OP == ADD3_U32) {
          asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(y[i]) : "v"(a), "v"(b));
        }
      }
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < 8; ++i) acc ^= (uint32_t)x[i] ^ (uint32_t)(x[i] >> 32) ^ y[i] ^ (uint32_t)c[i] ^ (uint32_t)(int)d[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
double run(uint32_t* out, int blocks_per_cu, int cus, int iters) {
  int blocks = blocks_per_cu * cus;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, 2, 1u);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0; CHK(hipEventElapsedTime(&ms, e0, e1));
  double ops = (double)blocks * 256 * iters * UNROLL * 8;
  CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
  return ops / (ms * 1e-3);
}

template <int OP>
void sweep(uint32_t* out, int cus, int iters) {
  printf("%-18s", kNames[OP]);
  for (int bpc : {1, 2, 4, 8}) {
    double r = run<OP>(out, bpc, cus, iters);
    printf("  %dw/SIMD %8.2f T/s", bpc, r / 1e12);
  }
  printf("\n");
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 2000;
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  printf("full-rate reference: %d CU x 64 lanes x 2.4 GHz = %.2f T lane-ops/s\n", cus, cus * 64 * 2.4e9 / 1e12);
  uint32_t* out;
  CHK(hipMalloc(&out, sizeof(uint32_t) * 256 * 8 * cus));
  sweep<ADD_U32>(out, cus, iters);
  sweep<ADD3_U32>(out, cus, iters);
  sweep<ADD_CO_U32>(out, cus, iters);
  sweep<ADDC_CO_U32>(out, cus, iters);
  sweep<MAD_U64_U32>(out, cus, iters);
  sweep<MUL_LO_U32>(out, cus, iters);
  sweep<MUL_HI_U32>(out, cus, iters);
  sweep<MAD_U32_U24>(out, cus, iters);
  sweep<MUL_HI_U32_U24>(out, cus, iters);
  sweep<FMA_F64>(out, cus, iters);
  CHK(hipFree(out));
  return 0;
}
