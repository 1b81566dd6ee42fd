// Static instruction mix of the hexad Miller step's pieces (compile only:
// tools/isa_counts.py --src tools/microbench/hex_ops_isa.hip): one kernel per
// piece, so each count is that piece's loop-body cost.
#define TBG_SCHED_FENCE 1
#include "tbls_launch.h"
#include "bls_lines.h"
#include "bls_hex.h"
using namespace tbg;

__global__ void __launch_bounds__(64, 2) k_isa_sqr(uint32_t* io) {
  Fp4h f = hex_load(io);
  f = hex_sqr(f);
  hex_store(io, f);
}
__global__ void __launch_bounds__(64, 2) k_isa_line_at(uint32_t* io, const uint32_t* lines, const G1A* P) {
  Fp4h f = hex_load(io);
  f = hex_line_at(f, lines, 0, P->x, P->y);
  hex_store(io, f);
}
__global__ void __launch_bounds__(64, 2) k_isa_line_folded(uint32_t* io, const uint32_t* lines) {
  Fp4h f = hex_load(io);
  f = hex_line_folded(f, lines, 0);
  hex_store(io, f);
}
__global__ void __launch_bounds__(64, 2) k_isa_pair_mul(uint32_t* io) {
  Fp a, ap, b, bp;
  for (int i = 0; i < NL; ++i) { a.l[i] = io[i]; ap.l[i] = io[NL + i]; b.l[i] = io[2 * NL + i]; bp.l[i] = io[3 * NL + i]; }
  const Fp r = pair_mul_lane(threadIdx.x & 1, a, ap, b, bp);
  for (int i = 0; i < NL; ++i) io[i] = r.l[i];
}
__global__ void __launch_bounds__(64, 2) k_isa_fp_mul(uint32_t* io) {
  Fp a, b;
  for (int i = 0; i < NL; ++i) { a.l[i] = io[i]; b.l[i] = io[NL + i]; }
  const Fp r = fp_mul(a, b);
  for (int i = 0; i < NL; ++i) io[i] = r.l[i];
}
__global__ void __launch_bounds__(64, 2) k_isa_fp_reduce(uint32_t* io) {
  Fp a;
  for (int i = 0; i < NL; ++i) a.l[i] = io[i];
  const Fp r = fp_reduce(a);
  for (int i = 0; i < NL; ++i) io[i] = r.l[i];
}
