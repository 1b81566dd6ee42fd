// Cofactor clearing of hash_to_G2 (the middle of k_hash.hip's chain),
// Budroni-Pintore (RFC 9380 G.3):
//   h(P) = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P)
//        = [x]([x]P + psi(P)) + psi^2(2P) - psi(P) - [x]P - P,
// in three lane-PAIR kernels (bls_pair.h: the Fp2 coordinates split over two
// lanes) so each holds at most two G2 points across its [x] loop and runs two
// waves per SIMD:
//   k_hash_clear_x1   P = Q0 + Q1, t1 = [x]P, u = t1 + psi(P)  (temporaries in h_jac)
//   k_hash_clear_x2   v = [x]u
//   k_hash_clear_fin  h = psi^2(2P) - psi(P) + v - t1 - P
// The single-lane form kept three live points across the second [x] loop and
// ran at one wave per SIMD (12.3 ms per 160k-message launch); it is kept as
// the host reference (g2_clear_cofactor_t, bls_curve.h) the tests check.
#define TBG_ADD_DBL_INLINE 1
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernels in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_h2c.h"
#include "bls_pair.h"

namespace tbg {

__device__ __forceinline__ Jac<Fp2x> px_psi(const Jac<Fp2x>& p) {
  return {f_mulc(f_conj(p.X), PSI_X), f_mulc(f_conj(p.Y), PSI_Y), f_reduce(f_conj(p.Z))};
}

// [x] p = -[|x|] p (63 doublings, 5 additions).  TBG_CLEAR_X: the additions
// without the doubling case (bls_pair.h jac_mul_xabs_x: inputs retired early,
// fewer live values), the rare doubling case (only points of tiny order)
// redone with the complete formulas; 0: the complete formulas throughout.
#ifndef TBG_CLEAR_X
#define TBG_CLEAR_X 1
#endif
__device__ __forceinline__ Jac<Fp2x> px_mul_x_full(const Jac<Fp2x>& p) {
  Jac<Fp2x> acc = p;
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl_in(acc);
    if ((X_ABS >> i) & 1) acc = jac_add_in<Fp2x, true>(acc, p);
  }
  return jac_neg(acc);
}
// The rare cases out of line (their registers do not count against the
// kernels' loop bodies; the complete formulas inline spilled ~360 VGPRs of
// k_hash_clear_x1 to scratch): [x] p with the complete formulas, and the
// complete addition.
__device__ __noinline__ Jac<Fp2x> px_mul_x_complete(const Jac<Fp2x>& p) { return px_mul_x_full(p); }
__device__ __noinline__ Jac<Fp2x> px_add_complete(const Jac<Fp2x>& a, const Jac<Fp2x>& b) {
  return jac_add(a, b);  // (its doubling case a call: a branch over an inline doubling is out of range here)
}
// a + b (b: psi(b) when PSI) from their slots, with the complete formulas
__device__ __forceinline__ Jac<Fp2x> px_psi(const Jac<Fp2x>& p);
__device__ __noinline__ Jac<Fp2x> px_add_complete_at(const G2J* a, const G2J* b, bool psi) {
  const Jac<Fp2x> q = px_load(*b);
  return px_add_complete(px_load(*a), psi ? px_psi(q) : q);
}
// [x] p for p in its h_jac slot, re-read at each of the five additions
// (the compiler barrier keeps the load where it is used: a base point held
// across the 63 doublings was spilled to scratch and reloaded every step)
__device__ __forceinline__ Jac<Fp2x> px_mul_x(const G2J& slot) {
#if TBG_CLEAR_X
  bool exc = false;
  Jac<Fp2x> acc = px_load(slot);
#pragma unroll 1
  for (int i = 62; i >= 0; --i) {
    acc = jac_dbl_lo(acc);
    if ((X_ABS >> i) & 1) {
      __asm__ __volatile__("" ::: "memory");
      acc = jac_add_x(acc, px_load(slot), exc);
    }
  }
  if (pair_all(!exc)) return jac_neg(acc);  // (pair-uniform)
  return px_mul_x_complete(px_load(slot));
#else
  return px_mul_x_full(px_load(slot));
#endif
}

__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_hash_clear_x1(DevBatch B) {
  const uint32_t m = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // both lanes of a pair take the same branches
  if (m >= B.n_msgs) return;
  G2J* h = B.h_jac + m;
  const uint32_t n = B.n_msgs;
  // P = Q0 + Q1, the two SSWU maps' points (k_hash_sswu); the rare doubling
  // case redone from the slots (nothing held in registers for it)
  bool exc = false;
  Jac<Fp2x> p = jac_add_x(px_load(h[0]), px_load(h[n]), exc);
  if (!pair_all(!exc)) p = px_add_complete_at(h, h + n, false);  // (pair-uniform)
  px_store(h[0], p);
  __asm__ __volatile__("" ::: "memory");
  const Jac<Fp2x> t1 = px_mul_x(h[0]);
  px_store(h[n], t1);
  __asm__ __volatile__("" ::: "memory");
  exc = false;
  Jac<Fp2x> u = jac_add_x(t1, px_psi(px_load(h[0])), exc);
  if (!pair_all(!exc)) u = px_add_complete_at(h + n, h, true);
  px_store(h[2 * n], u);
}

__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_hash_clear_x2(DevBatch B) {
  const uint32_t m = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (m >= B.n_msgs) return;
  G2J* u = B.h_jac + 2 * B.n_msgs + m;
  px_store(*u, px_mul_x(*u));
}

// The combination with the complete additions (out-of-line calls): the rare
// doubling case of the fast path below, out of line so its registers do not
// count against the kernel's body.
__device__ __noinline__ Jac<Fp2x> clear_fin_complete(const DevBatch& B, uint32_t m) {
  const Jac<Fp2x> p = px_load(B.h_jac[m]);
  Jac<Fp2x> t3 = px_psi(px_psi(jac_dbl(p)));                                    // psi^2(2P)
  t3 = jac_add(t3, jac_neg(px_psi(p)));                                          // - psi(P)
  t3 = jac_add(t3, px_load(B.h_jac[2 * B.n_msgs + m]));                          // + [x]([x]P + psi(P))
  t3 = jac_add(t3, jac_neg(px_load(B.h_jac[B.n_msgs + m])));                     // - [x]P
  return jac_add(t3, jac_neg(p));                                                // - P
}

// h = psi^2(2P) - [x]P + [x]([x]P + psi(P)) - psi(P) - P with the additions
// that skip the doubling case (bls_pair.h jac_add_x) and psi(P) formed where
// it is used: two live points instead of three (the complete form spilled
// 654 VGPRs and wrote 4.5 KB of scratch per message)
// (each operand is loaded where it is used and P read again for the last two
// terms -- the compiler barriers keep loads from being hoisted across the
// additions: three live points there spilled ~200 VGPRs)
__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_hash_clear_fin(DevBatch B) {
  const uint32_t m = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;
  if (m >= B.n_msgs) return;
  bool exc = false;
  Jac<Fp2x> t3 = px_psi(px_psi(jac_dbl_in(px_load(B.h_jac[m]))));              // psi^2(2P)
  __asm__ __volatile__("" ::: "memory");
  t3 = jac_add_x(t3, jac_neg(px_load(B.h_jac[B.n_msgs + m])), exc);             // - [x]P
  __asm__ __volatile__("" ::: "memory");
  t3 = jac_add_x(t3, px_load(B.h_jac[2 * B.n_msgs + m]), exc);                  // + [x]([x]P + psi(P))
  __asm__ __volatile__("" ::: "memory");
  const Jac<Fp2x> p = px_load(B.h_jac[m]);
  t3 = jac_add_x(t3, jac_neg(px_psi(p)), exc);                                  // - psi(P)
  t3 = jac_add_x(t3, jac_neg(p), exc);                                          // - P
  if (!pair_all(!exc)) t3 = clear_fin_complete(B, m);  // (pair-uniform)
  px_store(B.h_jac[m], t3);
}

void launch_hash_clear(const DevBatch& B, hipStream_t st) {
  if (!B.n_msgs) return;
  const dim3 grid = grid_for(2 * B.n_msgs);
  TBG_KLAUNCH(k_hash_clear_x1, grid, dim3(kBlock), st, B);
  TBG_KLAUNCH(k_hash_clear_x2, grid, dim3(kBlock), st, B);
  TBG_KLAUNCH(k_hash_clear_fin, grid, dim3(kBlock), st, B);
}

}  // namespace tbg
