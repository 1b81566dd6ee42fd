// Decode kernels: 48-byte G1 pubkeys (tblsconv.KeyFromBytes, tblsconv.go:30-37)
// and 96-byte G2 signatures (tblsconv.SigFromCore, tblsconv.go:125-132).
// The P == Q case of the mixed addition doubles inline (bls_curve.h): no
// out-of-line call inside the kernels' point loops.
#define TBG_ADD_DBL_INLINE 1
#ifndef TBG_SCHED_FENCE
#define TBG_SCHED_FENCE 1  // products in program order: fits the pair kernel in 256 VGPRs (bls_field.h)
#endif
#include "tbls_launch.h"
#include "bls_curve.h"
#include "bls_pair.h"
#include "bls_batchinv.h"

namespace tbg {

// Resident table entry: the key and [x]key (x the curve parameter), so the
// RLC scalars of k_rlc.hip can be applied in base-x digits with the G1
// endomorphism ([x^2] = -phi on G1) instead of 64-bit double-and-add.
// ([x]key's affine conversion batched over the workgroup, bls_batchinv.h)
__global__ void __launch_bounds__(BINV_BLOCK) k_decode_pubkeys(const uint8_t* pk48, uint32_t n, G1A* out, G1A* out_x,
                                                               int32_t* status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < n;
  G1A a{fp_zero(), fp_zero()}, ax = a;
  int32_t st = DEC_ERR_FLAGS;
  G1J xa = jac_inf<Fp>();
  if (in) {
    uint8_t b[48];
    for (int j = 0; j < 48; ++j) b[j] = pk48[48ull * i + j];
    st = g1_decompress(b, a);
    if (st == DEC_OK) xa = jac_neg(jac_mul_xabs(jac_from_aff(a)));
  }
  const bool ok = block_jac_to_aff<BINV_WAVES>(xa, in && st == DEC_OK, ax);  // every thread of the workgroup
  if (!in) return;
  if (st != DEC_OK || !ok) {
    if (st == DEC_OK) st = DEC_IDENTITY;  // unreachable for a prime-order point
    a.x = fp_zero();
    a.y = fp_zero();
    ax = a;
  }
  out[i] = a;
  out_x[i] = ax;
  status[i] = st;
}

// Decode in two kernels so each runs at the occupancy its own register
// footprint allows (one kernel would take the maximum of both):
//   k_decode_sigs    one lane per signature: flags, field, Fp2 square root
//                    (Fp exponentiations: small state, several waves per SIMD);
//   k_subgroup_sigs  one lane PAIR per decoded signature: psi(a) == [x] a with
//                    the Fp2 coordinates split over the pair (bls_pair.h).
__global__ void TBG_LAUNCH_N(TBG_DECODE_WAVES) k_decode_sigs(DevBatch B) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // The chain's first kernel zeroes its work-list counters and level 0's
  // bucket sizes (a runtime memset kernel queued behind other streams' waves
  // held each chain for ~2 ms in the pipelined bench)
  if (i < CNT_WORDS) B.counters[i] = 0;
  if (B.rlc_batch && i <= MSM_BUCKETS) B.msm_off[i] = 0;
  if (i >= B.n_partials) return;
  // decoded from the input bytes straight into the output slot: x and the
  // root's input wait there while the exponentiations run (the root inline:
  // the out-of-line form saved its callee-saved registers to scratch on
  // every call)
  G2A& a = B.sig_aff[i];
  int32_t st = g2_decompress_t<true, false>(B.sigs + 96ull * i, a, SlotKeep{&a.y});
  if (st == DEC_IDENTITY) st = TBG_PS_ERR_IDENTITY;
  if (st != DEC_OK) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  B.partial_status[i] = (st == DEC_OK) ? TBG_PS_NOT_VERIFIED : st;
}

__global__ void TBG_LAUNCH_N(TBG_PAIR_WAVES) k_subgroup_sigs(DevBatch B) {
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 1;  // both lanes of a pair take the same branches
  if (i >= B.n_partials) return;
  if (B.partial_status[i] != TBG_PS_NOT_VERIFIED) return;
  if (B.sgb && !B.sgb_bad[i / B.sgb_m]) return;  // every combination of its group is in G2 (k_sgb.hip)
  const Aff<Fp2x> a = px_load(B.sig_aff[i]);
  bool exc = false;
  bool ok = g2_in_subgroup_aff_g(a, exc);
  if (exc) {
    // an addition of [|x|] a met its doubling case (only for points of tiny
    // order, i.e. crafted signatures): decide on the single-lane reference
    // path, out of line so the loop above keeps its registers
    ok = g2_in_subgroup(jac_from_aff(B.sig_aff[i]));
  }
  if (!ok && pair_par() == 0) {
    B.partial_status[i] = TBG_PS_ERR_SUBGROUP;
    B.sig_aff[i] = G2A{fp2_zero(), fp2_zero()};
  }
}

void launch_decode_pubkeys(const uint8_t* pk48, uint32_t n, G1A* out, G1A* out_x, int32_t* status, hipStream_t st) {
  if (n) TBG_KLAUNCH(k_decode_pubkeys, dim3((n + BINV_BLOCK - 1) / BINV_BLOCK), dim3(BINV_BLOCK), st, pk48, n, out,
                     out_x, status);
}
void launch_decode_sigs(const DevBatch& B, hipStream_t st) {
  // at least enough lanes to zero the counters (and level 0's bucket sizes)
  uint32_t lanes = B.n_partials > CNT_WORDS ? B.n_partials : CNT_WORDS;
  if (B.rlc_batch && lanes < MSM_BUCKETS + 1) lanes = MSM_BUCKETS + 1;
  TBG_KLAUNCH(k_decode_sigs, grid_for(lanes), dim3(kBlock), st, B);
  launch_subgroup_batch(B, st);
  if (B.n_partials) TBG_KLAUNCH(k_subgroup_sigs, grid_for(2 * B.n_partials), dim3(kBlock), st, B);
}

}  // namespace tbg
