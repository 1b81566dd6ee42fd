// Montgomery's trick across a workgroup: ONE field inversion for every value
// the workgroup's threads hold, instead of one per thread.
//
// On a SIMD machine a per-thread inversion (fp_inv: ~378 squarings + ~100
// products) costs the same wave time whether one lane or 64 need it, so the
// trick pays only across waves: the workgroup's WAVES waves scan their
// values, ONE wave inverts the single product, and everybody recovers its
// own inverse from prefix and suffix products:
//
//   wave scans (registers, lane shuffles): inclusive prefix P_t and suffix
//     S_t of z within the wave (log2(64) = 6 products each), T_w = P_63;
//   wave 0 (LDS): the WAVES wave totals by the serial trick -- prefix
//     products, one fp_inv of their product, back-substitution -- into
//     1 / T_w for every wave;
//   thread t:  1 / z_t = P_{t-1} S_{t+1} / T_w    (2 products).
//
// Per value 14 products + (3 WAVES + one inversion) / (64 WAVES) instead of
// one inversion.  Absent values (the point at infinity, a thread past the
// end) take part as 1 and get 1 back; every thread of the workgroup must
// call it (barriers).  Used by the to-affine conversions of the per-item
// kernels (k_hash_affine, k_rlc_duty_sum, k_aggregate, k_decode_pubkeys,
// k_pubkey_tables) and the SSWU denominator of k_hash_map.  The host build
// runs the same steps over an array (batch_inv_emulate) for the CPU tests.
#pragma once
#include "bls_curve.h"

namespace tbg {

// One wave per workgroup by default: with three launches in flight, a
// workgroup of four waves needs four free SIMD slots on one CU at once and
// waits behind the other launches' one-wave workgroups (a 0.7 ms
// k_hash_affine took 30 ms inside a 20-step run, rocprof trace in
// profiles/r03/final4/); one-wave groups invert 4x as often but start at
// once: 2.18-2.21 M vs 2.12-2.16 M DV-duties/s (profiles/r03/prio/).
#ifndef TBG_BINV_WAVES
#define TBG_BINV_WAVES 1
#endif
constexpr int BINV_WAVES = TBG_BINV_WAVES;    // waves per workgroup of the batched kernels
constexpr int BINV_BLOCK = 64 * BINV_WAVES;   // their workgroup size

#if defined(__HIP__)  // (device code; declared in both passes of a .hip unit)
__device__ __forceinline__ Fp fp_shfl_up(const Fp& a, int d) {
  Fp r;
#pragma unroll
  for (int j = 0; j < NL; ++j) r.l[j] = (uint32_t)__shfl_up((int)a.l[j], d, 64);
  return r;
}
__device__ __forceinline__ Fp fp_shfl_down(const Fp& a, int d) {
  Fp r;
#pragma unroll
  for (int j = 0; j < NL; ++j) r.l[j] = (uint32_t)__shfl_down((int)a.l[j], d, 64);
  return r;
}

// 1 / z for present values (z != 0, any bound fp_mul accepts); 1 otherwise.
// Call from every thread of a workgroup of exactly WAVES waves.
template <int WAVES>
__device__ Fp block_batch_inv(const Fp& z_in, bool present) {
  __shared__ Fp s_tot[WAVES];  // wave totals, then their inverses
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const Fp one = fp_one();
  const Fp z = fp_select(present, z_in, one);
  // inclusive prefix / suffix products within the wave
  Fp pre = z, suf = z;
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const Fp o = fp_shfl_up(pre, d);
    if (lane >= d) pre = fp_mul(pre, o);
  }
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    const Fp o = fp_shfl_down(suf, d);
    if (lane + d < 64) suf = fp_mul(suf, o);
  }
  if (lane == 63) s_tot[w] = pre;
  __syncthreads();
  if (w == 0) {
    // serial trick over the WAVES totals, lane-uniform (every lane of wave 0
    // runs it; lane 0 stores; the totals are in registers before any store)
    Fp tot[WAVES], acc[WAVES];
#pragma unroll
    for (int k = 0; k < WAVES; ++k) tot[k] = s_tot[k];
    acc[0] = tot[0];
#pragma unroll
    for (int k = 1; k < WAVES; ++k) acc[k] = fp_mul(acc[k - 1], tot[k]);
    Fp inv = fp_inv(acc[WAVES - 1]);
    Fp out[WAVES];
#pragma unroll
    for (int k = WAVES - 1; k > 0; --k) {
      out[k] = fp_mul(inv, acc[k - 1]);
      inv = fp_mul(inv, tot[k]);
    }
    out[0] = inv;
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < WAVES; ++k) s_tot[k] = out[k];
    }
  }
  __syncthreads();
  const Fp pex = fp_shfl_up(pre, 1), sex = fp_shfl_down(suf, 1);
  Fp r = s_tot[w];
  if (lane > 0) r = fp_mul(r, pex);
  if (lane < 63) r = fp_mul(r, sex);
  return fp_select(present, r, one);
}

// Fp2: 1 / a = conj(a) / N(a), N(a) = a0^2 + a1^2 in Fp (batched).
template <int WAVES>
__device__ Fp2 block_batch_inv2(const Fp2& a, bool present) {
  const Fp t = block_batch_inv<WAVES>(fp_mul2(a.c0, a.c0, a.c1, a.c1), present);
  return {fp_mul(a.c0, t), fp_mul(fp_neg(a.c1), t)};
}

// Jacobian -> affine with the inversion batched over the workgroup; false
// (and `out` untouched) for the point at infinity.  Every thread calls it.
template <int WAVES>
__device__ bool block_jac_to_aff(const Jac<Fp>& p, bool want, Aff<Fp>& out) {
  const bool present = want && !jac_is_inf(p);
  const Fp zi = block_batch_inv<WAVES>(p.Z, present);
  if (!present) return false;
  const Fp zi2 = fp_sqr(zi);
  out.x = fp_mul(p.X, zi2);
  out.y = fp_mul(p.Y, fp_mul(zi2, zi));
  return true;
}
template <int WAVES>
__device__ bool block_jac_to_aff(const Jac<Fp2>& p, bool want, Aff<Fp2>& out) {
  const bool present = want && !jac_is_inf(p);
  const Fp2 zi = block_batch_inv2<WAVES>(p.Z, present);
  if (!present) return false;
  const Fp2 zi2 = fp2_sqr(zi);
  out.x = fp2_mul(p.X, zi2);
  out.y = fp2_mul(p.Y, fp2_mul(zi2, zi));
  return true;
}
#endif

// Host emulation of block_batch_inv over n values in workgroups of
// 64 * waves (tests/hostcheck): the same wave scans, wave-total trick and
// back-substitution, lane by lane.
inline void batch_inv_emulate(const Fp* z_in, const bool* present, Fp* out, int n, int waves) {
  const int block = 64 * waves;
  const Fp one = fp_one();
  for (int b0 = 0; b0 < n; b0 += block) {
    Fp z[1024], pre[1024], suf[1024], tot_inv[16];
    for (int t = 0; t < block; ++t) z[t] = (b0 + t < n && present[b0 + t]) ? z_in[b0 + t] : one;
    for (int w = 0; w < waves; ++w) {
      Fp* P = pre + 64 * w;
      Fp* S = suf + 64 * w;
      const Fp* Z = z + 64 * w;
      for (int l = 0; l < 64; ++l) P[l] = S[l] = Z[l];
      for (int d = 1; d < 64; d <<= 1) {  // Hillis-Steele, as the shuffles do it
        Fp np[64], ns[64];
        for (int l = 0; l < 64; ++l) {
          np[l] = l >= d ? fp_mul(P[l], P[l - d]) : P[l];
          ns[l] = l + d < 64 ? fp_mul(S[l], S[l + d]) : S[l];
        }
        for (int l = 0; l < 64; ++l) { P[l] = np[l]; S[l] = ns[l]; }
      }
    }
    Fp acc[16];
    acc[0] = pre[63];
    for (int k = 1; k < waves; ++k) acc[k] = fp_mul(acc[k - 1], pre[64 * k + 63]);
    Fp inv = fp_inv(acc[waves - 1]);
    for (int k = waves - 1; k > 0; --k) {
      tot_inv[k] = fp_mul(inv, acc[k - 1]);
      inv = fp_mul(inv, pre[64 * k + 63]);
    }
    tot_inv[0] = inv;
    for (int t = 0; t < block && b0 + t < n; ++t) {
      const int w = t / 64, l = t % 64;
      Fp r = tot_inv[w];
      if (l > 0) r = fp_mul(r, pre[t - 1]);
      if (l < 63) r = fp_mul(r, suf[t + 1]);
      out[b0 + t] = present[b0 + t] ? r : one;
    }
  }
}

}  // namespace tbg
