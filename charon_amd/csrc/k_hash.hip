// hash_to_G2 per distinct message (the H(m) of SigEth2.Verify, tss.go:190-197),
// in kernels split so each phase runs at the occupancy its own footprint
// allows (bls_pair.h):
//   k_hash_map     one lane per message: expand_message_xmd, hash_to_field,
//                  the two SSWU denominators and their inverse (batched over
//                  the workgroup); each map's u and x1 into h_jac;
//   k_hash_sswu    one lane per MAP (two per message): g(x1), the square
//                  root (two Fp exponentiations), the 3-isogeny -- Q0 and Q1
//                  (Jacobian) in place in h_jac (k_hash_clear_x1 adds them);
//   k_hash_clear   a lane pair per message: Budroni-Pintore cofactor clearing;
//   k_hash_affine  one lane per message: to affine (inversion batched over
//                  the workgroup), status.
// The one-kernel map (both maps per lane, the root and isogeny out of line)
// wrote ~6.4 KB of callee-saved registers to scratch per message and ran
// 2,500 two-map waves per 160k messages.
#define TBG_ADD_DBL_INLINE 1
#include "tbls_launch.h"
#include "bls_h2c.h"
#include "bls_batchinv.h"

namespace tbg {

// A map's input in its h_jac slot until k_hash_sswu overwrites it with the
// point: X = u, Y = x1, Z.c0.l[0] = 1 when the batched inverse exists.
__device__ __forceinline__ void sswu_in_store(G2J& s, const Fp2& u, const Fp2& x1, bool ok) {
  s.X = u;
  s.Y = x1;
  s.Z.c0.l[0] = ok ? 1u : 0u;
}

// The SSWU denominators' inversion is batched over the workgroup
// (Montgomery's trick, bls_batchinv.h): one field inversion per BINV_BLOCK
// messages instead of one per message.
__global__ void __launch_bounds__(BINV_BLOCK, TBG_DECODE_WAVES) k_hash_map(DevBatch B) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = m < B.n_msgs;
  Fp2 u0 = fp2_zero(), u1 = fp2_zero();
  if (in) {
    const uint32_t off = B.msg_off[m], len = B.msg_off[m + 1] - off;
    hash_to_field_fp2(B.msgs + off, len, u0, u1);
  }
  SswuPair w;
  const Fp2 dd = sswu_pair_den(u0, u1, w);
  const bool ok = in && !fp2_is_zero(dd);
  const Fp2 di = block_batch_inv2<BINV_WAVES>(dd, ok);  // every thread of the workgroup
  if (!in) return;
  sswu_in_store(B.h_jac[m], u0, sswu_x1(fp2_mul(w.den[1], di)), ok);
  sswu_in_store(B.h_jac[B.n_msgs + m], u1, sswu_x1(fp2_mul(w.den[0], di)), ok);
}

// (SlotKeep, bls_tower.h: fp2_sqrt_or_z_in's g(x1) waits in the slot's Z)

// One map per lane, everything inline (no call: no callee-saved registers
// through scratch).  u, x1 and g(x1) wait in the slot while the root's two
// exponentiations run (window width SSWU_WIN, bls_h2c.h), and
// the isogeny writes each coordinate as soon as it is formed.  The
// exceptional inputs (no batched inverse, or a root the closed form does not
// cover; ~2^-380 per hash) take the reference map, which gives the same
// affine point.
__global__ void TBG_LAUNCH_N(TBG_DECODE_WAVES) k_hash_sswu(DevBatch B) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // h_jac slot: map t / n_msgs of message t % n_msgs
  if (t >= 2 * B.n_msgs) return;
  G2J& s = B.h_jac[t];
  bool done = s.Z.c0.l[0] != 0;
  Fp2 r;
  bool sq = false;
  if (done) done = fp2_sqrt_or_z_in<SSWU_WIN>(sswu_gx(s.Y), r, sq, SlotKeep{&s.Z});
  __asm__ __volatile__("" ::: "memory");
  if (done) {
    Fp2 x, y;
    sswu_xy(s.X, s.Y, r, sq, x, y);
    iso3_emit(x, y, s);
  } else {
    s = map_to_curve_g2(s.X);
  }
}

__global__ void __launch_bounds__(BINV_BLOCK, TBG_DECODE_WAVES) k_hash_affine(DevBatch B) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = m < B.n_msgs;
  const G2J p = in ? B.h_jac[m] : jac_inf<Fp2>();
  G2A a;
  const bool ok = block_jac_to_aff<BINV_WAVES>(p, in, a);  // every thread of the workgroup
  if (!in) return;
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  B.h_aff[m] = a;
  B.h_status[m] = ok ? 0 : 1;
}

void launch_hash_msgs(const DevBatch& B, hipStream_t st) {
  if (!B.n_msgs) return;
  const dim3 grid((B.n_msgs + BINV_BLOCK - 1) / BINV_BLOCK);
  TBG_KLAUNCH(k_hash_map, grid, dim3(BINV_BLOCK), st, B);
  TBG_KLAUNCH(k_hash_sswu, grid_for(2 * B.n_msgs), dim3(kBlock), st, B);
  launch_hash_clear(B, st);  // k_hash_clear.hip
  TBG_KLAUNCH(k_hash_affine, grid, dim3(BINV_BLOCK), st, B);
}

}  // namespace tbg
