// Host-side view of the engine's kernels: the device batch layout and one
// launcher per kernel (each defined next to its kernel in a k_*.hip
// translation unit, so the units compile in parallel and no relocatable
// device code is needed).
#pragma once
#include <hip/hip_runtime.h>
#include "bls_curve.h"
#include "../../include/tbls_gpu.h"

namespace tbg {

constexpr int kBlock = 64;
inline dim3 grid_for(uint32_t n) { return dim3((n + kBlock - 1) / kBlock); }

// Device-side layout of one batch (all pointers into device memory).
struct DevBatch {
  uint32_t op, n_duties, n_partials, n_msgs;
  const uint8_t* msgs;
  const uint32_t* msg_off;
  const uint32_t* duty_msg;
  const uint32_t* duty_first;
  const uint32_t* duty_threshold;
  const uint32_t* partial_duty;
  const uint8_t* sigs;
  const uint8_t* identifiers;
  const uint32_t* pubkey_ids;
  // work buffers
  G2A* sig_aff;
  G2A* h_aff;
  int32_t* h_status;
  uint32_t* lam;       // [n_partials][8] scalar words
  uint32_t* sig_lines;  // [n_partials][LINES_WORDS] Miller lines of each signature (-g1 folded in)
  uint32_t* h_lines;    // [n_msgs][LINES_WORDS] Miller lines of each H(m) (G1 factor left out)
  // outputs
  int32_t* partial_status;
  int32_t* duty_status;
  uint8_t* agg;        // [n_duties][96]
};

// Participation of a partial in its duty's aggregate.
TBG_HD bool participates(uint32_t op, int32_t st) {
  return op == TBG_OP_VERIFY_AGGREGATE ? (st == TBG_PS_VALID) : (st == TBG_PS_NOT_VERIFIED);
}

// launchers (asynchronous on `st`)
void launch_decode_pubkeys(const uint8_t* pk48, uint32_t n, G1A* out, int32_t* status, hipStream_t st);
void launch_decode_sigs(const DevBatch& B, hipStream_t st);
void launch_hash_msgs(const DevBatch& B, hipStream_t st);
void launch_lines(const DevBatch& B, hipStream_t st_sig, hipStream_t st_h);
void launch_verify(const DevBatch& B, const G1A* pk_aff, const int32_t* pk_status, uint32_t n_pk, hipStream_t st);
void launch_lagrange(const DevBatch& B, hipStream_t st);
void launch_aggregate(const DevBatch& B, hipStream_t st);
void launch_sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* pk48, hipStream_t st);
void launch_sign(const uint8_t* sk32, const uint32_t* item_msg, uint32_t n, const G2A* h_aff, const int32_t* h_status,
                 uint8_t* sig96, hipStream_t st);

}  // namespace tbg
