// Plain BLS aggregation (sums with all coefficients 1) -- the multi-signature
// side of the DKG and of the cluster lock:
//   AggregateSignatures / AggregatePublicKeys   dkg/dkg.go:466-476 (aggLockHashSig)
//   FastAggregateVerify(pubshares, hash, sig)    cluster/lock.go:155-177
// A set's items are summed in chunks of SUM_CHUNK, one lane per chunk (the
// sum is latency-bound: a lock's pubshare set can hold thousands of keys),
// then one lane per set adds its chunk sums and compresses the result.
#include "tbls_launch.h"

namespace tbg {

constexpr uint32_t SUM_CHUNK = 32;

// chunk k of set s covers items off[s] + (k - chunk_first[s]) * SUM_CHUNK ...
__device__ __forceinline__ void sum_chunk_range(const uint32_t* off, const uint32_t* chunk_first, uint32_t s, uint32_t k,
                                                uint32_t& lo, uint32_t& hi) {
  lo = off[s] + (k - chunk_first[s]) * SUM_CHUNK;
  hi = min(lo + SUM_CHUNK, off[s + 1]);
}

// G1: resident keys by id.  A key that is unknown or failed to decode marks
// its set (every writer stores the same value).
__global__ void TBG_LAUNCH k_sum_g1_chunks(const G1A* table, const int32_t* pk_status, uint32_t n_pk,
                                           const uint32_t* ids, const uint32_t* off, const uint32_t* chunk_first,
                                           const uint32_t* chunk_set, uint32_t n_chunks, G1J* part, int32_t* set_bad) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_chunks) return;
  const uint32_t s = chunk_set[k];
  uint32_t lo, hi;
  sum_chunk_range(off, chunk_first, s, k, lo, hi);
  G1J acc = jac_inf<Fp>();
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t id = ids[i];
    if (id >= n_pk || pk_status[id] != DEC_OK) {
      set_bad[s] = 1;
      continue;
    }
    acc = jac_add_aff(acc, table[id]);
  }
  part[k] = acc;
}

// G2: 96-byte signatures, decoded here (flags, field, curve, subgroup).  The
// encoding of the identity decodes to the identity and adds nothing.
__global__ void TBG_LAUNCH k_sum_g2_chunks(const uint8_t* sigs96, const uint32_t* off, const uint32_t* chunk_first,
                                           const uint32_t* chunk_set, uint32_t n_chunks, G2J* part, int32_t* set_bad,
                                           int32_t* sig_status) {
  uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_chunks) return;
  const uint32_t s = chunk_set[k];
  uint32_t lo, hi;
  sum_chunk_range(off, chunk_first, s, k, lo, hi);
  G2J acc = jac_inf<Fp2>();
  for (uint32_t i = lo; i < hi; ++i) {
    G2A a;
    int32_t st = g2_decompress(sigs96 + 96ull * i, a);
    sig_status[i] = st == DEC_OK ? TBG_PS_NOT_VERIFIED : st == DEC_IDENTITY ? TBG_PS_ERR_IDENTITY : st;
    if (st == DEC_OK) acc = jac_add_aff(acc, a);
    else if (st != DEC_IDENTITY) set_bad[s] = 1;
  }
  part[k] = acc;
}

template <class F>
__device__ __forceinline__ Jac<F> sum_parts(const Jac<F>* part, uint32_t k0, uint32_t k1) {
  Jac<F> acc = jac_inf<F>();
  for (uint32_t k = k0; k < k1; ++k) acc = jac_add(acc, part[k]);
  return acc;
}

__global__ void TBG_LAUNCH k_sum_g1_sets(const G1J* part, const uint32_t* chunk_first, uint32_t n_sets,
                                         const int32_t* set_bad, uint8_t* out48, int32_t* status) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  G1A a;
  const bool ok = !set_bad[s] && jac_to_aff(sum_parts(part, chunk_first[s], chunk_first[s + 1]), a);
  g1_compress(a, !ok, out48 + 48ull * s);
  if (set_bad[s]) {  // not a point: the 48 bytes of a failed set do not decode
    for (int j = 0; j < 48; ++j) out48[48ull * s + j] = 0;
  }
  status[s] = set_bad[s] ? TBG_DS_DECODE : ok ? TBG_DS_OK : TBG_DS_AGG_IDENTITY;
}

__global__ void TBG_LAUNCH k_sum_g2_sets(const G2J* part, const uint32_t* chunk_first, uint32_t n_sets,
                                         const int32_t* set_bad, uint8_t* out96, int32_t* status) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sets) return;
  G2A a;
  const bool ok = !set_bad[s] && jac_to_aff(sum_parts(part, chunk_first[s], chunk_first[s + 1]), a);
  g2_compress(a, !ok, out96 + 96ull * s);
  if (set_bad[s]) {
    for (int j = 0; j < 96; ++j) out96[96ull * s + j] = 0;
  }
  status[s] = set_bad[s] ? TBG_DS_DECODE : ok ? TBG_DS_OK : TBG_DS_AGG_IDENTITY;
}

void launch_sum_g1(const G1A* table, const int32_t* pk_status, uint32_t n_pk, const uint32_t* ids, const SumPlan& p,
                   uint8_t* out48, int32_t* status, hipStream_t st) {
  if (p.n_chunks)
    TBG_KLAUNCH(k_sum_g1_chunks, grid_for(p.n_chunks), dim3(kBlock), st, table, pk_status, n_pk, ids, p.off,
                p.chunk_first, p.chunk_set, p.n_chunks, (G1J*)p.part, p.set_bad);
  TBG_KLAUNCH(k_sum_g1_sets, grid_for(p.n_sets), dim3(kBlock), st, (const G1J*)p.part, p.chunk_first, p.n_sets,
              p.set_bad, out48, status);
}

void launch_sum_g2(const uint8_t* sigs96, const SumPlan& p, uint8_t* out96, int32_t* status, int32_t* sig_status,
                   hipStream_t st) {
  if (p.n_chunks)
    TBG_KLAUNCH(k_sum_g2_chunks, grid_for(p.n_chunks), dim3(kBlock), st, sigs96, p.off, p.chunk_first, p.chunk_set,
                p.n_chunks, (G2J*)p.part, p.set_bad, sig_status);
  TBG_KLAUNCH(k_sum_g2_sets, grid_for(p.n_sets), dim3(kBlock), st, (const G2J*)p.part, p.chunk_first, p.n_sets,
              p.set_bad, out96, status);
}

uint32_t sum_chunk_size() { return SUM_CHUNK; }

}  // namespace tbg
