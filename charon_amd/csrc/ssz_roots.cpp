// Batched SSZ hash_tree_root and signing roots on the host (include/tbls_ssz.h).
//
// Every duty the hot path verifies is signed over
//   signing_root = hash_tree_root(SigningData{hash_tree_root(object), domain})
// (reference eth2util/signing/signing.go:73-85 over core/signeddata.go's
// MessageRoot methods).  For the fixed-size containers of the duty types the
// root is a handful of 64-byte SHA-256 compressions -- two blocks each, the
// second always the constant padding block of a 64-byte message -- so a batch
// is hashed here in one pass over contiguous SSZ bytes, split into ranges
// over host threads, instead of one go-ssz hasher walk per object.
//
// Merkleization (consensus-specs ssz/simple-serialize.md): basic values are
// packed little-endian into 32-byte chunks, a container's field roots are the
// leaves of a binary tree padded with zero subtrees to the next power of two,
// a byte vector longer than 32 bytes is its own chunk tree.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/tbls_gpu.h"
#include "../../include/tbls_ssz.h"

namespace {

// ------------------------------------------------------------------ SHA-256
constexpr uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
constexpr uint32_t IV256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                               0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
inline uint32_t load_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

void compress_portable(uint32_t st[8], const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i) w[i] = load_be32(blk + 4 * i);
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// x86 SHA extensions: two rounds per sha256rnds2, the state held as ABEF /
// CDGH, the schedule W[g] = msg2(msg1(W[g-4], W[g-3]) + alignr(W[g-1], W[g-2]), W[g-1]).
__attribute__((target("sha,sse4.1"))) void compress_shani(uint32_t st[8], const uint8_t* blk) {
  const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i t = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&st[0]), 0xB1);  // CDAB
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&st[4]), 0x1B); // EFGH
  __m128i s0 = _mm_alignr_epi8(t, s1, 8);                                        // ABEF
  s1 = _mm_blend_epi16(s1, t, 0xF0);                                             // CDGH
  const __m128i save0 = s0, save1 = s1;
  __m128i w[4];
  for (int g = 0; g < 16; ++g) {
    __m128i& wg = w[g & 3];
    if (g < 4) {
      wg = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(blk + 16 * g)), bswap);
    } else {
      const __m128i w1 = w[(g - 1) & 3], w2 = w[(g - 2) & 3], w3 = w[(g - 3) & 3];
      wg = _mm_sha256msg2_epu32(_mm_add_epi32(_mm_sha256msg1_epu32(wg, w3), _mm_alignr_epi8(w1, w2, 4)), w1);
    }
    __m128i m = _mm_add_epi32(wg, _mm_loadu_si128((const __m128i*)&K256[4 * g]));
    s1 = _mm_sha256rnds2_epu32(s1, s0, m);
    s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(m, 0x0E));
  }
  s0 = _mm_add_epi32(s0, save0);
  s1 = _mm_add_epi32(s1, save1);
  t = _mm_shuffle_epi32(s0, 0x1B);            // FEBA
  s1 = _mm_shuffle_epi32(s1, 0xB1);           // DCHG
  s0 = _mm_blend_epi16(t, s1, 0xF0);          // DCBA
  s1 = _mm_alignr_epi8(s1, t, 8);             // HGFE
  _mm_storeu_si128((__m128i*)&st[0], s0);
  _mm_storeu_si128((__m128i*)&st[4], s1);
}

using CompressFn = void (*)(uint32_t*, const uint8_t*);
CompressFn pick_compress() {
  const char* e = getenv("TBG_SHA_PORTABLE");
  if (e && e[0] == '1') return compress_portable;
  __builtin_cpu_init();
  return __builtin_cpu_supports("sha") ? compress_shani : compress_portable;
}
const CompressFn compress = pick_compress();

// The padding block of a 64-byte message: 0x80, zeros, bit length 512.
struct Pad64 {
  uint8_t b[64];
  Pad64() {
    memset(b, 0, 64);
    b[0] = 0x80;
    b[62] = 0x02;
  }
};
const Pad64 PAD64;

inline void store_state(const uint32_t st[8], uint8_t* out) {
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8);
    out[4 * i + 3] = (uint8_t)st[i];
  }
}

// out = SHA-256(a || b), a and b 32 bytes each (may alias out).
inline void hash_pair(const uint8_t* a, const uint8_t* b, uint8_t* out) {
  uint8_t blk[64];
  memcpy(blk, a, 32);
  memcpy(blk + 32, b, 32);
  uint32_t st[8];
  memcpy(st, IV256, sizeof(st));
  compress(st, blk);
  compress(st, PAD64.b);
  store_state(st, out);
}

// ------------------------------------------------------------ merkleization
typedef uint8_t Chunk[32];

struct ZeroHashes {
  Chunk z[8];  // z[k] = root of a zero subtree of 2^k chunks
  ZeroHashes() {
    memset(z[0], 0, 32);
    for (int k = 1; k < 8; ++k) hash_pair(z[k - 1], z[k - 1], z[k]);
  }
};
const ZeroHashes ZH;

// Root of `n` leaves (n >= 1) padded to the next power of two, in place.
void merkleize(Chunk* leaves, uint32_t n, uint8_t* root) {
  int depth = 0;
  while ((1u << depth) < n) ++depth;
  for (int lvl = 0; lvl < depth; ++lvl) {
    uint32_t m = (n + 1) / 2;
    for (uint32_t i = 0; i < m; ++i) {
      const uint8_t* r = 2 * i + 1 < n ? leaves[2 * i + 1] : ZH.z[lvl];
      hash_pair(leaves[2 * i], r, leaves[i]);
    }
    n = m;
  }
  memcpy(root, leaves[0], 32);
}

inline void leaf_u64(const uint8_t* le8, uint8_t* c) {
  memcpy(c, le8, 8);
  memset(c + 8, 0, 24);
}
inline void leaf_bytes(const uint8_t* p, uint32_t len, uint8_t* c) {  // len <= 32
  memcpy(c, p, len);
  memset(c + len, 0, 32 - len);
}
// hash_tree_root of a byte vector of `len` bytes (Bytes48 pubkey, Bytes96 signature).
void root_bytes(const uint8_t* p, uint32_t len, uint8_t* out) {
  Chunk c[4];
  uint32_t n = (len + 31) / 32;
  for (uint32_t i = 0; i < n; ++i) leaf_bytes(p + 32 * i, std::min<uint32_t>(32, len - 32 * i), c[i]);
  merkleize(c, n, out);
}
void root_checkpoint(const uint8_t* p, uint8_t* out) {  // epoch 8 | root 32
  Chunk e;
  leaf_u64(p, e);
  hash_pair(e, p + 8, out);
}

const uint32_t SIZES[TBG_SSZ_KINDS] = {32, 8, 128, 16, 16, 84, 88, 184, 36, 64, 40};

void object_root(uint32_t kind, const uint8_t* p, uint8_t* out) {
  Chunk c[8];
  switch (kind) {
    case TBG_SSZ_ROOT:
      memcpy(out, p, 32);
      return;
    case TBG_SSZ_UINT64:
      leaf_u64(p, out);
      return;
    case TBG_SSZ_ATTESTATION_DATA:  // slot, index, beacon_block_root, source, target
      leaf_u64(p, c[0]);
      leaf_u64(p + 8, c[1]);
      memcpy(c[2], p + 16, 32);
      root_checkpoint(p + 48, c[3]);
      root_checkpoint(p + 88, c[4]);
      merkleize(c, 5, out);
      return;
    case TBG_SSZ_VOLUNTARY_EXIT:      // epoch, validator_index
    case TBG_SSZ_SYNC_AGG_SELECTION:  // slot, subcommittee_index
      leaf_u64(p, c[0]);
      leaf_u64(p + 8, c[1]);
      hash_pair(c[0], c[1], out);
      return;
    case TBG_SSZ_VALIDATOR_REGISTRATION:  // fee_recipient[20], gas_limit, timestamp, pubkey[48]
      leaf_bytes(p, 20, c[0]);
      leaf_u64(p + 20, c[1]);
      leaf_u64(p + 28, c[2]);
      root_bytes(p + 36, 48, c[3]);
      merkleize(c, 4, out);
      return;
    case TBG_SSZ_DEPOSIT_MESSAGE:  // pubkey[48], withdrawal_credentials[32], amount
      root_bytes(p, 48, c[0]);
      memcpy(c[1], p + 48, 32);
      leaf_u64(p + 80, c[2]);
      merkleize(c, 3, out);
      return;
    case TBG_SSZ_DEPOSIT_DATA:  // + signature[96]
      root_bytes(p, 48, c[0]);
      memcpy(c[1], p + 48, 32);
      leaf_u64(p + 80, c[2]);
      root_bytes(p + 88, 96, c[3]);
      merkleize(c, 4, out);
      return;
    case TBG_SSZ_FORK_DATA:  // current_version[4], genesis_validators_root
      leaf_bytes(p, 4, c[0]);
      hash_pair(c[0], p + 4, out);
      return;
    case TBG_SSZ_SIGNING_DATA:  // object_root, domain
      hash_pair(p, p + 32, out);
      return;
    case TBG_SSZ_CHECKPOINT:
      root_checkpoint(p, out);
      return;
  }
}

// Run body(lo, hi) over [0, n) split into contiguous ranges on up to
// n_threads threads (small batches stay on the caller's thread).
template <class F>
void parallel_ranges(uint32_t n, uint32_t n_threads, F body) {
  if (n_threads == 0) n_threads = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  const uint32_t per = 2048;  // below this many objects per thread, threads cost more than they save
  n_threads = std::max(1u, std::min(n_threads, (n + per - 1) / per));
  if (n_threads == 1) {
    body(0u, n);
    return;
  }
  std::vector<std::thread> ts;
  const uint32_t step = (n + n_threads - 1) / n_threads;
  for (uint32_t t = 1; t < n_threads; ++t) {
    uint32_t lo = t * step, hi = std::min(n, lo + step);
    if (lo < hi) ts.emplace_back(body, lo, hi);
  }
  body(0u, std::min(n, step));
  for (auto& th : ts) th.join();
}

}  // namespace

extern "C" {

uint32_t tbg_ssz_size(uint32_t kind) { return kind < TBG_SSZ_KINDS ? SIZES[kind] : 0; }

int tbg_ssz_roots(uint32_t kind, const uint8_t* ssz, uint32_t n, uint8_t* roots32, uint32_t n_threads) {
  if (kind >= TBG_SSZ_KINDS || (n && (!ssz || !roots32))) return TBG_E_INVALID_ARG;
  const uint32_t sz = SIZES[kind];
  parallel_ranges(n, n_threads, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; ++i) object_root(kind, ssz + (size_t)sz * i, roots32 + 32ull * i);
  });
  return TBG_OK;
}

int tbg_compute_domain(const uint8_t* type4, const uint8_t* version4, const uint8_t* gvr32, uint8_t* domain32) {
  if (!type4 || !version4 || !gvr32 || !domain32) return TBG_E_INVALID_ARG;
  uint8_t fd[36], root[32];
  memcpy(fd, version4, 4);
  memcpy(fd + 4, gvr32, 32);
  object_root(TBG_SSZ_FORK_DATA, fd, root);
  memcpy(domain32, type4, 4);
  memcpy(domain32 + 4, root, 28);
  return TBG_OK;
}

int tbg_signing_roots(uint32_t kind, const uint8_t* ssz, uint32_t n, const uint8_t* domains32, uint32_t n_domains,
                      const uint32_t* domain_idx, uint8_t* out32, uint32_t n_threads) {
  if (kind >= TBG_SSZ_KINDS || !n_domains || !domains32 || (n && (!ssz || !out32))) return TBG_E_INVALID_ARG;
  if (domain_idx)
    for (uint32_t i = 0; i < n; ++i)
      if (domain_idx[i] >= n_domains) return TBG_E_INVALID_ARG;
  const uint32_t sz = SIZES[kind];
  parallel_ranges(n, n_threads, [&](uint32_t lo, uint32_t hi) {
    uint8_t root[32];
    for (uint32_t i = lo; i < hi; ++i) {
      object_root(kind, ssz + (size_t)sz * i, root);
      hash_pair(root, domains32 + 32ull * (domain_idx ? domain_idx[i] : 0), out32 + 32ull * i);
    }
  });
  return TBG_OK;
}

}  // extern "C"
