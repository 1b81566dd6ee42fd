// libtbls_gpu.so: the C ABI of include/tbls_gpu.h on top of the HIP kernels.
//
// Per context: one HIP stream on one device, a resident public-key table,
// and a ring of in-flight batch slots.  tbg_submit packs the caller's
// structure-of-arrays batch into one pinned buffer, issues a single H2D copy,
// the kernel chain and a single D2H copy of the results, then returns a
// ticket; tbg_collect waits for (or polls) the slot's event and unpacks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <functional>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <new>
#include <random>
#include <thread>
#include <vector>
#include "tbls_launch.h"
#include "bls_lines.h"

using namespace tbg;

namespace tbg {
void debug_after_launch(const char* kernel, hipStream_t st) {
  static const bool on = getenv("TBG_DEBUG_SYNC") && getenv("TBG_DEBUG_SYNC")[0] == '1';
  if (!on) return;
  hipEvent_t a;
  (void)hipEventCreate(&a);
  (void)hipEventRecord(a, st);
  hipError_t e = hipEventSynchronize(a);
  (void)hipEventDestroy(a);
  fprintf(stderr, "[tbg] %s done: %s\n", kernel, hipGetErrorString(e));
}

struct KProfRec {
  const char* name;
  hipEvent_t a, b;
};
static thread_local std::vector<KProfRec>* g_kprof = nullptr;
// Every launch pushes a record, even when an event could not be created (its
// null events are skipped by kprof_post and reported as failed by the
// readout), so a record never takes a neighbour's end event.
void kprof_pre(const char* kernel, hipStream_t st) {
  if (!g_kprof) return;
  KProfRec r{kernel, nullptr, nullptr};
  if (hipEventCreate(&r.a) != hipSuccess) r.a = nullptr;
  if (r.a && hipEventCreate(&r.b) != hipSuccess) {
    (void)hipEventDestroy(r.a);
    r.a = r.b = nullptr;
  }
  if (r.a) (void)hipEventRecord(r.a, st);
  g_kprof->push_back(r);
}
void kprof_post(hipStream_t st) {
  if (!g_kprof || g_kprof->empty() || !g_kprof->back().b) return;
  (void)hipEventRecord(g_kprof->back().b, st);
}
}  // namespace tbg

namespace {

constexpr int kChainEvents = 11;

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// One caller batch inside a slot: tbg_submit_group packs several batches into
// one device batch (one launch per kernel for all of them); each keeps its
// own ticket and its slice of the outputs.
struct Part {
  tbg_ticket ticket = 0;
  uint32_t d0 = 0, nd = 0, p0 = 0, np = 0, m0 = 0, nm = 0;
  bool pending = false;     // not collected yet
  bool collecting = false;  // a blocking tbg_collect waits on the slot outside the context mutex
};

struct Slot {
  bool busy = false;        // some part is still pending
  bool express = false;     // the high-priority slot of small batches (tbg_config.express_partials)
  std::vector<Part> parts;
  tbg_ticket ticket = 0;    // first part's ticket (LRU order of the slots)
  uint32_t op = 0, n_duties = 0, n_partials = 0, n_msgs = 0;
  // pinned host staging
  uint8_t* h_in = nullptr;
  size_t h_in_cap = 0;
  uint8_t* h_out = nullptr;
  size_t h_out_cap = 0;
  // device memory: one input arena + one work/output arena
  uint8_t* d_in = nullptr;
  size_t d_in_cap = 0;
  uint8_t* d_work = nullptr;
  size_t d_work_cap = 0;
  size_t out_bytes = 0;
  hipStream_t st = nullptr;   // per-signature chain (decode, lines, verify, aggregate)
  hipStream_t st2 = nullptr;  // per-message chain (hash_to_G2, H(m) lines), joins st before verify
  hipEvent_t ev[kChainEvents] = {};  // see launch_chain
  hipEvent_t done = nullptr;
  float ms[8] = {};
  uint64_t seen_bad = 0, seen_total = 0;  // invalid / verified partials of the parts collected so far
  uint64_t seen_nsub = 0, seen_dec = 0;   // non-subgroup / all partials of the parts collected so far
  tbg::DevBatch B{};           // device view of the last batch (resident until the slot is reused)
  tbg::DevBatch last{};        // the batch as its last run launched it (a replay's prefix and shape):
                               // what tbg_fetch_stats / _fallback / _shape / _subgroup describe
  size_t w_out = 0;
};

}  // namespace

struct tbg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;  // utility stream (pubkey table, test-vector generation)
  std::mutex mu;
  G1A* d_pk = nullptr;
  G1A* d_xpk = nullptr;  // [x] pk per entry (k_decode_pubkeys)
  G1A* d_pktab = nullptr;  // [PK_TAB per key] the RLC products' key tables (k_msm.hip k_pubkey_tables)
  int32_t* d_pk_status = nullptr;
  uint32_t n_pk = 0, cap_pk = 0;
  hipEvent_t retire_ev = nullptr;  // orders frees of outgrown pubkey tables after the slots' queued work
  hipEvent_t keys_ready = nullptr;  // the key table's last load / growth (slot streams wait on it)
  std::vector<Slot> slots;
  tbg_ticket next_ticket = 1;
  float last_ms[8] = {};
  // Defaults measured on MI355X (tools/sweep_rlc.sh, config 2): 16 duties per
  // level-1 group, 4 per Miller quad beat 8 / 2 by ~8 %: half the final
  // exponentiations and Fp12 squarings per duty.
  uint32_t rlc_group = 16;  // 0 = per-partial checks (TBG_VERIFY_EACH)
  uint32_t rlc_chunk = 4;
  bool chunk_auto = true;    // rlc_chunk not configured: level-0 launches of many duties take 8
  bool rlc_auto = false;     // rlc_group follows the observed invalid share (tbg_config.rlc_group = 0)
  uint32_t rlc_batch = TBG_RLC_L0_AUTO;  // level 0 (the whole device batch as one check)
  double invalid_ema = 0.0;  // exponential average of the invalid share of collected verified partials
  uint64_t rlc_seed = 0;   // 0 = OS randomness per batch
  uint64_t seed_ctr = 0;
  uint32_t gident = TBG_GIDENT_OFF;  // level 1g routing (tbg_config.gident)
  uint32_t fb_window = TBG_FB_WINDOW;  // fallback line buffer positions per pass (tbg_config.fb_window)
  uint32_t sgb_mode = TBG_SGB_AUTO;    // batched subgroup test (tbg_config.subgroup_batch)
  uint32_t express_max = TBG_EXPRESS_PARTIALS;  // batches up to this many partials prefer the express slot
  uint32_t n_simd = 1024;  // SIMDs of the device (CUs x 4): the level-0 shape rule's unit (l0_shape)
  // host-side work of the submit / collect calls (tbg_host_stats): [submits,
  // partials submitted, pack ns, enqueue ns, collects, partials collected,
  // gather ns, wait ns]
  std::atomic<uint64_t> host[8] = {};
  double nonsub_ema = 0.0;  // exponential average of the non-subgroup share of collected partials
};

#define HIP_TRY(x)                       \
  do {                                   \
    hipError_t e_ = (x);                 \
    if (e_ != hipSuccess) return TBG_E_DEVICE; \
  } while (0)

// Capacity for an arena of `need` bytes: 25 % headroom for small arenas; big
// ones (a 16 x 10k-DV slot's work arena is ~5.9 GB) get 1/16 headroom rounded
// up to 256 MiB, so batch sizes that jitter around a boundary do not hipFree
// + hipMalloc (a device-wide synchronisation) on every submit.
static size_t arena_size(size_t need) {
  return need < (1ull << 30) ? align_up(need + need / 4, 1 << 20) : align_up(need + need / 16, 1ull << 28);
}

static int grow_pinned(uint8_t** p, size_t* cap, size_t need) {
  if (*cap >= need) return TBG_OK;
  if (*p) hipHostFree(*p);
  *p = nullptr;
  const size_t n = arena_size(need);
  if (hipHostMalloc((void**)p, n, hipHostMallocDefault) != hipSuccess) { *cap = 0; return TBG_E_OOM; }
  *cap = n;
  return TBG_OK;
}

static int grow_device(uint8_t** p, size_t* cap, size_t need) {
  if (*cap >= need) return TBG_OK;
  if (*p) hipFree(*p);
  *p = nullptr;
  const size_t n = arena_size(need);
  if (hipMalloc((void**)p, n) != hipSuccess) { *cap = 0; return TBG_E_OOM; }
  *cap = n;
  return TBG_OK;
}

extern "C" {

const char* tbg_strerror(int code) {
  switch (code) {
    case TBG_OK: return "ok";
    case TBG_E_INVALID_ARG: return "invalid argument";
    case TBG_E_DEVICE: return "HIP device error";
    case TBG_E_OOM: return "out of memory";
    case TBG_E_NO_DEVICE: return "no gfx950 device";
    case TBG_E_BUSY: return "all batch slots busy";
    case TBG_E_PENDING: return "batch still running";
    case TBG_E_TICKET: return "unknown ticket";
    default: return "unknown error";
  }
}

int tbg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int tbg_device_cu_count(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return TBG_E_NO_DEVICE;
  if (device < 0 || device >= ndev) return TBG_E_INVALID_ARG;
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return TBG_E_DEVICE;
  return n_cu;
}

int tbg_synchronize(tbg_ctx* c) {
  if (!c) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  if (c->stream) HIP_TRY(hipStreamSynchronize(c->stream));
  for (auto& s : c->slots) {
    if (s.st) HIP_TRY(hipStreamSynchronize(s.st));
    if (s.st2 && s.st2 != s.st) HIP_TRY(hipStreamSynchronize(s.st2));
  }
  return TBG_OK;
}

int tbg_init(const tbg_config* cfg, tbg_ctx** out) {
  if (!out) return TBG_E_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return TBG_E_NO_DEVICE;
  int dev = cfg ? cfg->device : 0;
  if (dev < 0 || dev >= ndev) return TBG_E_INVALID_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return TBG_E_DEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return TBG_E_NO_DEVICE;
  tbg_ctx* c = new (std::nothrow) tbg_ctx();
  if (!c) return TBG_E_OOM;
  c->device = dev;
  if (cfg && cfg->verify_mode == TBG_VERIFY_EACH) c->rlc_group = 0;
  else if (cfg && cfg->verify_mode != TBG_VERIFY_RLC) { delete c; return TBG_E_INVALID_ARG; }
  else if (cfg && cfg->rlc_group) c->rlc_group = cfg->rlc_group;
  else c->rlc_auto = true;
  if (cfg && cfg->rlc_chunk) {
    c->rlc_chunk = cfg->rlc_chunk;
    c->chunk_auto = false;
  }
  if (c->rlc_group > 4096 || c->rlc_chunk > 4096) { delete c; return TBG_E_INVALID_ARG; }
  if (cfg && cfg->rlc_batch > TBG_RLC_L0_OFF) { delete c; return TBG_E_INVALID_ARG; }
  if (cfg) c->rlc_batch = cfg->rlc_batch;
  c->rlc_seed = cfg ? cfg->rlc_seed : 0;
  if (cfg && cfg->gident > TBG_GIDENT_CHUNKS) { delete c; return TBG_E_INVALID_ARG; }
  c->gident = cfg ? cfg->gident : (uint32_t)TBG_GIDENT_OFF;
  if (cfg && cfg->fb_window) c->fb_window = cfg->fb_window;
  if (cfg && cfg->subgroup_batch > TBG_SGB_OFF) { delete c; return TBG_E_INVALID_ARG; }
  if (cfg) c->sgb_mode = cfg->subgroup_batch;
  if (cfg && cfg->express_partials) c->express_max = cfg->express_partials;
  if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->retire_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->keys_ready, hipEventDisableTiming) != hipSuccess) {
    if (c->retire_ev) hipEventDestroy(c->retire_ev);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return TBG_E_DEVICE;
  }
  // Every in-flight slot owns its two streams, so back-to-back submits
  // overlap on the GPU (one batch's latency-bound stages fill the CUs the
  // other leaves idle).
  uint32_t nslots = (cfg && cfg->slots) ? cfg->slots : 3;
  const uint32_t spp = (cfg && cfg->streams_per_slot > 1) ? cfg->streams_per_slot : 1;
  // The express slot takes one stream more; a configuration with no stream
  // left for it runs without one rather than being refused.
  if (nslots * spp + 1 > TBG_MAX_SLOT_STREAMS) c->express_max = TBG_EXPRESS_OFF;
  const bool express = c->express_max != TBG_EXPRESS_OFF;
  if (nslots > TBG_MAX_SLOTS || spp > 2 || nslots * spp + (express ? 1 : 0) > TBG_MAX_SLOT_STREAMS) {
    hipStreamDestroy(c->stream);
    hipEventDestroy(c->retire_ev);
    hipEventDestroy(c->keys_ready);
    delete c;
    return TBG_E_INVALID_ARG;
  }
  // (+ the express slot: one more slot, last, on a high-priority stream)
  c->slots.resize(nslots + (express ? 1 : 0));
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n_cu > 0)
    c->n_simd = (uint32_t)n_cu * 4u;
  // One stream per slot by default: the HIP runtime maps streams onto a
  // few hardware queues (GPU_MAX_HW_QUEUES, 4 by default), so concurrency
  // comes from several batches in flight, one queue each.  Two streams
  // per slot also overlap a batch's hash_to_G2 with its decode (lower
  // single-batch latency when queues are plentiful).
  const bool two = cfg && cfg->streams_per_slot >= 2;
  // (Per-slot stream priorities were measured within noise, round 3.)
  int prio_least = 0, prio_greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = prio_least = 0;
  for (size_t k = 0; k < c->slots.size(); ++k) {
    auto& s = c->slots[k];
    s.express = express && k == nslots;
    auto mk = [&](hipStream_t* st) { return hipStreamCreateWithFlags(st, hipStreamNonBlocking); };
    if (s.express) {
      // A small batch's chain is ~50 short kernels in series: on a
      // high-priority queue their dispatches go ahead of the throughput
      // launches' pending workgroups instead of queueing behind them.
      if (hipStreamCreateWithPriority(&s.st, hipStreamNonBlocking, prio_greatest) != hipSuccess) {
        tbg_destroy(c);
        return TBG_E_DEVICE;
      }
      s.st2 = s.st;
    } else {
      if (mk(&s.st) != hipSuccess || (two && mk(&s.st2) != hipSuccess)) {
        tbg_destroy(c);
        return TBG_E_DEVICE;
      }
      if (!two) s.st2 = s.st;
    }
    for (auto& e : s.ev) hipEventCreate(&e);
    hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
  }
  *out = c;
  return TBG_OK;
}

void tbg_destroy(tbg_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  for (auto& s : c->slots) {
    if (s.st) hipStreamSynchronize(s.st);
    if (s.st2 && s.st2 != s.st) hipStreamSynchronize(s.st2);
    if (s.h_in) hipHostFree(s.h_in);
    if (s.h_out) hipHostFree(s.h_out);
    if (s.d_in) hipFree(s.d_in);
    if (s.d_work) hipFree(s.d_work);
    for (auto& e : s.ev)
      if (e) hipEventDestroy(e);
    if (s.done) hipEventDestroy(s.done);
    if (s.st2 && s.st2 != s.st) hipStreamDestroy(s.st2);
    if (s.st) hipStreamDestroy(s.st);
  }
  // the key tables are stream-ordered allocations of the utility stream
  if (c->stream) {
    for (void* p : {(void*)c->d_pk, (void*)c->d_xpk, (void*)c->d_pktab, (void*)c->d_pk_status})
      if (p) hipFreeAsync(p, c->stream);
    hipStreamSynchronize(c->stream);
    hipStreamDestroy(c->stream);
  }
  if (c->retire_ev) hipEventDestroy(c->retire_ev);
  if (c->keys_ready) hipEventDestroy(c->keys_ready);
  delete c;
}

uint32_t tbg_pubkey_count(const tbg_ctx* c) { return c ? c->n_pk : 0; }

int tbg_load_pubkeys(tbg_ctx* c, const uint8_t* pk48, uint32_t count, uint32_t* first_id, int32_t* status) {
  if (!c || (count && !pk48)) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  if (c->n_pk + (uint64_t)count > 0xFFFFFFF0ull) return TBG_E_INVALID_ARG;
  uint32_t need = c->n_pk + count;
  void* old_tabs[4] = {nullptr, nullptr, nullptr, nullptr};  // outgrown tables, freed below
  if (need > c->cap_pk) {
    // Stream-ordered allocations on the utility stream: no device-wide
    // synchronisation (hipMalloc / hipFree would wait for every batch in flight).
    uint32_t ncap = need + need / 2 + 1024;
    G1A* npk = nullptr;
    G1A* nxpk = nullptr;
    G1A* ntab = nullptr;
    int32_t* nst = nullptr;
    hipStream_t us = c->stream;
    if (hipMallocAsync((void**)&npk, sizeof(G1A) * (size_t)ncap, us) != hipSuccess) return TBG_E_OOM;
    if (hipMallocAsync((void**)&nxpk, sizeof(G1A) * (size_t)ncap, us) != hipSuccess) {
      hipFreeAsync(npk, us);
      return TBG_E_OOM;
    }
    if (hipMallocAsync((void**)&ntab, PK_TAB * sizeof(G1A) * (size_t)ncap, us) != hipSuccess) {
      hipFreeAsync(npk, us);
      hipFreeAsync(nxpk, us);
      return TBG_E_OOM;
    }
    if (hipMallocAsync((void**)&nst, sizeof(int32_t) * (size_t)ncap, us) != hipSuccess) {
      hipFreeAsync(npk, us);
      hipFreeAsync(nxpk, us);
      hipFreeAsync(ntab, us);
      return TBG_E_OOM;
    }
    if (c->n_pk) {
      HIP_TRY(hipMemcpyAsync(npk, c->d_pk, sizeof(G1A) * (size_t)c->n_pk, hipMemcpyDeviceToDevice, us));
      HIP_TRY(hipMemcpyAsync(nxpk, c->d_xpk, sizeof(G1A) * (size_t)c->n_pk, hipMemcpyDeviceToDevice, us));
      HIP_TRY(hipMemcpyAsync(ntab, c->d_pktab, PK_TAB * sizeof(G1A) * (size_t)c->n_pk, hipMemcpyDeviceToDevice, us));
      HIP_TRY(hipMemcpyAsync(nst, c->d_pk_status, sizeof(int32_t) * (size_t)c->n_pk, hipMemcpyDeviceToDevice, us));
    }
    old_tabs[0] = c->d_pk;
    old_tabs[1] = c->d_xpk;
    old_tabs[2] = c->d_pktab;
    old_tabs[3] = c->d_pk_status;
    c->d_pk = npk;
    c->d_xpk = nxpk;
    c->d_pktab = ntab;
    c->d_pk_status = nst;
    c->cap_pk = ncap;
  }
  if (first_id) *first_id = c->n_pk;
  uint8_t* d_bytes = nullptr;  // stream-ordered staging (freed on the same stream)
  if (count && hipMallocAsync((void**)&d_bytes, 48ull * count, c->stream) != hipSuccess) return TBG_E_OOM;
  int rc = TBG_OK;
  if (count == 0) goto ready;
  if (hipMemcpyAsync(d_bytes, pk48, 48ull * count, hipMemcpyHostToDevice, c->stream) != hipSuccess) rc = TBG_E_DEVICE;
  if (rc == TBG_OK) {
    launch_decode_pubkeys(d_bytes, count, c->d_pk + c->n_pk, c->d_xpk + c->n_pk, c->d_pk_status + c->n_pk, c->stream);
    launch_pubkey_tables(c->d_pk + c->n_pk, c->d_xpk + c->n_pk, c->d_pk_status + c->n_pk, count,
                         c->d_pktab + (size_t)PK_TAB * c->n_pk, c->stream);
    if (hipGetLastError() != hipSuccess) rc = TBG_E_DEVICE;
  }
  if (rc == TBG_OK && status &&
      hipMemcpyAsync(status, c->d_pk_status + c->n_pk, sizeof(int32_t) * count, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    rc = TBG_E_DEVICE;
ready:
  // Submits order their slot streams after this event, not after the frees below.
  if (hipEventRecord(c->keys_ready, c->stream) != hipSuccess) rc = TBG_E_DEVICE;
  if (old_tabs[0]) {
    // Batches already queued on the slot streams captured the old tables'
    // addresses: their free is ordered after everything queued so far on
    // every slot stream (one event recorded per stream, waited on by the
    // utility stream), without blocking the host or the device.
    for (auto& sl : c->slots)
      for (hipStream_t q : {sl.st, sl.st2}) {
        if (!q || (q == sl.st2 && sl.st2 == sl.st)) continue;
        if (hipEventRecord(c->retire_ev, q) != hipSuccess || hipStreamWaitEvent(c->stream, c->retire_ev, 0) != hipSuccess)
          rc = TBG_E_DEVICE;
      }
    for (void* p : old_tabs) hipFreeAsync(p, c->stream);
  }
  if (d_bytes) hipFreeAsync(d_bytes, c->stream);
  if (hipEventSynchronize(c->keys_ready) != hipSuccess) rc = TBG_E_DEVICE;
  if (rc == TBG_OK) c->n_pk += count;
  return rc;
}

// The aggregation the checks will mostly confirm (every candidate valid),
// enqueued mid-chain so the launch's tail is the verification plus the redo of
// the few duties with an invalid partial (none after a level-0 pass).
static void spec_aggregation(const DevBatch& B, hipStream_t st) {
  launch_lagrange(B, st, true);
  launch_aggregate(B, st, true);
  launch_aggregate_finish(B, st, true);
}

// The kernel chain of one batch.  Per-message work (hash_to_G2, H(m) lines)
// runs on st2 concurrently with the per-signature work (decode, RLC sums and
// group lines) on st; the product checks join both.
// Events: ev[0] start, ev[1] decode done, ev[2] combine done, ev[3]/ev[4]
// hash start/done and ev[5] H lines done (st2), ev[6] verify start, ev[7]
// verify done, ev[8] lagrange done, ev[9] aggregate done, ev[10] decode start.
// `stage` enqueues one part (0: start + the first chain, 1: the second
// chain, 2: the checks and the aggregation; -1: all three): a replay of
// several slots enqueues stage 0 of every slot before stage 1 of any, so the
// slots' first kernels start together instead of one chain's enqueue time
// (~100 launches) apart.
static int launch_chain(tbg_ctx* c, const Slot& sl, const DevBatch& B, hipEvent_t* ev, int stage = -1) {
  hipStream_t st = sl.st, st2 = sl.st2;
  const bool verify = B.op != TBG_OP_AGGREGATE;
  const G1A* pk = (const G1A*)c->d_pk;
  // With one stream per slot the two independent chains run one after the
  // other, the per-message chain first (running the per-signature chain
  // first on odd slots was measured no better, round 2).
  // The aggregation runs speculatively as soon as the candidates are final
  // (every candidate taken as valid), off the launch's serial tail, while
  // level 0 is on (TBG_SPEC_ALWAYS: on every VERIFY_AGGREGATE chain, redoing
  // only the duties with an invalid partial -- measured slower, round 5).
  const bool spec = B.op == TBG_OP_VERIFY_AGGREGATE && (TBG_SPEC_ALWAYS || (B.rlc_batch && B.rlc_group));
  auto msg_chain = [&]() -> int {
    HIP_TRY(hipEventRecord(ev[3], st2));
    if (verify) launch_hash_msgs(B, st2);
    HIP_TRY(hipEventRecord(ev[4], st2));
    if (verify) launch_h_lines(B, st2);
    HIP_TRY(hipEventRecord(ev[5], st2));
    return TBG_OK;
  };
  auto sig_chain = [&]() -> int {
    HIP_TRY(hipEventRecord(ev[10], st));
    launch_decode_sigs(B, st);  // zeroes B.counters (and level 0's bucket sizes) first
    HIP_TRY(hipEventRecord(ev[1], st));
    // The aggregation a level-0 pass will confirm runs as soon as the
    // candidates are final (after the key checks), before the bucket MSM:
    // placed after it, its small kernels waited behind the other launches'
    // long Miller waves for a free slot and delayed this launch's own Miller
    // kernel (k_lagrange<true> 7.7 ms instead of 0.05, profiles/r04/base/
    // timeline_s20.txt).
    if (verify)
      launch_rlc_prepare(B, pk, (const G1A*)c->d_xpk, (const G1A*)c->d_pktab, (const int32_t*)c->d_pk_status, c->n_pk,
                         st, spec ? spec_aggregation : nullptr);
    HIP_TRY(hipEventRecord(ev[2], st));
    return TBG_OK;
  };
  // TBG_ALT_ORDER: on one stream, odd slots run the per-signature chain
  // first, so launches in flight together are out of phase (one launch's
  // latency-bound subgroup / MSM tails beside another's hash).
  const bool alt = TBG_ALT_ORDER && st == st2 && ((&sl - c->slots.data()) & 1);
  int rc;
  if (stage < 0 || stage == 0) {
    HIP_TRY(hipEventRecord(ev[0], st));
    HIP_TRY(hipStreamWaitEvent(st2, ev[0], 0));
    if ((rc = alt ? sig_chain() : msg_chain()) != TBG_OK) return rc;
  }
  if (stage < 0 || stage == 1)
    if ((rc = alt ? msg_chain() : sig_chain()) != TBG_OK) return rc;
  if (stage >= 0 && stage != 2) return TBG_OK;
  HIP_TRY(hipStreamWaitEvent(st, ev[5], 0));
  HIP_TRY(hipEventRecord(ev[6], st));
  if (verify) launch_rlc_check(B, pk, (const G1A*)c->d_xpk, (const int32_t*)c->d_pk_status, c->n_pk, st);
  HIP_TRY(hipEventRecord(ev[7], st));
  if (B.op != TBG_OP_VERIFY) launch_lagrange(B, st);
  HIP_TRY(hipEventRecord(ev[8], st));
  launch_aggregate(B, st);
  if (B.op != TBG_OP_VERIFY) launch_aggregate_finish(B, st);
  HIP_TRY(hipEventRecord(ev[9], st));
  HIP_TRY(hipGetLastError());
  return TBG_OK;
}

// [decode, hash, combine, H lines, verify, lagrange, aggregate, total]
static void chain_times(hipEvent_t* e, float* ms) {
  hipEventElapsedTime(&ms[0], e[10], e[1]);
  hipEventElapsedTime(&ms[1], e[3], e[4]);
  hipEventElapsedTime(&ms[2], e[1], e[2]);
  hipEventElapsedTime(&ms[3], e[4], e[5]);
  hipEventElapsedTime(&ms[4], e[6], e[7]);
  hipEventElapsedTime(&ms[5], e[7], e[8]);
  hipEventElapsedTime(&ms[6], e[8], e[9]);
  hipEventElapsedTime(&ms[7], e[0], e[9]);
}

static int validate(const tbg_batch* b) {
  if (!b) return TBG_E_INVALID_ARG;
  if (b->op < TBG_OP_VERIFY || b->op > TBG_OP_VERIFY_AGGREGATE) return TBG_E_INVALID_ARG;
  if (b->n_duties == 0) return TBG_E_INVALID_ARG;
  if (!b->duty_first || (b->n_partials && (!b->sigs || !b->identifiers))) return TBG_E_INVALID_ARG;
  if (b->duty_first[0] != 0 || b->duty_first[b->n_duties] != b->n_partials) return TBG_E_INVALID_ARG;
  for (uint32_t d = 0; d < b->n_duties; ++d) {
    if (b->duty_first[d + 1] < b->duty_first[d]) return TBG_E_INVALID_ARG;
    if (b->duty_first[d + 1] - b->duty_first[d] > 255) return TBG_E_INVALID_ARG;
  }
  if (b->op != TBG_OP_AGGREGATE) {
    if (!b->msg_off || !b->duty_msg || !b->pubkey_ids || b->n_msgs == 0) return TBG_E_INVALID_ARG;
    if (b->msg_off[0] != 0) return TBG_E_INVALID_ARG;
    for (uint32_t m = 0; m < b->n_msgs; ++m)
      if (b->msg_off[m + 1] < b->msg_off[m]) return TBG_E_INVALID_ARG;
    if (b->msg_off[b->n_msgs] && !b->msgs) return TBG_E_INVALID_ARG;
    for (uint32_t d = 0; d < b->n_duties; ++d)
      if (b->duty_msg[d] >= b->n_msgs) return TBG_E_INVALID_ARG;
  }
  if (b->op == TBG_OP_VERIFY_AGGREGATE && !b->duty_threshold) return TBG_E_INVALID_ARG;
  return TBG_OK;
}

// The slot and part a ticket names.  want_busy: the part must be pending
// (collect / poll) or the slot idle (replay / fetch of a collected batch).
static Slot* find_ticket(tbg_ctx* c, tbg_ticket t, bool want_pending, Part** part) {
  for (auto& x : c->slots)
    for (auto& q : x.parts)
      if (q.ticket == t && (want_pending ? q.pending : !x.busy)) {
        if (part) *part = &q;
        return &x;
      }
  return nullptr;
}

int tbg_submit(tbg_ctx* c, const tbg_batch* b, tbg_ticket* ticket) { return tbg_submit_group(c, &b, 1, ticket); }

// Level-0 launch shape.  The level-0 Miller kernel's
// waves are long -- one hexad = the whole 68-step loop over C duties -- and
// issue-bound at ONE wave per SIMD: a lone wave runs its loop in 3.6 ms at
// C = 4, two sharing a SIMD take 6.8 ms each (profiles/r05/waves), so the
// kernel's time is ~ceil(waves / SIMDs) hexad lengths, and a launch whose
// waves spill just past a multiple of the SIMD count pays a whole hexad
// length for the remainder: config 4's 125k-duty shard at (G, C) = (16, 4)
// is 3,126 waves on 1,024 SIMDs.  A hexad of C duties costs 62 squarings +
// 68 C line products, w(C) = 0.95 M + 1.39 M C u32 mul-adds
// (profiles/work_model.json, l0_chunk_*), so fewer, longer hexads win where
// they save a unit: (16, 8) halves the squarings, (14, 7) runs 125k duties
// in 2 units instead of 4.  The rule picks the cheapest of (16, 4), (16, 8),
// (14, 7) by ceil(waves / SIMDs) x w(C) -- 100k duties keep (16, 4), 125k
// take (14, 7), 160k (16, 8), as the A/B runs of profiles/r05/chunk8_ab,
// shape_ab and sqrt_x2_ab measured best.  A configured group size G keeps G
// (C = 4 or 8 only).  tbg_replay_plan applies it to the duties of the
// launches it runs together (their Miller kernels share the SIMDs).
static double l0_shape_cost(uint64_t nd, uint32_t n_simd, uint32_t g, uint32_t ch) {
  const uint64_t hexads = (uint64_t)((nd + g - 1) / g) * ((g + ch - 1) / ch);
  const uint64_t waves = (hexads + 9) / 10;
  return (0.948 + 1.395 * ch) * (double)((waves + n_simd - 1) / n_simd);
}
// Round 6: with the group size free, every chunk C of
// 5 .. 10 duties is a candidate too, as (G, C) = (C, C) -- one chunk per
// group -- so the hexads can fill whole wave-slot rounds: the 20-step plan's
// 200k duties take (10, 10) (2,000 waves: 2 rounds) instead of (14, 7) (2,858
// waves: 3 rounds; +2.6 % at the driver shape, profiles/r06/shape), config
// 3's 100k (10, 10) instead of (16, 4) (Miller 8.0 vs 9.4 ms).  Chunks of 13
// and 16 duties were measured far off the model (a round of ~1,000 lone
// waves: (16, 16) 20.4 ms vs (16, 8) 12.2 ms at 160k duties, (13, 13) 16.8
// vs (14, 7) 11.0 ms at 125k: the C line loads of a step are not hidden by a
// second wave), so C stops at L0_SHAPE_MAX_C.
// `fits` (a replay's arenas, below) drops the candidates a launch cannot hold.
static bool l0_fits_any(uint32_t, uint32_t) { return true; }
static void l0_shape(uint64_t nd, uint32_t n_simd, bool g_free, uint32_t& G, uint32_t& C,
                     const std::function<bool(uint32_t, uint32_t)>& fits) {
  C = 4;
  if (!TBG_L0_SHAPE || G < 8) return;
  constexpr uint32_t L0_SHAPE_MAX_C = 10;
  uint32_t cand[3 + L0_SHAPE_MAX_C][2] = {{g_free ? 16u : G, 4}, {g_free ? 16u : G, 8}, {14, 7}};
  uint32_t n_cand = g_free ? 3u : 2u;
  for (uint32_t c = 5; TBG_L0_SHAPE_WIDE && g_free && c <= L0_SHAPE_MAX_C; ++c) {
    cand[n_cand][0] = c;
    cand[n_cand][1] = c;
    ++n_cand;
  }
  double best = 1e300;
  const uint32_t G0 = G;
  for (uint32_t k = 0; k < n_cand; ++k) {
    if (!fits(cand[k][0], cand[k][1])) continue;
    const double cost = l0_shape_cost(nd, n_simd, cand[k][0], cand[k][1]);
    if (cost < best - 1e-9) {
      best = cost;
      G = cand[k][0];
      C = cand[k][1];
    }
  }
  if (best == 1e300) G = G0;  // (nothing fits: the caller keeps its shapes)
}
// A launch of nd duties (a prefix of its slot's device batch) at (G, C) fits
// the slot's arena, whose group / chunk sections were sized at submit for
// the slot's nd0 duties at (G0, C0) (tbg_submit_group).
static bool l0_shape_fits(uint32_t nd0, uint32_t G0, uint32_t C0, uint32_t nd, uint32_t G, uint32_t C) {
  const uint64_t ng0 = (nd0 + G0 - 1) / G0, nch0 = (G0 + C0 - 1) / C0;
  const uint64_t ng = (nd + G - 1) / G, nch = (G + C - 1) / C;
  // every group / chunk section of the arena (tbg_submit_group's w_cf,
  // w_gidf: ng (nch + 1); w_cl, w_cfe, w_cidl: ng nch -- ADVICE r05: the
  // max() below alone let nd0 hide an overflow of these; w_cidp: ng nch C;
  // w_gidp: ng G; w_pend: max(ng nch, nd); grp_f: ng)
  return ng <= ng0 && ng * (nch + 1) <= ng0 * (nch0 + 1) && ng * nch <= ng0 * nch0 && ng * nch * C <= ng0 * nch0 * C0 &&
         ng * G <= ng0 * G0 && std::max(ng * nch, (uint64_t)nd) <= std::max(ng0 * nch0, (uint64_t)nd0) &&
         (G <= 64) == (G0 <= 64);
}

// Batched subgroup test plan from the non-subgroup share `rho` of the
// collected partials.  Per signature, in units of one
// per-signature test (psi(s) == [x] s: 63 doublings + 5 additions): the 16.6
// bucket additions with the sort and running sums 0.55 (measured: k_sgb_*
// 0.47-0.57 of k_subgroup_sigs' time per signature, profiles/r06/sgb), the
// group's 18 tests 1.1 x 18 / m (each on a lone lane pair), and the failed
// groups' members tested alone 1 - (1 - rho)^m.  The group size m is the
// cheapest power of two in [SGB_M_MIN, SGB_M]; the test runs while that
// costs under 0.95 of testing every signature alone -- up to rho ~ 2.5e-3
// (TBG_SGB_AUTO_MAX).  Clean traffic keeps m = 1,024; config 5's 1.25e-3
// takes m = 128 (at 1,024, 72 % of its groups would fail).
static bool sgb_plan(double rho, uint32_t& m) {
  double best = 1e9;
  m = SGB_M;
  for (uint32_t k = SGB_M; k >= SGB_M_MIN; k >>= 1) {
    const double cost = 0.55 + 1.1 * (double)SGB_K / k + (1.0 - std::pow(1.0 - std::min(rho, 1.0), (double)k));
    if (cost < best - 1e-12) {
      best = cost;
      m = k;
    }
  }
  return best < 0.95;
}

int tbg_submit_group(tbg_ctx* c, const tbg_batch* const* bs, uint32_t n_batches, tbg_ticket* tickets) {
  if (!c || !bs || !tickets || n_batches == 0) return TBG_E_INVALID_ARG;
  int rc;
  for (uint32_t k = 0; k < n_batches; ++k) {
    if ((rc = validate(bs[k])) != TBG_OK) return rc;
    if (bs[k]->op != bs[0]->op) return TBG_E_INVALID_ARG;  // one kernel chain per device batch
  }
  const uint32_t op = bs[0]->op;
  const bool verify = op != TBG_OP_AGGREGATE;
  uint64_t nd64 = 0, np64 = 0, nm64 = 0, mb64 = 0;
  for (uint32_t k = 0; k < n_batches; ++k) {
    nd64 += bs[k]->n_duties;
    np64 += bs[k]->n_partials;
    if (verify) {
      nm64 += bs[k]->n_msgs;
      mb64 += bs[k]->msg_off[bs[k]->n_msgs];
    }
  }
  if (np64 > 0x7FFFFFFFull || nd64 > 0x7FFFFFFFull || nm64 > 0x7FFFFFFFull || mb64 > 0xFFFFFFFFull)
    return TBG_E_INVALID_ARG;
  std::unique_lock<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  // Least recently used free slot: a collected batch stays resident (for
  // tbg_replay / tbg_fetch) until every other slot has been reused.  A batch
  // of at most express_max partials takes the express slot when it is free.
  Slot* s = nullptr;
  const bool small = np64 <= c->express_max;
  for (auto& x : c->slots)
    if (x.express && small && !x.busy) s = &x;
  if (!s)
    for (auto& x : c->slots)
      if (!x.express && !x.busy && (!s || x.ticket < s->ticket)) s = &x;
  if (!s) return TBG_E_BUSY;

  const uint32_t nd = (uint32_t)nd64, np = (uint32_t)np64, nm = (uint32_t)nm64;
  const size_t msg_bytes = (size_t)mb64;

  // ---- input arena layout (16-byte aligned sections) ----
  size_t o = 0;
  auto sec = [&](size_t bytes) { size_t at = o; o = align_up(o + bytes, 16); return at; };
  size_t o_msgs = sec(msg_bytes);
  size_t o_msg_off = sec(4ull * (nm + 1));
  size_t o_duty_msg = sec(4ull * nd);
  size_t o_duty_first = sec(4ull * (nd + 1));
  size_t o_thr = sec(4ull * nd);
  size_t o_pduty = sec(4ull * np);
  size_t o_sigs = sec(96ull * np);
  size_t o_ids = sec(np);
  size_t o_pk = sec(4ull * np);
  size_t in_bytes = o;
  // ---- work/output arena ----
  o = 0;
  size_t w_sig_aff = sec(sizeof(G2A) * (size_t)np);
  size_t w_h_aff = sec(sizeof(G2A) * (size_t)nm);
  size_t w_h_st = sec(4ull * nm);
  size_t w_h_jac = sec(3 * sizeof(G2J) * (size_t)nm);  // H(m) + the cofactor clearing's two temporaries
  size_t w_lam = sec(32ull * np);
  // The fallback levels' lines share one buffer of fb_w list positions,
  // consumed in passes (DevBatch::fb_window): a slot no longer holds 22.8 KB
  // per partial for lists that a clean batch leaves empty.
  const uint32_t fb_w = verify ? std::max<uint32_t>(1u, std::min<uint32_t>(c->fb_window, np)) : 0u;
  size_t w_sl = sec(4ull * LINES_WORDS * fb_w);
  size_t w_hl = sec(4ull * LINES_WORDS * nm);
  if (c->rlc_auto)
    c->rlc_group = c->invalid_ema < TBG_RLC_AUTO_TO8 ? 16 : c->invalid_ema < TBG_RLC_AUTO_TO4 ? 8 : 4;
  uint32_t G = verify ? c->rlc_group : 0;
  // Level 0 while the collected batches are clean (or as configured): one
  // failed level-0 check costs its own work on top of the group levels.
  const bool l0 = G != 0 && np < (1u << 28) &&
                  (c->rlc_batch == TBG_RLC_L0_ON || (c->rlc_batch == TBG_RLC_L0_AUTO && c->invalid_ema < TBG_RLC_AUTO_L0));
  uint32_t C = c->rlc_chunk;
  if (l0 && c->chunk_auto) l0_shape(nd, c->n_simd, c->rlc_auto && G == 16, G, C, l0_fits_any);
  if (C > G) C = G ? G : 1;
  const uint32_t ng = G ? (nd + G - 1) / G : 0;
  const uint32_t nch = G ? (G + C - 1) / C : 0;
  size_t w_pp = sec(G ? sizeof(G1J) * (size_t)np : 0);
  size_t w_ps = sec(G ? sizeof(G2J) * (size_t)np : 0);
  size_t w_cf = sec(G ? 4ull * 3 * 4 * NL * ng * (nch + 1) : 0);
  size_t w_cl = sec(G > 1 ? 4ull * ng * nch : 0);

  size_t w_dvp = sec(G ? sizeof(G1A) * (size_t)nd : 0);
  size_t w_dvs = sec(G ? sizeof(G2J) * (size_t)nd : 0);
  size_t w_dvst = sec(G ? 4ull * nd : 0);
  size_t w_gst = sec(4ull * ng);
  size_t w_gl = sec(4ull * LINES_WORDS * ng);
  size_t w_cnt = sec(4ull * CNT_WORDS);
  size_t w_pl = sec(verify ? 4ull * np : 0);
  size_t w_dvfe = sec(G > 1 ? 4ull * 3 * 4 * NL * nd : 0);
  size_t w_pend = sec(G ? sizeof(G2A) * (size_t)std::max<size_t>(std::max<size_t>(ng, (size_t)ng * nch), nd) : 0);
  size_t w_cfe = sec(G > 1 ? 4ull * 3 * 4 * NL * ng * nch : 0);
  size_t w_cidl = sec(G > 1 ? 4ull * ng * nch : 0);
  size_t w_cidp = sec(G > 1 ? sizeof(G1A) * (size_t)ng * nch * C : 0);

  size_t w_gfe = sec(G > 1 ? 4ull * 3 * 4 * NL * ng : 0);
  size_t w_gidl = sec(G > 1 ? 4ull * ng : 0);
  size_t w_gidp = sec(G > 1 ? sizeof(G1A) * (size_t)ng * G : 0);
  size_t w_gidf = sec(G > 1 ? 4ull * 3 * 4 * NL * ng * (nch + 1) : 0);
  size_t w_idl = sec(G > 1 ? 4ull * nd : 0);
  size_t w_idp = sec(G > 1 ? sizeof(G1A) * (size_t)nd : 0);
  size_t w_mr = sec(l0 ? 8ull * np : 0);
  size_t w_moff = sec(l0 ? 4ull * (MSM_BUCKETS + 1) : 0);
  size_t w_mcur = sec(l0 ? 4ull * MSM_BUCKETS : 0);
  size_t w_ment = sec(l0 ? 16ull * np : 0);
  size_t w_mbkt = sec(l0 ? sizeof(G2J) * (size_t)MSM_BUCKETS : 0);
  size_t w_mpart = sec(l0 ? sizeof(G2J) * (size_t)MSM_BUCKETS * MSM_SPLIT : 0);
  size_t w_msum = sec(l0 ? sizeof(G2J) * (size_t)MSM_SUM_ENTRIES : 0);
  size_t w_bpt = sec(l0 ? sizeof(G2A) : 0);
  size_t w_blines = sec(l0 ? 4ull * LINES_WORDS : 0);
  size_t w_bf = sec(l0 ? 4ull * 3 * 4 * NL : 0);
  size_t w_gf = sec(l0 ? 4ull * 3 * 4 * NL * grp_f_entries(ng) : 0);
  // level 1's group MSM (k_gmsm.hip): entries, offsets, bucket sums, leads, the failed groups' candidates
  const bool gm = TBG_GMSM && G != 0;
  size_t w_gmoff = sec(gm ? 4ull * (GM_BUCKETS + 1) * ng : 0);
  size_t w_gment = sec(gm ? 64ull * np : 0);
  size_t w_gmpart = sec(gm ? sizeof(G2J) * GM_BUCKETS * (size_t)ng : 0);
  size_t w_gmlead = sec(gm ? 4ull * ng : 0);
  size_t w_gmlist = sec(gm ? 4ull * np : 0);
  size_t w_gmhist = sec(gm ? 4ull * 256 : 0);
  size_t w_gmorder = sec(gm ? 4ull * GM_BUCKETS * ng : 0);
  // Batched subgroup test while the collected batches carry (almost) no
  // non-subgroup signature: groups of 1,024 partials, a failed group's members
  // tested alone (k_sgb.hip); small batches test every signature alone.
  uint32_t sgb_m = SGB_M;
  const bool sgb = np >= SGB_MIN_PARTIALS && c->sgb_mode != TBG_SGB_OFF &&
                   (sgb_plan(c->nonsub_ema, sgb_m) || c->sgb_mode == TBG_SGB_ON);
  const uint32_t sgb_split = sgb_split_for(sgb_m);
  const size_t n_sg = sgb ? sgb_groups(np, sgb_m) : 0;
  size_t w_sgoff = sec(4ull * (SGB_BUCKETS + 1) * n_sg);
  size_t w_sgent = sec(4ull * sgb_m * SGB_K * n_sg);
  size_t w_sgpart = sec(sizeof(G2J) * SGB_BUCKETS * sgb_split * n_sg);
  size_t w_sgbad = sec(4ull * n_sg);
  size_t w_aacc = sec(op != TBG_OP_VERIFY ? sizeof(G2J) * (size_t)nd : 0);
  size_t w_alist = sec(op != TBG_OP_VERIFY ? 4ull * nd : 0);
  size_t w_out = o;  // outputs are contiguous so one D2H copy brings them back
  size_t w_pst = sec(4ull * np);
  size_t w_dst = sec(4ull * nd);
  size_t w_agg = sec(96ull * nd);
  size_t work_bytes = o;
  size_t out_bytes = work_bytes - w_out;

  if ((rc = grow_pinned(&s->h_in, &s->h_in_cap, in_bytes)) != TBG_OK) return rc;
  if ((rc = grow_pinned(&s->h_out, &s->h_out_cap, out_bytes)) != TBG_OK) return rc;
  if ((rc = grow_device(&s->d_in, &s->d_in_cap, in_bytes)) != TBG_OK) return rc;
  if ((rc = grow_device(&s->d_work, &s->d_work_cap, work_bytes)) != TBG_OK) return rc;
  // Reserve the slot (busy, its old tickets expired) and pack WITHOUT the
  // context lock: a 16-batch group is ~70 MB of host copies, during which
  // other threads' tbg_poll / tbg_collect / tbg_submit must not wait.
  s->parts.clear();
  s->busy = true;
  lk.unlock();
  const auto t_pack = std::chrono::steady_clock::now();

  // ---- pack: batch k's duties / partials / messages follow batch k-1's,
  // every index rebased by the running offsets ----
  uint8_t* h = s->h_in;
  uint32_t* msg_off = (uint32_t*)(h + o_msg_off);
  uint32_t* duty_msg = (uint32_t*)(h + o_duty_msg);
  uint32_t* duty_first = (uint32_t*)(h + o_duty_first);
  uint32_t* thr = (uint32_t*)(h + o_thr);
  uint32_t* pd = (uint32_t*)(h + o_pduty);
  // offsets first, then every caller batch packed by its own worker (the
  // sections are disjoint): a 16-batch group is ~70 MB of host copies, which
  // one thread would take longer to pack than the GPU takes to run it
  std::vector<Part> parts(n_batches);
  std::vector<uint32_t> mb0(n_batches);
  uint32_t D = 0, P = 0, M = 0, MB = 0;
  for (uint32_t k = 0; k < n_batches; ++k) {
    const tbg_batch* b = bs[k];
    parts[k].d0 = D;
    parts[k].nd = b->n_duties;
    parts[k].p0 = P;
    parts[k].np = b->n_partials;
    parts[k].m0 = M;
    parts[k].nm = verify ? b->n_msgs : 0;
    mb0[k] = MB;
    D += parts[k].nd;
    P += parts[k].np;
    M += parts[k].nm;
    if (verify) MB += b->msg_off[b->n_msgs];
  }
  auto pack = [&](uint32_t k) {
    const tbg_batch* b = bs[k];
    const uint32_t D = parts[k].d0, P = parts[k].p0, M = parts[k].m0, MB = mb0[k];
    const uint32_t bnd = b->n_duties, bnp = b->n_partials, bnm = parts[k].nm;
    if (verify) {
      const uint32_t bmb = b->msg_off[bnm];
      if (bmb) memcpy(h + o_msgs + MB, b->msgs, bmb);
      for (uint32_t m = 0; m < bnm; ++m) msg_off[M + m] = MB + b->msg_off[m];
      for (uint32_t d = 0; d < bnd; ++d) duty_msg[D + d] = M + b->duty_msg[d];
      memcpy(h + o_pk + 4ull * P, b->pubkey_ids, 4ull * bnp);
    }
    for (uint32_t d = 0; d < bnd; ++d) {
      duty_first[D + d] = P + b->duty_first[d];
      for (uint32_t j = b->duty_first[d]; j < b->duty_first[d + 1]; ++j) pd[P + j] = D + d;
    }
    if (op == TBG_OP_VERIFY_AGGREGATE) memcpy(thr + D, b->duty_threshold, 4ull * bnd);
    else memset(thr + D, 0, 4ull * bnd);
    if (bnp) {
      memcpy(h + o_sigs + 96ull * P, b->sigs, 96ull * bnp);
      memcpy(h + o_ids + P, b->identifiers, bnp);
    }
  };
  const uint32_t workers = (np >= (1u << 16) && n_batches > 1) ? std::min<uint32_t>(n_batches, 8) : 1;
  if (workers == 1) {
    for (uint32_t k = 0; k < n_batches; ++k) pack(k);
  } else {
    std::vector<std::thread> th;
    for (uint32_t w = 0; w < workers; ++w)
      th.emplace_back([&, w] {
        for (uint32_t k = w; k < n_batches; k += workers) pack(k);
      });
    for (auto& t : th) t.join();
  }
  duty_first[nd] = np;
  if (verify) msg_off[nm] = MB;
  const auto t_packed = std::chrono::steady_clock::now();

  lk.lock();
  // from here on a failure releases the reserved slot
  auto release = [&](int code) {
    s->busy = false;
    return code;
  };
  if (hipSetDevice(c->device) != hipSuccess) return release(TBG_E_DEVICE);
  DevBatch B{};
  memset(&B, 0, sizeof(B));
  B.op = op;
  B.n_duties = nd;
  B.n_partials = np;
  B.n_msgs = nm;
  uint8_t* di = s->d_in;
  uint8_t* dw = s->d_work;
  B.msgs = di + o_msgs;
  B.msg_off = (const uint32_t*)(di + o_msg_off);
  B.duty_msg = (const uint32_t*)(di + o_duty_msg);
  B.duty_first = (const uint32_t*)(di + o_duty_first);
  B.duty_threshold = (const uint32_t*)(di + o_thr);
  B.partial_duty = (const uint32_t*)(di + o_pduty);
  B.sigs = di + o_sigs;
  B.identifiers = di + o_ids;
  B.pubkey_ids = (const uint32_t*)(di + o_pk);
  B.sig_aff = (G2A*)(dw + w_sig_aff);
  B.h_aff = (G2A*)(dw + w_h_aff);
  B.h_status = (int32_t*)(dw + w_h_st);
  B.h_jac = (G2J*)(dw + w_h_jac);
  B.lam = (uint32_t*)(dw + w_lam);
  B.sig_lines = (uint32_t*)(dw + w_sl);
  B.h_lines = (uint32_t*)(dw + w_hl);
  B.rlc_group = G;
  {
    uint64_t k[4];
    if (c->rlc_seed) {
      uint64_t z = c->rlc_seed;  // splitmix64: fixed, reproducible scalars (tests only)
      for (auto& w : k) {
        z += 0x9E3779B97F4A7C15ull;
        uint64_t x = z;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        w = x ^ (x >> 31);
      }
    } else {
      std::random_device rd;  // the OS entropy source (getrandom / /dev/urandom)
      for (auto& w : k) w = ((uint64_t)rd() << 32) ^ rd() ^ (++c->seed_ctr * 0x9E3779B97F4A7C15ull);
    }
    for (int j = 0; j < 4; ++j) {
      B.rlc_seed[2 * j] = (uint32_t)(k[j] >> 32);
      B.rlc_seed[2 * j + 1] = (uint32_t)k[j];
    }
    // The batched subgroup test's key never follows rlc_seed:
    // its soundness needs coefficients a submitter cannot predict.
    std::random_device rd;
    for (auto& w : B.sgb_seed) w = rd() ^ (uint32_t)(++c->seed_ctr * 0x9E3779B9u);
  }
  B.rlc_chunk = C;
  B.part_p = (G1J*)(dw + w_pp);
  B.part_s = (G2J*)(dw + w_ps);
  B.chunk_f = (uint32_t*)(dw + w_cf);
  B.chunk_list = (uint32_t*)(dw + w_cl);
  B.chunk_lines = B.sig_lines;  // (one fallback line buffer, see w_sl)
  B.dv_p = (G1A*)(dw + w_dvp);
  B.dv_s = (G2J*)(dw + w_dvs);
  B.dv_state = (int32_t*)(dw + w_dvst);
  B.grp_state = (int32_t*)(dw + w_gst);
  B.grp_lines = (uint32_t*)(dw + w_gl);
  B.counters = (uint32_t*)(dw + w_cnt);
  B.part_list = (uint32_t*)(dw + w_pl);
  B.id_fe = (uint32_t*)(dw + w_dvfe);
  B.pend_pts = (G2A*)(dw + w_pend);
  B.chunk_fe = (uint32_t*)(dw + w_cfe);
  B.cid_list = (uint32_t*)(dw + w_cidl);
  B.cid_p = (G1A*)(dw + w_cidp);
  B.cid_lines = B.sig_lines;
  // Level 1g is opt-in (tbg_config.gident).  Measured
  // (profiles/r03/gident/): +7 % at 1 % invalid in 20-step runs, whose three
  // launches reach their latency-bound fallback levels together, but -3 % at
  // 48 steps and -11 % on config 5, where launches overlap and the
  // narrowing's shorter lists matter more than its extra levels.
  B.gident = G > 1 && G <= 64 ? c->gident : 0u;  // (level 1g's lines kernel runs a lane per duty of a group)
  B.grp_fe = (uint32_t*)(dw + w_gfe);
  B.gid_list = (uint32_t*)(dw + w_gidl);
  B.gid_p = (G1A*)(dw + w_gidp);
  B.gid_lines = B.sig_lines;
  B.gid_f = (uint32_t*)(dw + w_gidf);
  B.id_list = (uint32_t*)(dw + w_idl);
  B.id_p = (G1A*)(dw + w_idp);
  B.id_lines = B.sig_lines;
  B.fb_window = fb_w;
  {
    // full-grid passes of the duty / partial lists: those the collected
    // batches' invalid share makes likely (10x margin), every pass for the
    // per-partial schedule
    const double share = std::min(1.0, 10.0 * c->invalid_ema);
    const uint64_t expect = (uint64_t)((double)np * share);
    B.fb_full = (!TBG_FB_EXPECT || G == 0 || fb_w == 0) ? 0xFFFFFFFFu
                                      : (uint32_t)std::min<uint64_t>(0xFFFFFFFFull, (expect / fb_w + 1) * (uint64_t)fb_w);
  }
  B.fb_base = 0;
  B.partial_status = (int32_t*)(dw + w_pst);
  B.duty_status = (int32_t*)(dw + w_dst);
  B.agg = dw + w_agg;
  B.rlc_batch = l0 ? 1u : 0u;
  B.msm_r = (uint64_t*)(dw + w_mr);
  B.msm_off = (uint32_t*)(dw + w_moff);
  B.msm_cur = (uint32_t*)(dw + w_mcur);
  B.msm_ent = (uint32_t*)(dw + w_ment);
  B.msm_bkt = (G2J*)(dw + w_mbkt);
  B.msm_part = (G2J*)(dw + w_mpart);
  B.msm_sum = (G2J*)(dw + w_msum);
  B.batch_pt = (G2A*)(dw + w_bpt);
  B.batch_lines = (uint32_t*)(dw + w_blines);
  B.batch_f = (uint32_t*)(dw + w_bf);
  B.grp_f = (uint32_t*)(dw + w_gf);
  B.gm_off = (uint32_t*)(dw + w_gmoff);
  B.gm_ent = (uint32_t*)(dw + w_gment);
  B.gm_part = (G2J*)(dw + w_gmpart);
  B.gm_lead = (uint32_t*)(dw + w_gmlead);
  B.gm_list = (uint32_t*)(dw + w_gmlist);
  B.gm_hist = (uint32_t*)(dw + w_gmhist);
  B.gm_order = (uint32_t*)(dw + w_gmorder);
  B.sgb = sgb ? 1u : 0u;
  B.sgb_m = sgb_m;
  B.sgb_split = sgb_split;
  B.sgb_off = (uint32_t*)(dw + w_sgoff);
  B.sgb_ent = (uint32_t*)(dw + w_sgent);
  B.sgb_part = (G2J*)(dw + w_sgpart);
  B.sgb_bad = (uint32_t*)(dw + w_sgbad);
  B.agg_acc = (G2J*)(dw + w_aacc);
  B.agg_list = (uint32_t*)(dw + w_alist);

  hipStream_t st = s->st;
  // The resident pubkey table may have been (re)loaded on the utility stream
  // (already complete: tbg_load_pubkeys waits for it; ordered anyway).
  if (hipStreamWaitEvent(st, c->keys_ready, 0) != hipSuccess ||
      hipMemcpyAsync(s->d_in, s->h_in, in_bytes, hipMemcpyHostToDevice, st) != hipSuccess)
    return release(TBG_E_DEVICE);
  rc = launch_chain(c, *s, B, s->ev);
  if (rc != TBG_OK) return release(rc);
  if (hipMemcpyAsync(s->h_out, dw + w_out, out_bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipEventRecord(s->done, st) != hipSuccess)
    return release(TBG_E_DEVICE);
  {
    const auto t_end = std::chrono::steady_clock::now();
    using ns = std::chrono::nanoseconds;
    c->host[0] += 1;
    c->host[1] += np;
    c->host[2] += (uint64_t)std::chrono::duration_cast<ns>(t_packed - t_pack).count();
    c->host[3] += (uint64_t)std::chrono::duration_cast<ns>(t_end - t_packed).count();
  }

  for (uint32_t k = 0; k < n_batches; ++k) {
    parts[k].ticket = c->next_ticket++;
    parts[k].pending = true;
    tickets[k] = parts[k].ticket;
  }
  s->parts = std::move(parts);
  s->seen_bad = s->seen_total = 0;
  s->seen_nsub = s->seen_dec = 0;
  s->busy = true;
  s->ticket = s->parts[0].ticket;
  s->op = op;
  s->n_duties = nd;
  s->n_partials = np;
  s->n_msgs = nm;
  s->out_bytes = out_bytes;
  s->B = B;
  s->last = B;
  s->w_out = w_out;
  return TBG_OK;
}

int tbg_poll(tbg_ctx* c, tbg_ticket t) {
  if (!c) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, true, nullptr);
  if (!s) return TBG_E_TICKET;
  HIP_TRY(hipSetDevice(c->device));
  hipError_t q = hipEventQuery(s->done);
  if (q == hipErrorNotReady) return TBG_E_PENDING;
  return q == hipSuccess ? TBG_OK : TBG_E_DEVICE;
}

// A part's slice of the slot's (pinned) output image.
static void copy_part(const Slot* s, const Part& q, int32_t* pst, int32_t* dst, uint8_t* agg) {
  const uint32_t np = s->n_partials, nd = s->n_duties;
  size_t o = 0;
  auto sec = [&](size_t bytes) { size_t at = o; o = align_up(o + bytes, 16); return at; };
  size_t o_pst = sec(4ull * np), o_dst = sec(4ull * nd), o_agg = sec(96ull * nd);
  if (pst) memcpy(pst, s->h_out + o_pst + 4ull * q.p0, 4ull * q.np);
  if (dst) memcpy(dst, s->h_out + o_dst + 4ull * q.d0, 4ull * q.nd);
  if (agg) memcpy(agg, s->h_out + o_agg + 96ull * q.d0, 96ull * q.nd);
}

static void part_done(Slot* s, Part* q) {
  q->pending = false;
  bool any = false;
  for (const auto& x : s->parts) any |= x.pending;
  s->busy = any;
}

int tbg_collect(tbg_ctx* c, tbg_ticket t, int32_t* pst, int32_t* dst, uint8_t* agg, int block) {
  if (!c) return TBG_E_INVALID_ARG;
  std::unique_lock<std::mutex> lk(c->mu);
  Part* q = nullptr;
  Slot* s = find_ticket(c, t, true, &q);
  if (!s || q->collecting) return TBG_E_TICKET;
  HIP_TRY(hipSetDevice(c->device));
  hipError_t e = hipEventQuery(s->done);
  if (e == hipErrorNotReady) {
    if (!block) return TBG_E_PENDING;
    // Wait without the context mutex: other threads keep submitting and
    // polling meanwhile.  The slot stays busy (this part is pending) and
    // `collecting` keeps a second collect of the same ticket out.
    q->collecting = true;
    hipEvent_t done = s->done;
    int dev = c->device;
    lk.unlock();
    const auto t_wait = std::chrono::steady_clock::now();
    (void)hipSetDevice(dev);  // the HIP current device is per thread
    e = hipEventSynchronize(done);
    c->host[7] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                                 t_wait).count();
    lk.lock();
    q->collecting = false;
  }
  if (e != hipSuccess) {
    part_done(s, q);
    return TBG_E_DEVICE;
  }
  const auto t_gather = std::chrono::steady_clock::now();
  copy_part(s, *q, pst, dst, agg);
  if (s->op != TBG_OP_AGGREGATE && q->np) {  // the adaptive group size's and level 0's input
    const int32_t* st = (const int32_t*)s->h_out;  // partial statuses lead the output region
    uint32_t bad = 0;
    for (uint32_t i = 0; i < q->np; ++i) bad += st[q->p0 + i] == TBG_PS_INVALID ? 1u : 0u;
    s->seen_bad += bad;
    s->seen_total += q->np;
  }
  if (q->np) {  // the batched subgroup test's input: non-subgroup share of all partials
    const int32_t* st = (const int32_t*)s->h_out;
    uint32_t ns = 0;
    for (uint32_t i = 0; i < q->np; ++i) ns += st[q->p0 + i] == TBG_PS_ERR_SUBGROUP ? 1u : 0u;
    s->seen_nsub += ns;
    s->seen_dec += q->np;
  }
  c->host[4] += 1;
  c->host[5] += q->np;
  c->host[6] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                               t_gather).count();
  chain_times(s->ev, s->ms);
  memcpy(c->last_ms, s->ms, sizeof(c->last_ms));
  part_done(s, q);
  // One update per DEVICE batch, over all of its parts (whatever order they
  // are collected in), once its last part is collected.
  if (!s->busy && s->seen_total) {
    c->invalid_ema = 0.5 * c->invalid_ema + 0.5 * (double)s->seen_bad / (double)s->seen_total;
    s->seen_bad = s->seen_total = 0;
  }
  if (!s->busy && s->seen_dec) {
    c->nonsub_ema = 0.5 * c->nonsub_ema + 0.5 * (double)s->seen_nsub / (double)s->seen_dec;
    s->seen_nsub = s->seen_dec = 0;
  }
  return TBG_OK;
}

int tbg_run(tbg_ctx* c, const tbg_batch* b, int32_t* pst, int32_t* dst, uint8_t* agg) {
  tbg_ticket t;
  int rc = tbg_submit(c, b, &t);
  if (rc != TBG_OK) return rc;
  return tbg_collect(c, t, pst, dst, agg, 1);
}

int tbg_replay_plan(tbg_ctx* c, const tbg_ticket* tickets, const uint32_t* n_parts, uint32_t n_launches, float* ms8) {
  if (!c || !tickets || n_launches == 0) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  std::vector<Slot*> sl(n_launches, nullptr);
  std::vector<DevBatch> bs(n_launches);
  for (uint32_t k = 0; k < n_launches; ++k) {
    sl[k] = find_ticket(c, tickets[k], false, nullptr);
    if (!sl[k]) return TBG_E_TICKET;
    // A prefix of the packed device batch is itself a batch: batch j's
    // duties, partials and messages all follow batch j-1's.
    DevBatch B = sl[k]->B;
    const uint32_t np = n_parts ? n_parts[k] : 0;
    if (np > sl[k]->parts.size()) return TBG_E_INVALID_ARG;
    if (np && np < sl[k]->parts.size()) {
      const Part& last = sl[k]->parts[np - 1];
      B.n_duties = last.d0 + last.nd;
      B.n_partials = last.p0 + last.np;
      B.n_msgs = last.m0 + last.nm;
    }
    bs[k] = B;
  }
  HIP_TRY(hipSetDevice(c->device));
  std::vector<hipEvent_t> ev((size_t)kChainEvents * n_launches);
  for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
  int rc = TBG_OK;
  // Launch k on the streams of its slot: launches of different slots are in
  // flight together, launches of one slot run in order.  Runs of launches on
  // distinct slots are enqueued stage by stage (launch_chain), so their
  // first kernels start together (each launch waiting for the previous one's
  // hash or H(m) lines was measured 11-12 % slower at 20 steps, round 5:
  // profiles/r05/stagger/).
  for (uint32_t k0 = 0; k0 < n_launches && rc == TBG_OK;) {
    uint32_t k1 = k0 + 1;
    while (k1 < n_launches && std::find(sl.begin() + k0, sl.begin() + k1, sl[k1]) == sl.begin() + k1) ++k1;
#if TBG_REPLAY_SHAPE
    // The level-0 launches run together share the SIMDs: their shape follows
    // their duties together (l0_shape), where each launch's arena fits it.
    if (c->chunk_auto && c->rlc_auto) {
      uint64_t nd = 0;
      bool all_l0 = true;
      for (uint32_t k = k0; k < k1; ++k) {
        nd += bs[k].n_duties;
        all_l0 = all_l0 && bs[k].rlc_batch && bs[k].rlc_group >= 8;
      }
      // the cheapest shape every launch of the run can hold (round 6: the
      // candidates that one of them cannot are skipped, not the reshape)
      uint32_t G = 16, C = 4;
      auto fits_all = [&](uint32_t g, uint32_t ch) {
        for (uint32_t k = k0; k < k1; ++k)
          if (!l0_shape_fits(sl[k]->n_duties, sl[k]->B.rlc_group, sl[k]->B.rlc_chunk, bs[k].n_duties, g, ch))
            return false;
        return true;
      };
      if (all_l0) l0_shape(nd, c->n_simd, true, G, C, fits_all);
      for (uint32_t k = k0; k < k1 && all_l0; ++k)
        if (l0_shape_fits(sl[k]->n_duties, sl[k]->B.rlc_group, sl[k]->B.rlc_chunk, bs[k].n_duties, G, C)) {
          bs[k].rlc_group = G;
          bs[k].rlc_chunk = C;
        }
    }
#endif
    for (int stage = 0; stage < 3 && rc == TBG_OK; ++stage) {
#if TBG_L0_JOIN
      // The run's level-0 Miller kernels start once every launch of the run
      // has its signature side (S, P_d, S's lines): a Miller kernel that
      // starts early holds the SIMDs for ~14 ms while the other launches'
      // one-workgroup MSM tails wait for a slot behind it.
      if (stage == 2 && k1 - k0 > 1)
        for (uint32_t k = k0; k < k1 && rc == TBG_OK; ++k)
          for (uint32_t j = k0; j < k1; ++j)
            if (j != k && bs[k].rlc_batch && bs[j].rlc_batch &&
                hipStreamWaitEvent(sl[k]->st, ev[(size_t)kChainEvents * j + 2], 0) != hipSuccess)
              rc = TBG_E_DEVICE;
#endif
      for (uint32_t k = k0; k < k1 && rc == TBG_OK; ++k)
        rc = launch_chain(c, *sl[k], bs[k], ev.data() + (size_t)kChainEvents * k, stage);
    }
    for (uint32_t k = k0; k < k1; ++k) sl[k]->last = bs[k];
    k0 = k1;
  }
  for (uint32_t k = 0; k < n_launches; ++k) {
    if (hipStreamSynchronize(sl[k]->st) != hipSuccess) rc = TBG_E_DEVICE;
    if (hipStreamSynchronize(sl[k]->st2) != hipSuccess) rc = TBG_E_DEVICE;
  }
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rc == TBG_OK) {
    for (uint32_t k = 0; k < n_launches; ++k) {
      float m[8];
      chain_times(ev.data() + (size_t)kChainEvents * k, m);
      for (int j = 0; j < 7; ++j) acc[j] += m[j];
    }
    // wall time: first launch's start to the latest chain end
    for (uint32_t k = 0; k < n_launches; ++k) {
      float w = 0;
      hipEventElapsedTime(&w, ev[0], ev[(size_t)kChainEvents * k + 9]);
      if (w > acc[7]) acc[7] = w;
    }
    if (ms8) memcpy(ms8, acc, sizeof(acc));
    memcpy(c->last_ms, acc, sizeof(acc));
  }
  for (auto& e : ev) hipEventDestroy(e);
  return rc;
}

int tbg_replay_profile(tbg_ctx* c, tbg_ticket t, tbg_kernel_time* out, uint32_t max_entries, uint32_t* n_entries) {
  if (!c || !n_entries || (max_entries && !out)) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, false, nullptr);
  if (!s) return TBG_E_TICKET;
  HIP_TRY(hipSetDevice(c->device));
  // nothing else of this context in flight: every kernel runs alone
  for (auto& x : c->slots) {
    HIP_TRY(hipStreamSynchronize(x.st));
    HIP_TRY(hipStreamSynchronize(x.st2));
  }
  std::vector<KProfRec> rec;
  hipEvent_t ev[kChainEvents];
  for (auto& e : ev) HIP_TRY(hipEventCreate(&e));
  g_kprof = &rec;
  int rc = launch_chain(c, *s, s->B, ev);
  s->last = s->B;
  g_kprof = nullptr;
  if (hipStreamSynchronize(s->st) != hipSuccess || hipStreamSynchronize(s->st2) != hipSuccess) rc = TBG_E_DEVICE;
  uint32_t n = 0;
  for (auto& r : rec) {
    if (rc == TBG_OK && n < max_entries) {
      float ms = 0;
      if (!r.a || !r.b || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) rc = TBG_E_DEVICE;
      snprintf(out[n].name, sizeof(out[n].name), "%s", r.name);
      out[n].ms = ms;
      ++n;
    }
    if (r.a) hipEventDestroy(r.a);
    if (r.b) hipEventDestroy(r.b);
  }
  for (auto& e : ev) hipEventDestroy(e);
  *n_entries = n;
  return rc;
}

int tbg_replay_multi(tbg_ctx* c, const tbg_ticket* tickets, uint32_t n_tickets, uint32_t iters, float* ms8) {
  if (!c || !tickets || n_tickets == 0 || iters == 0) return TBG_E_INVALID_ARG;
  std::vector<tbg_ticket> plan(iters);
  for (uint32_t k = 0; k < iters; ++k) plan[k] = tickets[k % n_tickets];  // round-robin over the resident batches
  return tbg_replay_plan(c, plan.data(), nullptr, iters, ms8);
}

int tbg_replay(tbg_ctx* c, tbg_ticket t, uint32_t iters, float* ms8) { return tbg_replay_multi(c, &t, 1, iters, ms8); }

int tbg_fetch(tbg_ctx* c, tbg_ticket t, int32_t* pst, int32_t* dst, uint8_t* agg) {
  if (!c) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Part* q = nullptr;
  Slot* s = find_ticket(c, t, false, &q);
  if (!s) return TBG_E_TICKET;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(s->h_out, s->d_work + s->w_out, s->out_bytes, hipMemcpyDeviceToHost, s->st));
  HIP_TRY(hipStreamSynchronize(s->st));
  copy_part(s, *q, pst, dst, agg);
  return TBG_OK;
}

int tbg_fetch_stats(tbg_ctx* c, tbg_ticket t, uint32_t* out4) {
  if (!c || !out4) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, false, nullptr);
  if (!s) return TBG_E_TICKET;
  HIP_TRY(hipSetDevice(c->device));
  uint32_t cnt[CNT_WORDS] = {};
  if (s->op != TBG_OP_AGGREGATE) {
    HIP_TRY(hipMemcpyAsync(cnt, s->last.counters, sizeof(cnt), hipMemcpyDeviceToHost, s->st));
    HIP_TRY(hipStreamSynchronize(s->st));
  }
  uint32_t ng = s->last.rlc_group ? (s->last.n_duties + s->last.rlc_group - 1) / s->last.rlc_group : 0;
  out4[0] = ng;
  out4[1] = cnt[CNT_DUTIES];
  out4[2] = cnt[CNT_PARTIALS];
  out4[3] = s->last.rlc_group;
  return TBG_OK;
}

int tbg_fetch_fallback(tbg_ctx* c, tbg_ticket t, uint32_t* out8) {
  if (!c || !out8) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, false, nullptr);
  if (!s) return TBG_E_TICKET;
  HIP_TRY(hipSetDevice(c->device));
  uint32_t cnt[CNT_WORDS] = {};
  if (s->op != TBG_OP_AGGREGATE) {
    HIP_TRY(hipMemcpyAsync(cnt, s->last.counters, sizeof(cnt), hipMemcpyDeviceToHost, s->st));
    HIP_TRY(hipStreamSynchronize(s->st));
  }
  out8[0] = s->last.rlc_group ? (s->last.n_duties + s->last.rlc_group - 1) / s->last.rlc_group : 0;
  out8[1] = cnt[CNT_GID];
  out8[2] = cnt[CNT_CHUNKS];
  out8[3] = cnt[CNT_CID];
  out8[4] = cnt[CNT_DUTIES];
  out8[5] = cnt[CNT_PARTIALS];
  out8[6] = s->last.rlc_group;
  out8[7] = s->op == TBG_OP_AGGREGATE || !s->last.rlc_batch ? (uint32_t)TBG_L0_NOT_RUN
            : cnt[CNT_L0_OK]                              ? (uint32_t)TBG_L0_PASSED
                                                          : (uint32_t)TBG_L0_FAILED;
  return TBG_OK;
}

int tbg_fetch_shape(tbg_ctx* c, tbg_ticket t, uint32_t* out4) {
  if (!c || !out4) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, false, nullptr);
  if (!s) return TBG_E_TICKET;
  const uint32_t G = s->last.rlc_group, C = s->last.rlc_chunk;
  out4[0] = G;
  out4[1] = G ? C : 0;
  out4[2] = s->last.rlc_batch ? 1u : 0u;
  out4[3] = G ? ((s->last.n_duties + G - 1) / G) * ((G + C - 1) / C) : 0;
  return TBG_OK;
}

int tbg_fetch_subgroup(tbg_ctx* c, tbg_ticket t, uint32_t* out3) {
  if (!c || !out3) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, false, nullptr);
  if (!s) return TBG_E_TICKET;
  HIP_TRY(hipSetDevice(c->device));
  out3[0] = out3[1] = out3[2] = 0;
  if (!s->last.sgb) return TBG_OK;
  out3[2] = s->last.sgb_m;
  const uint32_t n_sg = sgb_groups(s->last.n_partials, s->last.sgb_m);
  std::vector<uint32_t> bad(n_sg);
  HIP_TRY(hipMemcpyAsync(bad.data(), s->last.sgb_bad, 4ull * n_sg, hipMemcpyDeviceToHost, s->st));
  HIP_TRY(hipStreamSynchronize(s->st));
  out3[0] = n_sg;
  for (uint32_t g = 0; g < n_sg; ++g) out3[1] += bad[g] ? 1u : 0u;
  return TBG_OK;
}

int tbg_host_stats(tbg_ctx* c, uint64_t* out8, int reset) {
  if (!c || !out8) return TBG_E_INVALID_ARG;
  for (int k = 0; k < 8; ++k) out8[k] = reset ? c->host[k].exchange(0) : c->host[k].load();
  return TBG_OK;
}

int tbg_slot_bytes(tbg_ctx* c, tbg_ticket t, uint64_t* device_bytes, uint64_t* pinned_bytes) {
  if (!c || !device_bytes || !pinned_bytes) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, false, nullptr);
  if (!s) return TBG_E_TICKET;
  *device_bytes = (uint64_t)s->d_in_cap + (uint64_t)s->d_work_cap;
  *pinned_bytes = (uint64_t)s->h_in_cap + (uint64_t)s->h_out_cap;
  return TBG_OK;
}

int tbg_fetch_level0(tbg_ctx* c, tbg_ticket t, int32_t* state) {
  if (!c || !state) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  Slot* s = find_ticket(c, t, false, nullptr);
  if (!s) return TBG_E_TICKET;
  *state = TBG_L0_NOT_RUN;
  if (s->op == TBG_OP_AGGREGATE || !s->last.rlc_batch) return TBG_OK;
  HIP_TRY(hipSetDevice(c->device));
  uint32_t cnt[CNT_WORDS] = {};
  HIP_TRY(hipMemcpyAsync(cnt, s->last.counters, sizeof(cnt), hipMemcpyDeviceToHost, s->st));
  HIP_TRY(hipStreamSynchronize(s->st));
  *state = cnt[CNT_L0_OK] ? TBG_L0_PASSED : TBG_L0_FAILED;
  return TBG_OK;
}

int tbg_last_timings(const tbg_ctx* c, float* ms8) {
  if (!c || !ms8) return TBG_E_INVALID_ARG;
  memcpy(ms8, c->last_ms, sizeof(c->last_ms));
  return TBG_OK;
}

}  // extern "C"

extern "C" {

int tbg_sk_to_pk(tbg_ctx* c, const uint8_t* sk32, uint32_t n, uint8_t* pk48) {
  if (!c || (n && (!sk32 || !pk48))) return TBG_E_INVALID_ARG;
  if (n == 0) return TBG_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  uint8_t *d_sk = nullptr, *d_pk = nullptr;
  if (hipMalloc(&d_sk, 32ull * n) != hipSuccess) return TBG_E_OOM;
  if (hipMalloc(&d_pk, 48ull * n) != hipSuccess) { hipFree(d_sk); return TBG_E_OOM; }
  int rc = TBG_OK;
  if (hipMemcpyAsync(d_sk, sk32, 32ull * n, hipMemcpyHostToDevice, c->stream) != hipSuccess) rc = TBG_E_DEVICE;
  if (rc == TBG_OK) {
    launch_sk_to_pk(d_sk, n, d_pk, c->stream);
    if (hipGetLastError() != hipSuccess) rc = TBG_E_DEVICE;
  }
  if (rc == TBG_OK && hipMemcpyAsync(pk48, d_pk, 48ull * n, hipMemcpyDeviceToHost, c->stream) != hipSuccess) rc = TBG_E_DEVICE;
  if (hipStreamSynchronize(c->stream) != hipSuccess) rc = TBG_E_DEVICE;
  hipFree(d_sk);
  hipFree(d_pk);
  return rc;
}

int tbg_sign(tbg_ctx* c, const uint8_t* sk32, uint32_t n, const uint8_t* msgs, const uint32_t* msg_off, uint32_t n_msgs,
             const uint32_t* item_msg, uint8_t* sig96) {
  if (!c || (n && (!sk32 || !sig96 || !item_msg)) || n_msgs == 0 || !msg_off) return TBG_E_INVALID_ARG;
  if (msg_off[0] != 0) return TBG_E_INVALID_ARG;
  for (uint32_t m = 0; m < n_msgs; ++m)
    if (msg_off[m + 1] < msg_off[m]) return TBG_E_INVALID_ARG;
  for (uint32_t i = 0; i < n; ++i)
    if (item_msg[i] >= n_msgs) return TBG_E_INVALID_ARG;
  if (n == 0) return TBG_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  size_t mb = msg_off[n_msgs];
  size_t need = align_up(32ull * n, 16) + align_up(mb + 1, 16) + align_up(4ull * (n_msgs + 1), 16) + align_up(4ull * n, 16) +
                align_up(sizeof(G2A) * (size_t)n_msgs, 16) + align_up(4ull * n_msgs, 16) + align_up(96ull * n, 16) +
                align_up(3 * sizeof(G2J) * (size_t)n_msgs, 16);
  uint8_t* base = nullptr;
  if (hipMalloc(&base, need) != hipSuccess) return TBG_E_OOM;
  size_t o = 0;
  auto sec = [&](size_t bytes) { uint8_t* p = base + o; o += align_up(bytes, 16); return p; };
  uint8_t* d_sk = sec(32ull * n);
  uint8_t* d_msgs = sec(mb + 1);
  uint32_t* d_off = (uint32_t*)sec(4ull * (n_msgs + 1));
  uint32_t* d_im = (uint32_t*)sec(4ull * n);
  G2A* d_h = (G2A*)sec(sizeof(G2A) * (size_t)n_msgs);
  int32_t* d_hs = (int32_t*)sec(4ull * n_msgs);
  uint8_t* d_sig = sec(96ull * n);
  G2J* d_hj = (G2J*)sec(3 * sizeof(G2J) * (size_t)n_msgs);
  int rc = TBG_OK;
  hipStream_t st = c->stream;
  if (hipMemcpyAsync(d_sk, sk32, 32ull * n, hipMemcpyHostToDevice, st) != hipSuccess ||
      (mb && hipMemcpyAsync(d_msgs, msgs, mb, hipMemcpyHostToDevice, st) != hipSuccess) ||
      hipMemcpyAsync(d_off, msg_off, 4ull * (n_msgs + 1), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(d_im, item_msg, 4ull * n, hipMemcpyHostToDevice, st) != hipSuccess)
    rc = TBG_E_DEVICE;
  if (rc == TBG_OK) {
    DevBatch B{};
    memset(&B, 0, sizeof(B));
    B.n_msgs = n_msgs;
    B.msgs = d_msgs;
    B.msg_off = d_off;
    B.h_aff = d_h;
    B.h_status = d_hs;
    B.h_jac = d_hj;
    launch_hash_msgs(B, st);
    launch_sign(d_sk, d_im, n, d_h, d_hs, d_sig, st);
    if (hipGetLastError() != hipSuccess) rc = TBG_E_DEVICE;
  }
  if (rc == TBG_OK && hipMemcpyAsync(sig96, d_sig, 96ull * n, hipMemcpyDeviceToHost, st) != hipSuccess) rc = TBG_E_DEVICE;
  if (hipStreamSynchronize(st) != hipSuccess) rc = TBG_E_DEVICE;
  hipFree(base);
  return rc;
}

// ---- plain sums and FastAggregateVerify (k_sum.hip) -----------------------
// dkg/dkg.go:466-476 (AggregateSignatures / AggregatePublicKeys of the lock
// hash), cluster/lock.go:155-177 (FastAggregateVerify over every pubshare).

}  // extern "C"

namespace {

// One device allocation for a utility call, freed on scope exit.
struct DevArena {
  uint8_t* base = nullptr;
  size_t o = 0;
  ~DevArena() {
    if (base) hipFree(base);
  }
  int alloc(size_t bytes) { return hipMalloc(&base, bytes ? bytes : 16) == hipSuccess ? TBG_OK : TBG_E_OOM; }
  uint8_t* sec(size_t bytes) {
    uint8_t* p = base + o;
    o += align_up(bytes, 16);
    return p;
  }
};

bool offsets_ok(const uint32_t* off, uint32_t n_sets) {
  if (!off || off[0] != 0) return false;
  for (uint32_t s = 0; s < n_sets; ++s)
    if (off[s + 1] < off[s]) return false;
  return true;
}

// Host half of a sum plan and its device copy inside `a`.
struct SumHost {
  std::vector<uint32_t> chunk_first, chunk_set;
  static size_t bytes(uint32_t n_sets, uint32_t n_chunks, size_t part_elem) {
    return align_up(4ull * (n_sets + 1), 16) * 2 + align_up(4ull * n_chunks + 4, 16) +
           align_up(part_elem * n_chunks + 16, 16) + align_up(4ull * n_sets + 4, 16);
  }
  SumHost(const uint32_t* off, uint32_t n_sets) {
    const uint32_t ch = tbg::sum_chunk_size();
    chunk_first.resize(n_sets + 1);
    chunk_first[0] = 0;
    for (uint32_t s = 0; s < n_sets; ++s) {
      const uint32_t nc = (off[s + 1] - off[s] + ch - 1) / ch;
      chunk_first[s + 1] = chunk_first[s] + nc;
      for (uint32_t k = 0; k < nc; ++k) chunk_set.push_back(s);
    }
  }
  uint32_t n_chunks() const { return chunk_first.back(); }
  int upload(DevArena& a, const uint32_t* off, uint32_t n_sets, size_t part_elem, hipStream_t st, tbg::SumPlan& p) {
    uint32_t* d_off = (uint32_t*)a.sec(4ull * (n_sets + 1));
    uint32_t* d_cf = (uint32_t*)a.sec(4ull * (n_sets + 1));
    uint32_t* d_cs = (uint32_t*)a.sec(4ull * n_chunks() + 4);
    p.part = a.sec(part_elem * n_chunks() + 16);
    p.set_bad = (int32_t*)a.sec(4ull * n_sets + 4);
    p.n_sets = n_sets;
    p.n_chunks = n_chunks();
    p.off = d_off;
    p.chunk_first = d_cf;
    p.chunk_set = d_cs;
    if (hipMemcpyAsync(d_off, off, 4ull * (n_sets + 1), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(d_cf, chunk_first.data(), 4ull * (n_sets + 1), hipMemcpyHostToDevice, st) != hipSuccess ||
        (n_chunks() && hipMemcpyAsync(d_cs, chunk_set.data(), 4ull * n_chunks(), hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipMemsetAsync(p.set_bad, 0, 4ull * n_sets, st) != hipSuccess)
      return TBG_E_DEVICE;
    return TBG_OK;
  }
};

}  // namespace

extern "C" {

int tbg_sum_pubkeys(tbg_ctx* c, const uint32_t* pubkey_ids, const uint32_t* off, uint32_t n_sets, uint8_t* out48,
                    int32_t* status) {
  if (!c || !n_sets || !out48 || !status || !offsets_ok(off, n_sets)) return TBG_E_INVALID_ARG;
  const uint32_t ni = off[n_sets];
  if (ni && !pubkey_ids) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  SumHost h(off, n_sets);
  DevArena a;
  int rc = a.alloc(SumHost::bytes(n_sets, h.n_chunks(), sizeof(G1J)) + align_up(4ull * ni + 4, 16) +
                   align_up(48ull * n_sets, 16) + align_up(4ull * n_sets, 16));
  if (rc != TBG_OK) return rc;
  hipStream_t st = c->stream;
  tbg::SumPlan p;
  if ((rc = h.upload(a, off, n_sets, sizeof(G1J), st, p)) != TBG_OK) return rc;
  uint32_t* d_ids = (uint32_t*)a.sec(4ull * ni + 4);
  uint8_t* d_out = a.sec(48ull * n_sets);
  int32_t* d_st = (int32_t*)a.sec(4ull * n_sets);
  if (ni) HIP_TRY(hipMemcpyAsync(d_ids, pubkey_ids, 4ull * ni, hipMemcpyHostToDevice, st));
  tbg::launch_sum_g1(c->d_pk, c->d_pk_status, c->n_pk, d_ids, p, d_out, d_st, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out48, d_out, 48ull * n_sets, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(status, d_st, 4ull * n_sets, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return TBG_OK;
}

int tbg_sum_sigs(tbg_ctx* c, const uint8_t* sigs96, const uint32_t* off, uint32_t n_sets, uint8_t* out96,
                 int32_t* status, int32_t* sig_status) {
  if (!c || !n_sets || !out96 || !status || !offsets_ok(off, n_sets)) return TBG_E_INVALID_ARG;
  const uint32_t ni = off[n_sets];
  if (ni && !sigs96) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  SumHost h(off, n_sets);
  DevArena a;
  int rc = a.alloc(SumHost::bytes(n_sets, h.n_chunks(), sizeof(G2J)) + align_up(96ull * ni + 4, 16) +
                   align_up(4ull * ni + 4, 16) + align_up(96ull * n_sets, 16) + align_up(4ull * n_sets, 16));
  if (rc != TBG_OK) return rc;
  hipStream_t st = c->stream;
  tbg::SumPlan p;
  if ((rc = h.upload(a, off, n_sets, sizeof(G2J), st, p)) != TBG_OK) return rc;
  uint8_t* d_sigs = a.sec(96ull * ni + 4);
  int32_t* d_sst = (int32_t*)a.sec(4ull * ni + 4);
  uint8_t* d_out = a.sec(96ull * n_sets);
  int32_t* d_st = (int32_t*)a.sec(4ull * n_sets);
  if (ni) HIP_TRY(hipMemcpyAsync(d_sigs, sigs96, 96ull * ni, hipMemcpyHostToDevice, st));
  tbg::launch_sum_g2(d_sigs, p, d_out, d_st, d_sst, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out96, d_out, 96ull * n_sets, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(status, d_st, 4ull * n_sets, hipMemcpyDeviceToHost, st));
  if (sig_status && ni) HIP_TRY(hipMemcpyAsync(sig_status, d_sst, 4ull * ni, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return TBG_OK;
}

int tbg_fast_aggregate_verify(tbg_ctx* c, const uint32_t* pubkey_ids, const uint32_t* key_off, uint32_t n_sets,
                              const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* sigs96, int32_t* status) {
  if (!c || !n_sets || !sigs96 || !status || !offsets_ok(key_off, n_sets) || !offsets_ok(msg_off, n_sets))
    return TBG_E_INVALID_ARG;
  const uint32_t nk = key_off[n_sets];
  const size_t mb = msg_off[n_sets];
  if ((nk && !pubkey_ids) || (mb && !msgs)) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  HIP_TRY(hipSetDevice(c->device));
  const uint32_t n = n_sets;
  SumHost h(key_off, n);
  std::vector<uint32_t> iota(n + 1);
  for (uint32_t i = 0; i <= n; ++i) iota[i] = i;
  const size_t lines = 4ull * LINES_WORDS * n;
  DevArena a;
  int rc = a.alloc(SumHost::bytes(n, h.n_chunks(), sizeof(G1J)) + align_up(4ull * nk + 4, 16) +
                   align_up(48ull * n, 16) * 2 + align_up(sizeof(G1A) * n, 16) * 2 + align_up(4ull * n, 16) * 6 +
                   align_up(mb + 1, 16) + align_up(4ull * (n + 1), 16) * 2 + align_up(96ull * n, 16) + align_up(n, 16) +
                   align_up(sizeof(G2A) * n, 16) * 2 + align_up(3 * sizeof(G2J) * n, 16) + 2 * align_up(lines, 16) +
                   align_up(4ull * tbg::CNT_WORDS, 16));
  if (rc != TBG_OK) return rc;
  hipStream_t st = c->stream;
  // 1. the key sums, compressed, then decoded into a table of their own
  tbg::SumPlan p;
  if ((rc = h.upload(a, key_off, n, sizeof(G1J), st, p)) != TBG_OK) return rc;
  uint32_t* d_ids = (uint32_t*)a.sec(4ull * nk + 4);
  uint8_t* d_pk48 = a.sec(48ull * n);
  int32_t* d_kst = (int32_t*)a.sec(4ull * n);
  G1A* t_pk = (G1A*)a.sec(sizeof(G1A) * n);
  G1A* t_xpk = (G1A*)a.sec(sizeof(G1A) * n);
  int32_t* t_pkst = (int32_t*)a.sec(4ull * n);
  if (nk) HIP_TRY(hipMemcpyAsync(d_ids, pubkey_ids, 4ull * nk, hipMemcpyHostToDevice, st));
  tbg::launch_sum_g1(c->d_pk, c->d_pk_status, c->n_pk, d_ids, p, d_pk48, d_kst, st);
  tbg::launch_decode_pubkeys(d_pk48, n, t_pk, t_xpk, t_pkst, st);  // a failed / identity sum: not DEC_OK
  // 2. one CoreVerify per set against that table (the per-item schedule)
  DevBatch B{};
  memset(&B, 0, sizeof(B));
  B.op = TBG_OP_VERIFY;
  B.n_duties = B.n_partials = B.n_msgs = n;
  uint8_t* d_msgs = a.sec(mb + 1);
  uint32_t* d_moff = (uint32_t*)a.sec(4ull * (n + 1));
  uint32_t* d_iota = (uint32_t*)a.sec(4ull * (n + 1));
  uint8_t* d_sigs = a.sec(96ull * n);
  uint8_t* d_idf = a.sec(n);
  B.msgs = d_msgs;
  B.msg_off = d_moff;
  B.duty_msg = B.duty_first = B.partial_duty = B.pubkey_ids = d_iota;
  B.duty_threshold = d_iota;  // unused by TBG_OP_VERIFY
  B.sigs = d_sigs;
  B.identifiers = d_idf;
  B.sig_aff = (G2A*)a.sec(sizeof(G2A) * n);
  B.h_aff = (G2A*)a.sec(sizeof(G2A) * n);
  B.h_status = (int32_t*)a.sec(4ull * n);
  B.h_jac = (G2J*)a.sec(3 * sizeof(G2J) * n);
  B.sig_lines = (uint32_t*)a.sec(lines);
  B.h_lines = (uint32_t*)a.sec(lines);
  B.counters = (uint32_t*)a.sec(4ull * tbg::CNT_WORDS);
  B.part_list = (uint32_t*)a.sec(4ull * n);
  B.partial_status = (int32_t*)a.sec(4ull * n);
  B.duty_status = (int32_t*)a.sec(4ull * n);
  B.rlc_group = 0;
  B.fb_full = 0xFFFFFFFFu;
  if (mb) HIP_TRY(hipMemcpyAsync(d_msgs, msgs, mb, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(d_moff, msg_off, 4ull * (n + 1), hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(d_iota, iota.data(), 4ull * (n + 1), hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(d_sigs, sigs96, 96ull * n, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemsetAsync(d_idf, 0, n, st));
  HIP_TRY(hipMemsetAsync(B.counters, 0, 4 * tbg::CNT_WORDS, st));
  tbg::launch_decode_sigs(B, st);
  tbg::launch_hash_msgs(B, st);
  tbg::launch_h_lines(B, st);
  tbg::launch_rlc_prepare(B, t_pk, t_xpk, nullptr, t_pkst, n, st);
  tbg::launch_rlc_check(B, t_pk, t_xpk, t_pkst, n, st);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(status, B.partial_status, 4ull * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return TBG_OK;
}

}  // extern "C"
