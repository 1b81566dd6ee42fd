// libtbls_gpu.so, multi-device part: one process driving several GPUs
// (BASELINE config 4: 1 M DV-duties over 8 x MI355X with a host gather).
//
// A multi-context owns one single-device context per entry of devices[].
// Duties are independent (no cross-device math), so a batch --
// or a group of callers' batches taken back to back -- is cut into contiguous
// duty ranges of about equal partial counts; every piece becomes a sub-batch
// that shares the caller's arrays by pointer offset (only duty_first is
// rebased and the messages a range uses are re-indexed), and each context's
// pieces are packed into ONE device batch (tbg_submit_group) and submitted
// concurrently on persistent per-context host workers.  Collection writes each shard's statuses and aggregates straight
// into the caller's arrays at the shard's offsets, so the gather is the
// per-DV loop order of core/parsigex/parsigex.go:101-107 and
// core/parsigdb/memory.go:96-134 -> core/sigagg/sigagg.go:53-103 by
// construction.  Host code only.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <unordered_map>
#include <vector>
#include "../../include/tbls_gpu.h"

namespace {

// One piece of a caller batch: its duties [d0, d1) (partials [p0, p1)),
// submitted to context `ctx` as part `ticket` of that context's device batch.
struct Shard {
  uint32_t ctx = 0;
  tbg_ticket ticket = 0;
  uint32_t d0 = 0, d1 = 0, p0 = 0, p1 = 0;
};

// One caller batch (one multi ticket): its pieces, at most one per context.
struct Job {
  std::vector<Shard> shards;
  std::vector<uint32_t> duty_lo;  // [size + 1] cut points in the batch's duties (empty shards included)
  bool collecting = false;
};

// Sub-batch of duties [d0, d1): pointers into the caller's arrays plus the
// few rebased index arrays it owns.
struct SubBatch {
  tbg_batch b{};
  std::vector<uint32_t> duty_first, duty_msg, msg_off;
  std::vector<uint8_t> msgs;

  void build(const tbg_batch& src, uint32_t d0, uint32_t d1) {
    const uint32_t p0 = src.duty_first[d0], p1 = src.duty_first[d1];
    b = src;
    b.n_duties = d1 - d0;
    b.n_partials = p1 - p0;
    duty_first.resize(b.n_duties + 1);
    for (uint32_t i = 0; i <= b.n_duties; ++i) duty_first[i] = src.duty_first[d0 + i] - p0;
    b.duty_first = duty_first.data();
    b.sigs = src.sigs ? src.sigs + 96ull * p0 : nullptr;
    b.identifiers = src.identifiers ? src.identifiers + p0 : nullptr;
    b.pubkey_ids = src.pubkey_ids ? src.pubkey_ids + p0 : nullptr;
    b.duty_threshold = src.duty_threshold ? src.duty_threshold + d0 : nullptr;
    if (src.op == TBG_OP_AGGREGATE) return;
    // Messages: a contiguous increasing run (one message per duty, the usual
    // attestation batch) is shared by offset; anything else (committees that
    // share a signing root) is re-indexed to the messages this range uses.
    bool run = true;
    for (uint32_t d = d0 + 1; d < d1 && run; ++d) run = src.duty_msg[d] == src.duty_msg[d - 1] + 1;
    duty_msg.resize(b.n_duties);
    if (run) {
      const uint32_t m0 = src.duty_msg[d0], nm = d1 - d0;
      msg_off.resize(nm + 1);
      for (uint32_t i = 0; i <= nm; ++i) msg_off[i] = src.msg_off[m0 + i] - src.msg_off[m0];
      for (uint32_t i = 0; i < nm; ++i) duty_msg[i] = i;
      b.msgs = src.msgs ? src.msgs + src.msg_off[m0] : nullptr;
      b.n_msgs = nm;
    } else {
      std::unordered_map<uint32_t, uint32_t> local;
      local.reserve(2 * (size_t)b.n_duties);
      msg_off.assign(1, 0);
      for (uint32_t d = d0; d < d1; ++d) {
        const uint32_t m = src.duty_msg[d];
        auto it = local.find(m);
        if (it == local.end()) {
          it = local.emplace(m, (uint32_t)local.size()).first;
          const uint32_t len = src.msg_off[m + 1] - src.msg_off[m];
          msgs.insert(msgs.end(), src.msgs + src.msg_off[m], src.msgs + src.msg_off[m] + len);
          msg_off.push_back((uint32_t)msgs.size());
        }
        duty_msg[d - d0] = it->second;
      }
      if (msgs.empty()) msgs.push_back(0);  // a valid pointer for empty messages
      b.msgs = msgs.data();
      b.n_msgs = (uint32_t)local.size();
    }
    b.msg_off = msg_off.data();
    b.duty_msg = duty_msg.data();
  }
};

// What the per-context validate() checks, for the parts the split relies on.
int validate_split(const tbg_batch* b) {
  if (!b || b->n_duties == 0 || !b->duty_first) return TBG_E_INVALID_ARG;
  if (b->op < TBG_OP_VERIFY || b->op > TBG_OP_VERIFY_AGGREGATE) return TBG_E_INVALID_ARG;
  if (b->duty_first[0] != 0 || b->duty_first[b->n_duties] != b->n_partials) return TBG_E_INVALID_ARG;
  for (uint32_t d = 0; d < b->n_duties; ++d)
    if (b->duty_first[d + 1] < b->duty_first[d]) return TBG_E_INVALID_ARG;
  if (b->op != TBG_OP_AGGREGATE) {
    if (!b->msg_off || !b->duty_msg || b->n_msgs == 0) return TBG_E_INVALID_ARG;
    if (b->msg_off[0] != 0) return TBG_E_INVALID_ARG;
    for (uint32_t m = 0; m < b->n_msgs; ++m)
      if (b->msg_off[m + 1] < b->msg_off[m]) return TBG_E_INVALID_ARG;
    if (b->msg_off[b->n_msgs] && !b->msgs) return TBG_E_INVALID_ARG;
    for (uint32_t d = 0; d < b->n_duties; ++d)
      if (b->duty_msg[d] >= b->n_msgs) return TBG_E_INVALID_ARG;
  }
  return TBG_OK;
}

// Persistent host workers (one per context but the first, whose piece runs
// on the calling thread): run(n, fn) hands fn(i), i = 1 .. n - 1, to worker
// i - 1's FIFO and waits for all of them -- no thread is created per call
// (round 4 spawned and joined n - 1 std::threads on every submit and
// collect).  Calls from several caller threads interleave on each worker's
// queue.  A multi-context owns two pools, so a collect blocked on the device
// never delays a submit queued behind it.
class Pool {
 public:
  explicit Pool(uint32_t n) : q_(n) {
    for (uint32_t w = 0; w < n; ++w) th_.emplace_back([this, w] { loop(w); });
  }
  ~Pool() {
    for (auto& q : q_) {
      std::lock_guard<std::mutex> lk(q.mu);
      q.stop = true;
      q.cv.notify_one();
    }
    for (auto& t : th_) t.join();
  }
  template <class F>
  void run(uint32_t n, F fn) {
    struct Latch {
      std::mutex mu;
      std::condition_variable cv;
      uint32_t left;
    } latch;
    latch.left = n > 1 ? n - 1 : 0;
    for (uint32_t i = 1; i < n; ++i) {
      Queue& q = q_[(i - 1) % q_.size()];
      std::lock_guard<std::mutex> lk(q.mu);
      q.tasks.emplace_back([&fn, &latch, i] {
        fn(i);
        std::lock_guard<std::mutex> l2(latch.mu);
        if (--latch.left == 0) latch.cv.notify_one();
      });
      q.cv.notify_one();
    }
    if (n) fn(0);
    std::unique_lock<std::mutex> lk(latch.mu);
    latch.cv.wait(lk, [&] { return latch.left == 0; });
  }

 private:
  struct Queue {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> tasks;
    bool stop = false;
  };
  void loop(uint32_t w) {
    Queue& q = q_[w];
    for (;;) {
      std::function<void()> task;
      {
        std::unique_lock<std::mutex> lk(q.mu);
        q.cv.wait(lk, [&] { return q.stop || !q.tasks.empty(); });
        if (q.tasks.empty()) return;  // stopping, nothing left
        task = std::move(q.tasks.front());
        q.tasks.pop_front();
      }
      task();
    }
  }
  std::vector<Queue> q_;
  std::vector<std::thread> th_;
};

inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct tbg_multi {
  std::vector<tbg_ctx*> ctx;
  std::mutex mu;
  std::unordered_map<tbg_ticket, Job> jobs;
  tbg_ticket next_ticket = 1;
  Pool* submit_pool = nullptr;   // pieces' sub-batch builds and per-context submits
  Pool* collect_pool = nullptr;  // shards' waits and copy-outs
  // host-side work (tbg_multi_host_stats): [submit calls, partials, ns in
  // sub-batch builds (summed over workers), submit wall ns, collect calls,
  // collect wall ns]
  std::atomic<uint64_t> host[6] = {};
};

extern "C" {

int tbg_multi_init(const tbg_config* cfg, const int32_t* devices, uint32_t n_devices, tbg_multi** out) {
  if (!out || !devices || n_devices == 0 || n_devices > 64) return TBG_E_INVALID_ARG;
  *out = nullptr;
  tbg_multi* m = new (std::nothrow) tbg_multi();
  if (!m) return TBG_E_OOM;
  tbg_config c{};
  if (cfg) c = *cfg;
  // no express slot unless asked for: n contexts' streams add up per process
  // (TBG_MAX_SLOT_STREAMS)
  if (c.express_partials == 0) c.express_partials = TBG_EXPRESS_OFF;
  for (uint32_t i = 0; i < n_devices; ++i) {
    c.device = devices[i];
    tbg_ctx* x = nullptr;
    int rc = tbg_init(&c, &x);
    if (rc != TBG_OK) {
      tbg_multi_destroy(m);
      return rc;
    }
    m->ctx.push_back(x);
  }
  const uint32_t workers = n_devices > 1 ? n_devices - 1 : 1;
  m->submit_pool = new (std::nothrow) Pool(workers);
  m->collect_pool = new (std::nothrow) Pool(workers);
  if (!m->submit_pool || !m->collect_pool) {
    tbg_multi_destroy(m);
    return TBG_E_OOM;
  }
  *out = m;
  return TBG_OK;
}

void tbg_multi_destroy(tbg_multi* m) {
  if (!m) return;
  delete m->submit_pool;  // (joins the workers: no call may be in flight)
  delete m->collect_pool;
  for (auto* x : m->ctx) tbg_destroy(x);
  delete m;
}

uint32_t tbg_multi_size(const tbg_multi* m) { return m ? (uint32_t)m->ctx.size() : 0; }

tbg_ctx* tbg_multi_context(tbg_multi* m, uint32_t i) { return (m && i < m->ctx.size()) ? m->ctx[i] : nullptr; }

int tbg_multi_load_pubkeys(tbg_multi* m, const uint8_t* pk48, uint32_t count, uint32_t* first_id, int32_t* status) {
  if (!m || (count && !pk48)) return TBG_E_INVALID_ARG;
  const uint32_t n = (uint32_t)m->ctx.size();
  std::vector<int> rc(n, TBG_OK);
  std::vector<uint32_t> first(n, 0);
  // The same table decoded on every device (in parallel); the status of
  // context 0 is reported (every device computes the same one).
  m->submit_pool->run(n, [&](uint32_t i) {
    rc[i] = tbg_load_pubkeys(m->ctx[i], pk48, count, &first[i], i == 0 ? status : nullptr);
  });
  for (uint32_t i = 0; i < n; ++i)
    if (rc[i] != TBG_OK) return rc[i];
  for (uint32_t i = 1; i < n; ++i)
    if (first[i] != first[0]) return TBG_E_INVALID_ARG;  // a context was loaded outside the multi-context
  if (first_id) *first_id = first[0];
  return TBG_OK;
}

int tbg_multi_submit(tbg_multi* m, const tbg_batch* b, tbg_ticket* ticket) {
  return tbg_multi_submit_group(m, &b, 1, ticket);
}

int tbg_multi_submit_group(tbg_multi* m, const tbg_batch* const* bs, uint32_t n_batches, tbg_ticket* tickets) {
  if (!m || !bs || !tickets || n_batches == 0) return TBG_E_INVALID_ARG;
  const uint64_t t_call = now_ns();
  for (uint32_t k = 0; k < n_batches; ++k) {
    const int rc = validate_split(bs[k]);
    if (rc != TBG_OK) return rc;
    if (bs[k]->op != bs[0]->op) return TBG_E_INVALID_ARG;  // one kernel chain per device batch
  }
  const uint32_t n = (uint32_t)m->ctx.size();
  // The caller batches back to back form one sequence of duties; context i
  // takes the duties from the first one whose first partial is at or past
  // i * P / n (P = all partials; duties are never split, a duty with many
  // partials stays whole), so every context gets an equal share of the
  // partials however the callers' batches are sized.  With no partials at all
  // the duties are split evenly.  A context's range may span several caller
  // batches: their pieces go to it as ONE tbg_submit_group (one device batch,
  // one launch per kernel), the way a single context packs callers' batches.
  std::vector<uint64_t> d_base(n_batches + 1, 0), p_base(n_batches + 1, 0);
  for (uint32_t k = 0; k < n_batches; ++k) {
    d_base[k + 1] = d_base[k] + bs[k]->n_duties;
    p_base[k + 1] = p_base[k] + bs[k]->n_partials;
  }
  const uint64_t ND = d_base[n_batches], NP = p_base[n_batches];
  if (ND > 0x7FFFFFFFull * n || NP > 0x7FFFFFFFull * n) return TBG_E_INVALID_ARG;
  // global duty index of the first duty whose global first partial >= target
  // (the first duty of batch k starts at p_base[k], its last at most at
  // p_base[k + 1]: the search starts at the first batch that can hold one)
  auto duty_at_partial = [&](uint64_t target) -> uint64_t {
    uint32_t k = (uint32_t)(std::lower_bound(p_base.begin() + 1, p_base.end(), target) - (p_base.begin() + 1));
    while (k < n_batches) {
      const tbg_batch* b = bs[k];
      const uint64_t local = target > p_base[k] ? target - p_base[k] : 0;
      const uint32_t d = (uint32_t)(std::lower_bound(b->duty_first, b->duty_first + b->n_duties + 1, local) -
                                    b->duty_first);
      if (d < b->n_duties) return d_base[k] + d;
      ++k;  // past this batch's last duty: the next batch's first
    }
    return ND;
  };
  std::vector<uint64_t> cut(n + 1, 0);
  cut[n] = ND;
  for (uint32_t i = 1; i < n; ++i) {
    const uint64_t c = NP ? duty_at_partial(NP * i / n) : ND * i / n;
    cut[i] = std::max(cut[i - 1], std::min(c, ND));
  }
  // Pieces per context: (caller batch, its duty range).
  struct Piece { uint32_t k, d0, d1; };
  std::vector<std::vector<Piece>> pieces(n);
  for (uint32_t i = 0; i < n; ++i)
    for (uint32_t k = 0; k < n_batches; ++k) {
      const uint64_t lo = std::max(cut[i], d_base[k]), hi = std::min(cut[i + 1], d_base[k + 1]);
      if (hi > lo) pieces[i].push_back({k, (uint32_t)(lo - d_base[k]), (uint32_t)(hi - d_base[k])});
    }
  std::vector<uint32_t> use;
  for (uint32_t i = 0; i < n; ++i)
    if (!pieces[i].empty()) use.push_back(i);
  std::vector<int> src(use.size(), TBG_OK);
  std::vector<std::vector<tbg_ticket>> part_tickets(use.size());
  m->submit_pool->run((uint32_t)use.size(), [&](uint32_t u) {
    const uint32_t i = use[u];
    const uint64_t t0 = now_ns();
    std::vector<SubBatch> sb(pieces[i].size());
    std::vector<const tbg_batch*> ptr(pieces[i].size());
    for (size_t j = 0; j < sb.size(); ++j) {
      sb[j].build(*bs[pieces[i][j].k], pieces[i][j].d0, pieces[i][j].d1);
      ptr[j] = &sb[j].b;
    }
    m->host[2] += now_ns() - t0;
    part_tickets[u].resize(sb.size());
    src[u] = tbg_submit_group(m->ctx[i], ptr.data(), (uint32_t)ptr.size(), part_tickets[u].data());  // copies
  });
  for (size_t u = 0; u < src.size(); ++u) {
    if (src[u] == TBG_OK) continue;
    // undo: drain the contexts that did start, then report the first error
    for (size_t v = 0; v < src.size(); ++v)
      if (src[v] == TBG_OK)
        for (tbg_ticket t : part_tickets[v]) tbg_collect(m->ctx[use[v]], t, nullptr, nullptr, nullptr, 1);
    return src[u];
  }
  std::vector<Job> jobs(n_batches);
  for (uint32_t k = 0; k < n_batches; ++k) {
    Job& job = jobs[k];
    job.duty_lo.resize(n + 1);
    for (uint32_t i = 0; i <= n; ++i)
      job.duty_lo[i] = (uint32_t)(std::min(std::max(cut[i], d_base[k]), d_base[k + 1]) - d_base[k]);
  }
  for (size_t u = 0; u < use.size(); ++u) {
    const uint32_t i = use[u];
    for (size_t j = 0; j < pieces[i].size(); ++j) {
      const Piece& pc = pieces[i][j];
      Shard s;
      s.ctx = i;
      s.ticket = part_tickets[u][j];
      s.d0 = pc.d0;
      s.d1 = pc.d1;
      s.p0 = bs[pc.k]->duty_first[pc.d0];
      s.p1 = bs[pc.k]->duty_first[pc.d1];
      jobs[pc.k].shards.push_back(s);
    }
  }
  std::lock_guard<std::mutex> lk(m->mu);
  for (uint32_t k = 0; k < n_batches; ++k) {
    tickets[k] = m->next_ticket++;
    m->jobs.emplace(tickets[k], std::move(jobs[k]));
  }
  m->host[0] += 1;
  m->host[1] += NP;
  m->host[3] += now_ns() - t_call;
  return TBG_OK;
}

int tbg_multi_collect(tbg_multi* m, tbg_ticket t, int32_t* pst, int32_t* dst, uint8_t* agg, int block) {
  if (!m) return TBG_E_INVALID_ARG;
  Job* job = nullptr;
  {
    std::lock_guard<std::mutex> lk(m->mu);
    auto it = m->jobs.find(t);
    if (it == m->jobs.end() || it->second.collecting) return TBG_E_TICKET;
    job = &it->second;
    if (!block) {
      for (const Shard& s : job->shards) {
        int q = tbg_poll(m->ctx[s.ctx], s.ticket);
        if (q == TBG_E_PENDING) return TBG_E_PENDING;
      }
    }
    job->collecting = true;  // the map node stays put: unordered_map references are stable
  }
  // Every shard's wait and copy-out runs on its own thread, straight into the
  // caller's arrays at the shard's offsets (caller order by construction).
  const uint64_t t_call = now_ns();
  std::vector<int> rc(job->shards.size(), TBG_OK);
  m->collect_pool->run((uint32_t)job->shards.size(), [&](uint32_t k) {
    const Shard& s = job->shards[k];
    rc[k] = tbg_collect(m->ctx[s.ctx], s.ticket, pst ? pst + s.p0 : nullptr, dst ? dst + s.d0 : nullptr,
                        agg ? agg + 96ull * s.d0 : nullptr, 1);
  });
  {
    std::lock_guard<std::mutex> lk(m->mu);
    m->jobs.erase(t);
  }
  m->host[4] += 1;
  m->host[5] += now_ns() - t_call;
  for (int r : rc)
    if (r != TBG_OK) return r;
  return TBG_OK;
}

int tbg_multi_host_stats(tbg_multi* m, uint64_t* out16, int reset) {
  if (!m || !out16) return TBG_E_INVALID_ARG;
  for (int k = 0; k < 6; ++k) out16[k] = reset ? m->host[k].exchange(0) : m->host[k].load();
  uint64_t sum[8] = {};
  for (auto* x : m->ctx) {
    uint64_t v[8];
    const int rc = tbg_host_stats(x, v, reset);
    if (rc != TBG_OK) return rc;
    for (int k = 0; k < 8; ++k) sum[k] += v[k];
  }
  for (int k = 0; k < 8; ++k) out16[6 + k] = sum[k];
  out16[14] = m->ctx.size();
  out16[15] = 0;
  return TBG_OK;
}

int tbg_multi_layout(tbg_multi* m, tbg_ticket t, uint32_t* duty_lo) {
  if (!m || !duty_lo) return TBG_E_INVALID_ARG;
  std::lock_guard<std::mutex> lk(m->mu);
  auto it = m->jobs.find(t);
  if (it == m->jobs.end()) return TBG_E_TICKET;
  std::copy(it->second.duty_lo.begin(), it->second.duty_lo.end(), duty_lo);
  return TBG_OK;
}

}  // extern "C"
