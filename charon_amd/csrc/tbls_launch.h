// Host-side view of the engine's kernels: the device batch layout and one
// launcher per kernel (each defined next to its kernel in a k_*.hip
// translation unit, so the units compile in parallel and no relocatable
// device code is needed).
#pragma once
#include <hip/hip_runtime.h>
#include "bls_curve.h"
#include "bls_lines.h"
#include "../../include/tbls_gpu.h"

namespace tbg {

constexpr int kBlock = 64;
// Default list positions per pass of the fallback levels' shared line buffer
// (22.8 KB each: 0.75 GB per slot; tbg_config.fb_window overrides it).
// Level-0 launch shape: a launch whose Miller hexads at (G, C) = (16, 4)
// need more than one round of the device's wave slots picks (G, C) among
// (16, 4), (16, 8), (14, 7) by rounds x hexad length (tbls_engine.hip,
// l0_shape); 0: always (16, 4).
// Per-key G1 tables for the RLC products [r_i] pk_i: 1 = the 8-entry window
// table (bls_rlc.h rlc_mul_key_w2: 14 doublings + 16 additions), 0 = the
// 2-entry pair table pk +- [x]pk (15 + 32)
#ifndef TBG_PK_W2
#define TBG_PK_W2 1
#endif
constexpr uint32_t PK_TAB = TBG_PK_W2 ? 8u : 2u;  // G1A entries per key in the resident table
// tbg_replay_plan: the launches a plan runs together take the level-0 shape
// of their duties together (1), or keep their submitted shapes (0)
#ifndef TBG_REPLAY_SHAPE
#define TBG_REPLAY_SHAPE 1
#endif
#ifndef TBG_L0_SHAPE
#define TBG_L0_SHAPE 1
#endif
// 1 (round 6): one-chunk groups of 5 .. 10 duties are level-0 shape
// candidates too; 0: (16, 4), (16, 8), (14, 7) only
#ifndef TBG_L0_SHAPE_WIDE
#define TBG_L0_SHAPE_WIDE 1
#endif
#ifndef TBG_FB_WINDOW
#define TBG_FB_WINDOW 32768u
#endif
// 1 (round 6): the duty / partial list passes beyond the expected list
// length launch small grids that loop (DevBatch::fb_full); 0: every pass full
#ifndef TBG_FB_EXPECT
#define TBG_FB_EXPECT 1
#endif

// Minimum waves per SIMD requested from the register allocator (1 lets a
// kernel use all 512 / 2 = 256 VGPRs at two waves per SIMD; 3 caps it at
// 168).  A tuning knob: tools/ab_variants.py builds -DTBG_MIN_WAVES=N.
#ifndef TBG_MIN_WAVES
#define TBG_MIN_WAVES 1
#endif
#define TBG_LAUNCH __launch_bounds__(64, TBG_MIN_WAVES)
// Kernels split by phase ask for the occupancy their footprint allows: at
// least two waves per SIMD (<= 256 VGPRs), because a lone wave issues the
// multiply-adds at ~58 % of the two-wave rate (profiles/r02/valu_rates.txt).
#ifndef TBG_PAIR_WAVES
#define TBG_PAIR_WAVES 2    // lane-pair G2 kernels (bls_pair.h)
#endif
#ifndef TBG_DECODE_WAVES
#define TBG_DECODE_WAVES 2  // k_decode_sigs (square roots only)
#endif
#define TBG_LAUNCH_N(w) __launch_bounds__(64, w)
// Latency-critical kernels of a launch's serial tail (the level-0 bucket
// reduction, S's lines, the product tree, the one final exponentiation) run
// a few waves each, often on SIMDs that also host other launches' long
// Miller / decode waves, which halve their issue rate (k_l0_final 3.4 ms
// alone, 6.8 ms beside a Miller kernel, profiles/r04/base/timeline_s20.txt).
// s_setprio 3 makes their waves win the SIMD's instruction arbitration;
// the throughput kernels lose nothing but the slots these few waves use.
#if defined(__HIP_DEVICE_COMPILE__)
#define TBG_URGENT() __builtin_amdgcn_s_setprio(3)
#else
#define TBG_URGENT() ((void)0)
#endif
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
  G2J* h_jac;          // [3 n_msgs] H(m) before affine conversion (k_hash_map / _clear / _affine), then
                       // the cofactor clearing's temporaries [x]P and [x]P + psi(P) (k_hash_clear.hip)
  uint32_t* lam;       // [n_partials][8] scalar words
  uint32_t* sig_lines;  // [fb window][LINES_WORDS] Miller lines of listed signatures (-g1 folded in)
  uint32_t* h_lines;    // [n_msgs][LINES_WORDS] Miller lines of each H(m) (G1 factor left out)
  // random-linear-combination verification (k_rlc.hip)
  uint32_t rlc_seed[8];   // secret per-batch key of the scalars r_i
  uint32_t rlc_group;     // duties per level-1 group; 0 = per-partial checks only
  G1J* part_p;            // [n_partials] r_i pk_i
  G2J* part_s;            // [n_partials] r_i sig_i
  uint32_t rlc_chunk;     // duties per level-1 Miller chunk (quads per group = ceil(G / chunk))
  uint32_t* chunk_f;      // [n_groups * (chunks + 1)][3][4 NL] Miller products of the chunks (quad layout);
                          // chunk index `chunks` of a group is its S pair alone
  uint32_t* chunk_list;   // [n_groups * chunks] level-1.5 chunks of failed groups (group * chunks + c)
  uint32_t* chunk_lines;  // [fb window][LINES_WORDS] lines of S_c, by chunk-list position - fb_base
  G1A* dv_p;              // [n_duties] sum r_i pk_i (affine), stored as (-x, y)
  G2J* dv_s;              // [n_duties] sum r_i sig_i
  int32_t* dv_state;      // [n_duties] RLC_*
  int32_t* grp_state;     // [n_groups] GRP_*
  uint32_t* grp_lines;    // [n_groups][LINES_WORDS] lines of the group's S (-g1 folded in)
  uint32_t* counters;     // [CNT_*] work-list lengths
  uint32_t* part_list;    // [n_partials] level-3 partials (sig_lines by list position)
  G2A* pend_pts;          // [max(n_groups, n_groups * chunks, n_duties)] affine points whose folded Miller
                          // lines k_lines_fold computes next (group S, then the fallback lists' sums)
  uint32_t* chunk_fe;     // [n_groups * chunks][3][4 NL] final-exponentiated value of failed chunks (by list position)
  uint32_t* cid_list;     // [n_groups * chunks] level-1.5b entries: chunk-list positions
  G1A* cid_p;             // [n_groups * chunks][rlc_chunk] w_d P_d as (-x, y), by level-1.5b position
  uint32_t* cid_lines;    // [fb window][LINES_WORDS] lines of sum w_d S_d, by level-1.5b position - fb_base
  // level 1g: the exponent test over a failed GROUP's partials, right after
  // level 1 (most failed groups hold exactly one bad partial)
  uint32_t gident;        // 1: failed groups go to level 1g first, its unresolved ones to level 3
                          // (2: to level 1.5; 0: no level 1g)
  uint32_t* grp_fe;       // [n_groups][3][4 NL] final-exponentiated value A_g of a level-1g group (by list position)
  uint32_t* gid_list;     // [n_groups] level-1g entries: group index (| ID_DEGENERATE)
  G1A* gid_p;             // [n_groups][rlc_group] sum_(i in d) w_i r_i pk_i as (-x, y): level-1g position, duty in group
  uint32_t* gid_lines;    // lines of sum w_i r_i sig_i by level-1g position - fb_base (the fallback line buffer)
  uint32_t* gid_f;        // [n_groups][chunks + 1][3][4 NL] Miller products of a level-1g entry (chunks, then S')
  uint32_t* id_fe;        // [n_duties][3][4 NL] value A_d of each level-2b duty (by list position)
  uint32_t* id_list;      // [n_duties] level-2b entries: failed duties with several candidates
  G1A* id_p;              // [n_duties] sum w_i r_i pk_i (affine), by level-2b position
  // The fallback levels' line buffers (chunk_lines, cid_lines, id_lines,
  // sig_lines) are ONE buffer of fb_window entries (0: unbounded), used in
  // stream order: each level's lines are written and consumed in passes of
  // fb_window list positions [fb_base, fb_base + fb_window) before the next
  // level writes (launch_rlc_check) -- a slot's HBM no longer scales with the
  // worst-case list length (22.8 KB per partial of every batch).
  uint32_t fb_window, fb_base;
  // Passes of the duty (level 2b) and partial (level 3) lists start full grids
  // only below fb_full list positions (the list lengths the collected batches'
  // invalid share makes likely); later passes launch a few waves that loop
  // over the pass (k_verify_list, k_lines_sig_list, k_rlc_ident_check,
  // k_lines_fold), so a clean batch does not dispatch ~80k empty waves of 20
  // partial passes per 16-batch launch (round 6).  UINT32_MAX: every pass full.
  uint32_t fb_full;
  uint32_t* id_lines;     // lines of sum w_i r_i sig_i by level-2b position: aliases sig_lines,
                          // which level 3 only fills after level 2b has consumed them
  // level 0 (k_msm.hip, k_rlc.hip): the whole device batch as ONE RLC check,
  //   prod_d e(P_d, H(m_d)) * e(-g1, S) == 1,  S = sum_i r_i s_i,
  // S as a bucket MSM over the signatures and their psi images (no per-partial
  // G2 scalar multiplication); a failure falls through to the group levels
  uint32_t rlc_batch;     // 1: level 0 runs first (every candidate's r_i random, no group lead)
  uint64_t* msm_r;        // [n_partials] r_i of the candidates
  uint32_t* msm_off;      // [MSM_BUCKETS + 1] bucket sizes, then their offsets
  uint32_t* msm_cur;      // [MSM_BUCKETS] scatter cursors
  uint32_t* msm_ent;      // [4 n_partials] bucket entries: partial << 3 | k << 1 | negative
  G2J* msm_part;          // [MSM_BUCKETS * MSM_SPLIT] sums of the bucket slices
  G2J* msm_bkt;           // [MSM_BUCKETS] (2j + 1) * (bucket j's sum)
  G2J* msm_sum;           // [MSM_SUM_ENTRIES] tree sums of msm_bkt
  G2A* batch_pt;          // [1] S in affine form
  uint32_t* batch_lines;  // [LINES_WORDS] Miller lines of S (-g1 folded in)
  uint32_t* batch_f;      // [3][4 NL] Miller product of the S pair (quad layout)
  uint32_t* grp_f;        // [GRP_F_ENTRIES(n_groups)][3][4 NL] each group's P-chunk product, then the product tree
  // level 1's group sums S_g = sum_i r_i s_i as one bucket MSM per group
  // (k_gmsm.hip): 4-bit windows of the four psi digits,
  // no per-partial G2 scalar multiplication; the per-partial products r_i s_i
  // are formed afterwards for the failed groups' candidates only
  uint32_t* gm_off;       // [n_groups][GM_BUCKETS + 1] bucket offsets into the group's entries
  uint32_t* gm_ent;       // [16 n_partials] entries (partial << 3 | k << 1 | negative); group g's
                          // start at 16 * (its first partial)
  G2J* gm_part;           // [n_groups][GM_BUCKETS] bucket sums, then the window sums T_w at w * GM_V
  uint32_t* gm_lead;      // [n_groups] the group's r = 1 partial (UINT32_MAX: none / level 0's scalars)
  uint32_t* gm_list;      // [n_partials] candidates of failed groups, whose r_i s_i are formed afterwards
  uint32_t* gm_hist;      // [256] bucket-size histogram, then the size-order cursors
  uint32_t* gm_order;     // [n_groups * GM_BUCKETS] buckets by decreasing size (k_gm_bucket's order)
  // batched subgroup test of the decoded signatures (k_sgb.hip): per group
  // of SGB_M consecutive partials, SGB_K random combinations sum c_i s_i with
  // c_i uniform mod 13 are tested psi(Q) == [x] Q; only the members of a
  // failed group take the per-signature test (k_subgroup_sigs)
  uint32_t sgb;           // 1: the batched test runs (0: every signature is tested alone)
  uint32_t sgb_m;         // consecutive partials per group (a power of two, SGB_M_MIN..SGB_M)
  uint32_t sgb_split;     // slices per bucket (k_sgb_bucket / k_sgb_fold)
  uint32_t sgb_seed[8];   // secret per-batch key of the combinations' digits: always fresh OS
                          // entropy, even under a fixed rlc_seed (a predictable key would let a
                          // submitter craft torsion components that cancel across combinations)
  uint32_t* sgb_off;      // [n_sg][SGB_BUCKETS + 1] bucket offsets into the group's entries
  uint32_t* sgb_ent;      // [n_sg][sgb_m * SGB_K] entries: member << 1 | negative
  G2J* sgb_part;          // [n_sg][SGB_BUCKETS][sgb_split] bucket slice sums
  uint32_t* sgb_bad;      // [n_sg] 1: some combination is outside G2 (members tested alone)
  // recombination (k_aggregate.hip)
  G2J* agg_acc;           // [n_duties] integer-coefficient sums awaiting [1/D] (listed duties only)
  uint32_t* agg_list;     // [n_duties] duties whose Lagrange denominator D > 1
  // outputs
  int32_t* partial_status;
  int32_t* duty_status;
  uint8_t* agg;        // [n_duties][96]
};

enum RlcState : int32_t { RLC_NONE = 0, RLC_COMBINED = 1, RLC_EACH = 2 };
enum GroupState : int32_t { GRP_EMPTY = 0, GRP_LINES = 1, GRP_OK = 2, GRP_FAIL = 3, GRP_GID = 4 };  // GRP_GID: at level 1g
// CNT_DUTIES: level-2b duties (id_list), CNT_PARTIALS: level-3 partials, CNT_AGG: [1/D] duties,
// CNT_CHUNKS: level-1.5 chunks, CNT_CID: level-1.5b chunks, CNT_L0_BAD: level 0 cannot
// hold (a degenerate sum, a duty checked per partial, an unusable H(m)), CNT_L0_OK: level 0 passed
enum Counter : int { CNT_DUTIES = 0, CNT_PARTIALS = 1, CNT_AGG = 2, CNT_CHUNKS = 3, CNT_CID = 4, CNT_L0_BAD = 5,
                     CNT_L0_OK = 6, CNT_GID = 7, CNT_LAZY = 8, CNT_WORDS = 9 };  // CNT_GID: level-1g groups,
                                                                                // CNT_LAZY: gm_list entries

// Level-0 MSM: a digit a (odd, |a| < 2^16) of r_i puts psi^k(s_i) into bucket
// (|a| - 1) / 2; the tree sums (k_msm_tree) leave one point per workgroup in
// msm_sum.
constexpr uint32_t MSM_BUCKETS = 32768;
constexpr uint32_t MSM_SPLIT = 4;  // slices per bucket (k_msm_bucket_part)
constexpr uint32_t MSM_SUM_ENTRIES = 128;
// Batched subgroup test (k_sgb.hip).  A point of E2(Fp2) outside G2 has a
// component of order divisible by a prime factor of the G2 cofactor, the
// smallest of which is 13: with c_i uniform mod 13 (signed digits -6..6) a
// combination hides such a component with probability <= 1/13, so SGB_K =
// 18 independent combinations leave 13^-18 < 2^-66.
#ifndef TBG_SGB_M
#define TBG_SGB_M 1024
#endif
#ifndef TBG_SGB_SPLIT
#define TBG_SGB_SPLIT 4
#endif
// The group size follows the non-subgroup share of the collected batches
// (sgb_plan, tbls_engine.hip): SGB_M while clean, down to SGB_M_MIN when a
// few signatures per thousand are outside G2 (a failed group costs its
// members' per-signature tests).
constexpr uint32_t SGB_M = TBG_SGB_M;  // largest group: consecutive partials (LDS of k_sgb_sort)
constexpr uint32_t SGB_M_MIN = 64;
constexpr uint32_t SGB_K = 18;         // combinations per group
constexpr uint32_t SGB_V = 6;          // buckets per combination (|c| = 1..6)
constexpr uint32_t SGB_BUCKETS = SGB_K * SGB_V;
constexpr uint32_t SGB_SPLIT = TBG_SGB_SPLIT;  // slices per bucket at SGB_M (~40 additions each)
constexpr uint32_t SGB_MIN_PARTIALS = 2 * SGB_M;  // smaller batches test each signature alone
TBG_HD uint32_t sgb_groups(uint32_t n_partials, uint32_t m) { return (n_partials + m - 1) / m; }
// slices per bucket for groups of m: ~40 entries per slice, at least one
TBG_HD uint32_t sgb_split_for(uint32_t m) {
  const uint32_t s = SGB_SPLIT * m / SGB_M;
  return s ? s : 1u;
}
// Level-0 product tree over the groups' P-chunk products.  Each pass is a
// chain of F - 1 Fp12 products on one lane group (~24 us each at one wave per
// SIMD), so the tree's latency ~ log_F(n) * F is smallest near F = 4 (16: 1.3
// ms for 10k groups; 4: ~0.7 ms) -- it sits on every launch's critical path.
constexpr uint32_t L0_TREE_FAN = 4;
// (sum over the passes of ceil(n / F^k) <= n / (F - 1) + one per pass)
TBG_HD uint32_t grp_f_entries(uint32_t n_groups) { return n_groups + n_groups / (L0_TREE_FAN - 1) + 40; }
// k_miller_hex modes
enum MillerMode : int { MILLER_GROUPS = 0, MILLER_L0 = 1, MILLER_GROUP_S = 2 };
// k_rlc_duty_sum phases
//   DSUM_P: P_d only (level 1's S comes from the group MSM, k_gmsm.hip);
//   DSUM_FALLBACK_S: S_d of the failed groups' duties, from the r_i s_i formed
//   for them after the group checks
enum DutySumPhase : int { DSUM_BOTH = 0, DSUM_L0_P = 1, DSUM_FALLBACK_S = 2, DSUM_P = 3 };
// Level 1's group MSM (k_gmsm.hip): each 16-bit digit a_k of r_i (bls_rlc.h)
// read as four 4-bit windows of signed binary digits, v = 2 nibble - 15 (odd,
// |v| <= 15): 16 entries per partial into GM_BUCKETS = 4 windows x 8 buckets
// (|v| = 2b + 1) per group.
#ifndef TBG_GMSM
#define TBG_GMSM 1  // 0: the per-partial products r_i s_i for every candidate (k_rlc_partial2, before round 6)
#endif
constexpr uint32_t GM_W = 4, GM_V = 8, GM_BUCKETS = GM_W * GM_V;

// Flags in the fallback lists (k_rlc.hip): the entry's sum is the point at
// infinity -- no lines, its members go to an exact level.
constexpr uint32_t CHUNK_DEGENERATE = 0x80000000u;
constexpr uint32_t ID_DEGENERATE = 0x80000000u;
// k_lines_fold<KIND>: which pending points get lines, and where they go.
enum FoldKind : int { FOLD_GROUPS = 0, FOLD_CHUNKS = 1, FOLD_CID = 2, FOLD_IDENT = 3, FOLD_GID = 5 };

// Fallback list position k in the current pass, and its slot in the line buffer.
TBG_HD bool fb_in_pass(const DevBatch& B, uint32_t k) { return B.fb_window == 0 || k - B.fb_base < B.fb_window; }
TBG_HD size_t fb_slot(const DevBatch& B, uint32_t k) { return (size_t)LINES_WORDS * (k - B.fb_base); }
// The list positions of the current pass, from `first` in steps of `stride`
// (a grid smaller than the pass loops): stops at the list's end or the pass's.
template <class F>
TBG_HD void fb_pass_loop(const DevBatch& B, uint32_t first, uint32_t stride, uint32_t count, F&& body) {
  const uint32_t w = B.fb_window ? B.fb_window : 0xFFFFFFFFu;
  for (uint32_t s = first; s < w; s += stride) {
    const uint32_t k = B.fb_base + s;
    if (k >= count) break;
    body(k);
  }
}

// 1: every VERIFY_AGGREGATE chain aggregates speculatively and redoes only
// the duties with an invalid partial; 0 (default): speculate only while level
// 0 runs, aggregate every duty again after a failed level 0.  Measured at 1 %
// invalid (level 0 off) and on config 5 (round 5, profiles/r05/inv1/): 1.48 /
// 1.47 M vs 1.49 / 1.50 M and 1.17 / 1.19 M vs 1.24 / 1.24 M -- the
// speculative pass's throughput cost outweighs the shorter redo at the tail.
#ifndef TBG_SPEC_ALWAYS
#define TBG_SPEC_ALWAYS 0
#endif
#ifndef TBG_ALT_ORDER
#define TBG_ALT_ORDER 0
#endif
#ifndef TBG_L0_JOIN
#define TBG_L0_JOIN 0
#endif
// Participation of a partial in its duty's aggregate.  SPEC: the
// speculative aggregation that runs BEFORE verification while level 0 is on
// (launch_chain): every candidate counts as valid, which is what a level-0
// pass concludes; after a failed level 0 the aggregation runs again.
template <bool SPEC = false>
TBG_HD bool participates(uint32_t op, int32_t st) {
  return op == TBG_OP_VERIFY_AGGREGATE ? (st == TBG_PS_VALID || (SPEC && st == TBG_PS_NOT_VERIFIED))
                                       : (st == TBG_PS_NOT_VERIFIED);
}

// Debug aid: with TBG_DEBUG_SYNC=1 in the environment every launch is
// followed by a stream synchronisation and a line on stderr (kernel, ms,
// status), so a faulting or runaway kernel names itself.  Off by default.
void debug_after_launch(const char* kernel, hipStream_t st);
// Per-kernel timing (tbg_replay_profile): while a recorder is active on the
// launching thread every launch is bracketed by a HIP event pair on its own
// stream; otherwise these are a thread-local pointer test.
void kprof_pre(const char* kernel, hipStream_t st);
void kprof_post(hipStream_t st);
#define TBG_KLAUNCH(kernel, grid, block, st, ...)                      \
  do {                                                                \
    kprof_pre(#kernel, st);                                           \
    hipLaunchKernelGGL(kernel, grid, block, 0, st, __VA_ARGS__);      \
    kprof_post(st);                                                   \
    debug_after_launch(#kernel, st);                                  \
  } while (0)

// launchers (asynchronous on `st`)
// Device arrays of one plain-sum call (k_sum.hip): n_sets sets of items,
// summed in chunks of sum_chunk_size() items.
struct SumPlan {
  uint32_t n_sets, n_chunks;
  const uint32_t* off;          // [n_sets + 1] item offsets of the sets
  const uint32_t* chunk_first;  // [n_sets + 1] first chunk of each set
  const uint32_t* chunk_set;    // [n_chunks] set of each chunk
  void* part;                   // [n_chunks] G1J / G2J chunk sums
  int32_t* set_bad;             // [n_sets] zeroed before the launch
};
uint32_t sum_chunk_size();
void launch_sum_g1(const G1A* table, const int32_t* pk_status, uint32_t n_pk, const uint32_t* ids, const SumPlan& p,
                   uint8_t* out48, int32_t* status, hipStream_t st);
void launch_sum_g2(const uint8_t* sigs96, const SumPlan& p, uint8_t* out96, int32_t* status, int32_t* sig_status,
                   hipStream_t st);
void launch_decode_pubkeys(const uint8_t* pk48, uint32_t n, G1A* out, G1A* out_x, int32_t* status, hipStream_t st);
void launch_decode_sigs(const DevBatch& B, hipStream_t st);
// the batched subgroup test (B.sgb): sort, bucket sums, combination checks
void launch_subgroup_batch(const DevBatch& B, hipStream_t st);
void launch_hash_msgs(const DevBatch& B, hipStream_t st);
void launch_hash_clear(const DevBatch& B, hipStream_t st);
void launch_h_lines(const DevBatch& B, hipStream_t st);
// after_keys (optional) is enqueued once the candidates are final (the
// ERR_PUBKEY marks made), before the level-0 bucket MSM: the chain's
// speculative aggregation goes there, off the Miller kernel's critical path
void launch_rlc_prepare(const DevBatch& B, const G1A* pk_aff, const G1A* xpk_aff, const G1A* pk_tab,
                        const int32_t* pk_status, uint32_t n_pk, hipStream_t st,
                        void (*after_keys)(const DevBatch&, hipStream_t) = nullptr);
void launch_rlc_check(const DevBatch& B, const G1A* pk_aff, const G1A* xpk_aff, const int32_t* pk_status, uint32_t n_pk,
                      hipStream_t st);
void launch_lines_fold(const DevBatch& B, int kind, uint32_t max_entries, hipStream_t st);
// level 0 (k_msm.hip)
void launch_pubkey_tables(const G1A* pk, const G1A* xpk, const int32_t* status, uint32_t n, G1A* tab, hipStream_t st);
void launch_l0_keys(const DevBatch& B, const G1A* pk_tab, const int32_t* pk_status, uint32_t n_pk, hipStream_t st);
void launch_l0_msm(const DevBatch& B, hipStream_t st);
void launch_l0_check(const DevBatch& B, hipStream_t st);
// level 0's P-chunk and S Miller products on hexads (k_miller_hex.hip)
void launch_l0_miller_hex(const DevBatch& B, hipStream_t st);
// level 1's P-chunk and group-S Miller products on hexads (k_miller_hex.hip)
void launch_groups_miller_hex(const DevBatch& B, hipStream_t st);
// after a level-0 failure: the groups' S Miller products only (k_miller_hex.hip)
void launch_group_s_miller_hex(const DevBatch& B, hipStream_t st);
// pk_tab: the keys' pair tables (k_pubkey_tables); unused after a level-0 failure (level 0 formed the G1 products)
void launch_rlc_partials(const DevBatch& B, const G1A* pk_tab, const G1A* pk_aff, const int32_t* pk_status,
                         uint32_t n_pk, hipStream_t st);
// level 1 by group MSMs (k_gmsm.hip): the G1 products and key marks (no
// level 0), the groups' S in affine form in pend_pts (grp_state set as
// k_rlc_group_lines does), and after the group checks the failed groups'
// r_i s_i (k_pair.hip, list mode) and S_d
void launch_rlc_g1(const DevBatch& B, const G1A* pk_tab, const G1A* pk_aff, const int32_t* pk_status, uint32_t n_pk,
                   hipStream_t st);
void launch_gm_group_s(const DevBatch& B, hipStream_t st);
void launch_gm_failed_partials(const DevBatch& B, const G1A* pk_aff, hipStream_t st);
void launch_rlc_partials_list(const DevBatch& B, const G1A* pk_aff, hipStream_t st);
// spec: the speculative pass (level 0 on, before verification; skipped when
// level 0 already cannot pass); the regular pass then returns at once if
// level 0 passed (TBG_SPEC_ALWAYS: see above)
void launch_lagrange(const DevBatch& B, hipStream_t st, bool spec = false);
void launch_aggregate(const DevBatch& B, hipStream_t st, bool spec = false);
void launch_aggregate_finish(const DevBatch& B, hipStream_t st, bool spec = false);
void launch_sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* pk48, hipStream_t st);
void launch_sign(const uint8_t* sk32, const uint32_t* item_msg, uint32_t n, const G2A* h_aff, const int32_t* h_status,
                 uint8_t* sig96, hipStream_t st);

}  // namespace tbg
