/*
 * tbls_gpu.h -- C ABI of the MI355X threshold-BLS engine (libtbls_gpu.so).
 *
 * Drop-in boundary for Charon's threshold-BLS hot path (singhhp1069/charon):
 *   tbls.Verify              reference tbls/tss.go:190-197
 *   tbls.Aggregate           reference tbls/tss.go:142-149
 *   tbls.VerifyAndAggregate  reference tbls/tss.go:153-187
 *   tblsconv.SigFromCore     reference tbls/tblsconv/tblsconv.go:125-132 (G2 decode, done on the GPU)
 *   tblsconv.SigToCore       reference tbls/tblsconv/tblsconv.go:119-122     (G2 encode, done on the GPU)
 *   tblsconv.KeyFromBytes    reference tbls/tblsconv/tblsconv.go:30-37       (G1 decode, tbg_load_pubkeys)
 * plus the batch entry points the new batch-aware call sites use
 * (core/parsigex/parsigex.go:101-107, core/validatorapi/validatorapi.go:228-287,
 *  core/parsigdb/memory.go:96-134 -> core/sigagg/sigagg.go:53-103).
 *
 * Plain C: pointers and sizes only.  All input buffers are caller-owned and
 * copied into pinned staging inside tbg_submit, so nothing is retained after
 * the call returns (cgo pointer rules).  Output buffers are caller-owned and
 * filled by tbg_collect.  One context drives one GPU; contexts are
 * thread-safe (an internal mutex serialises submit/collect).
 */
#ifndef TBLS_GPU_H
#define TBLS_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- call-level return codes ------------------------------------------ */
#define TBG_OK 0
#define TBG_E_INVALID_ARG (-1)  /* malformed batch (bad offsets, ids, sizes)   */
#define TBG_E_DEVICE (-2)       /* HIP runtime / kernel failure                */
#define TBG_E_OOM (-3)          /* device or pinned allocation failed          */
#define TBG_E_NO_DEVICE (-4)    /* no usable gfx950 device                     */
#define TBG_E_BUSY (-5)         /* every in-flight slot is taken               */
#define TBG_E_PENDING (-6)      /* tbg_collect(block=0): not finished yet      */
#define TBG_E_TICKET (-7)       /* unknown or already collected ticket         */

/* ---- per-partial-signature status (int32) ------------------------------ */
#define TBG_PS_INVALID 0         /* valid encodings, pairing check false: Go (false, nil) */
#define TBG_PS_VALID 1           /* pairing check true                                     */
#define TBG_PS_NOT_VERIFIED 2    /* decoded fine, op did not verify (TBG_OP_AGGREGATE)     */
#define TBG_PS_ERR_FLAGS (-1)    /* compression flag missing / bad infinity encoding       */
#define TBG_PS_ERR_FIELD (-2)    /* x coordinate >= p                                      */
#define TBG_PS_ERR_CURVE (-3)    /* not on the curve                                       */
#define TBG_PS_ERR_SUBGROUP (-4) /* not in the prime-order subgroup                        */
#define TBG_PS_ERR_IDENTITY (-5) /* signature is the point at infinity                     */
#define TBG_PS_ERR_PUBKEY (-6)   /* pubkey id unknown / pubkey invalid or identity         */

/* ---- per-duty status (int32) ------------------------------------------- */
#define TBG_DS_OK 0
#define TBG_DS_INSUFFICIENT (-20)        /* "insufficient signatures"        (tss.go:154-156) */
#define TBG_DS_INSUFFICIENT_VALID (-21)  /* "insufficient valid signatures"  (tss.go:176-178) */
#define TBG_DS_AGG_TOO_FEW (-22)         /* CombineSignatures: < 2 partials                   */
#define TBG_DS_AGG_DUPLICATE_ID (-23)    /* CombineSignatures: identifiers collide            */
#define TBG_DS_AGG_IDENTITY (-24)        /* CombineSignatures: identity input or result       */
#define TBG_DS_DECODE (-25)              /* a partial failed to decode (SigFromCore error)    */
#define TBG_DS_NOT_AGGREGATED 1          /* TBG_OP_VERIFY: no aggregate produced              */

#define TBG_NO_PUBKEY 0xFFFFFFFFu        /* pubkey_ids[] entry: identifier not in the TSS     */

typedef enum {
  TBG_OP_VERIFY = 1,           /* per partial: CoreVerify(pk, msg(duty), sig)                 */
  TBG_OP_AGGREGATE = 2,        /* per duty: CombineSignatures(all partials), no verification  */
  TBG_OP_VERIFY_AGGREGATE = 3  /* per duty: VerifyAndAggregate(tss, partials, msg)            */
} tbg_op;

typedef struct tbg_ctx tbg_ctx;
typedef uint64_t tbg_ticket;

/* Bounds of tbg_config.slots and of the streams they own: every slot owns
 * streams_per_slot (1 or 2) HIP streams, and past ~16 streams per process the
 * HSA runtime runs out of queue resources (observed on MI355X).  tbg_init
 * refuses slots > TBG_MAX_SLOTS and slots * streams_per_slot >
 * TBG_MAX_SLOT_STREAMS with TBG_E_INVALID_ARG instead of failing inside HIP.
 * The express slot (express_partials) owns one stream more: when
 * slots * streams_per_slot + 1 would pass the bound, the context runs
 * without an express slot instead.
 * The bound is per context: several contexts on ONE device (tbg_multi_init
 * with a repeated ordinal) add their streams up, so keep their sum below it. */
#define TBG_MAX_SLOTS 12
#define TBG_MAX_SLOT_STREAMS 16

typedef struct {
  int32_t device;         /* HIP device ordinal                           */
  uint32_t max_partials;  /* staging capacity hint (grows on demand)       */
  uint32_t max_duties;
  uint32_t max_msg_bytes;
  uint32_t slots;         /* in-flight batches, each on its own streams (0 -> 3, <= TBG_MAX_SLOTS) */
  uint32_t verify_mode;   /* TBG_VERIFY_RLC (0, default) or TBG_VERIFY_EACH     */
  uint32_t rlc_group;     /* duties per level-1 RLC group; 0 -> adaptive: 16 while the
                           * collected batches are clean, 8 / 4 once their share of
                           * invalid partials passes 0.3 % / 3 % (TBG_RLC_AUTO_*)   */
  uint64_t rlc_seed;      /* 0: fresh OS randomness per batch; else fixed (tests).
                           * Keys the RLC scalars only: the batched subgroup test's
                           * combinations always take fresh OS randomness            */
  uint32_t rlc_chunk;     /* duties per Miller-loop quad inside a group (0 -> 4)  */
  uint32_t streams_per_slot; /* 1 (0 -> 1) or 2: hash_to_G2 on its own stream   */
  uint32_t rlc_batch;     /* level 0, the whole device batch as ONE check (RLC mode):
                           * TBG_RLC_L0_AUTO (0) while the collected batches are clean,
                           * TBG_RLC_L0_ON always, TBG_RLC_L0_OFF never              */
  uint32_t gident;        /* level 1g (exponent test over a failed group's partials):
                           * TBG_GIDENT_OFF (0, default), TBG_GIDENT_L3 (unresolved
                           * groups to the per-partial level) or TBG_GIDENT_CHUNKS
                           * (unresolved groups to the chunk level).  Fixed at init:
                           * the library reads no environment variables.             */
  uint32_t fb_window;     /* list positions per pass of the fallback levels' shared
                           * Miller-line buffer (22.8 KB of HBM each; 0 -> 32768):
                           * longer lists run in several passes                       */
  uint32_t subgroup_batch; /* G2 subgroup checks of the decoded signatures:
                           * TBG_SGB_AUTO (0) random-combination tests per group of
                           * consecutive partials, each member tested alone only when
                           * its group fails; the group size (1,024 down to 64)
                           * follows the collected batches' non-subgroup share, and
                           * past ~TBG_SGB_AUTO_MAX every signature is tested alone;
                           * TBG_SGB_ON always (the same group sizes); TBG_SGB_OFF
                           * every signature alone.  Batches below 2,048 partials
                           * always test each signature alone.                        */
  uint32_t express_partials; /* batches of at most this many partials go to an extra
                           * slot on a high-priority stream when it is free (a small
                           * batch's ~50 short kernels then dispatch ahead of the
                           * throughput launches' workgroups): 0 -> TBG_EXPRESS_PARTIALS,
                           * TBG_EXPRESS_OFF -> no express slot                        */
} tbg_config;
#define TBG_EXPRESS_PARTIALS 4096u
#define TBG_EXPRESS_OFF 0xFFFFFFFFu
#define TBG_SGB_AUTO 0
#define TBG_SGB_ON 1
#define TBG_SGB_OFF 2
/* Where the automatic mode stops: past this non-subgroup share even the best
 * group size (128) fails ~30 % of its groups, and the batched test would cost
 * more than ~0.95 of testing every signature alone (tbls_engine.hip sgb_plan). */
#define TBG_SGB_AUTO_MAX 2.5e-3
#define TBG_GIDENT_OFF 0
#define TBG_GIDENT_L3 1
#define TBG_GIDENT_CHUNKS 2

/* Verification schedule.  Both give every partial the verdict of the exact
 * per-item CoreVerify: RLC checks random linear combinations of groups of
 * duties first and falls back to duties, then to single partials, on any
 * failure (a false accept has probability <= 2^-64 per check). */
#define TBG_VERIFY_RLC 0
#define TBG_VERIFY_EACH 1
/* Adaptive level-1 group size (rlc_group = 0): an exponential average (weight
 * 1/2 per device batch, i.e. per tbg_submit_group, updated once every part of
 * it is collected) of the invalid share of verified partials picks
 * the group for the next submit (measured at 1 % invalid: 8 beats 16 by 1 %,
 * at 0 % 16 beats 8 by 6 %). */
#define TBG_RLC_AUTO_TO8 0.003
#define TBG_RLC_AUTO_TO4 0.03
/* Level 0 (rlc_batch): every candidate of the device batch (all batches of
 * one tbg_submit_group) in one product check whose signature side is a
 * bucket multi-scalar multiplication -- no per-partial G2 scalar
 * multiplication; a failure falls through to the group levels.  AUTO runs it
 * while the invalid-share average is below TBG_RLC_AUTO_L0 (a failed level
 * 0 costs ~10 % on top of the group levels; a pass saves ~20 %). */
#define TBG_RLC_L0_AUTO 0
#define TBG_RLC_L0_ON 1
#define TBG_RLC_L0_OFF 2
#define TBG_RLC_AUTO_L0 2e-6
/* tbg_fetch_level0 states */
#define TBG_L0_NOT_RUN 0
#define TBG_L0_PASSED 1
#define TBG_L0_FAILED 2

/* A batch of DV-duties in structure-of-arrays form.
 * Duty d owns partials [duty_first[d], duty_first[d+1]) and message duty_msg[d];
 * message m is msgs[msg_off[m] .. msg_off[m+1]). */
typedef struct {
  uint32_t op;                     /* tbg_op                                          */
  uint32_t n_duties;
  uint32_t n_partials;
  uint32_t n_msgs;
  const uint8_t* msgs;             /* concatenated message bytes (VERIFY*)            */
  const uint32_t* msg_off;         /* [n_msgs + 1]                                    */
  const uint32_t* duty_msg;        /* [n_duties]     (VERIFY*)                        */
  const uint32_t* duty_first;      /* [n_duties + 1]                                  */
  const uint32_t* duty_threshold;  /* [n_duties]     (VERIFY_AGGREGATE)               */
  const uint8_t* sigs;             /* [n_partials * 96] ZCash-compressed G2           */
  const uint8_t* identifiers;      /* [n_partials] share index (Lagrange x)           */
  const uint32_t* pubkey_ids;      /* [n_partials] resident pubkey id (VERIFY*)       */
} tbg_batch;

int tbg_init(const tbg_config* cfg, tbg_ctx** out);
void tbg_destroy(tbg_ctx* ctx);
const char* tbg_strerror(int code);
int tbg_device_count(void);
/* Compute units of HIP device `device` (the engine's SIMD count / 4), or a
 * negative TBG_E_* code.  Lets a host size work for the launch shape without
 * another HIP runtime in the process (a second libamdhip64 -- e.g. PyTorch's
 * bundled copy -- that initialises after this library's finds no devices). */
int tbg_device_cu_count(int device);
/* Wait for every stream of the context (slots, express slot, utility
 * stream): the bench's "synchronize" on both sides of its timed region. */
int tbg_synchronize(tbg_ctx* ctx);

/* Decode and validate `count` 48-byte compressed G1 public keys on the GPU
 * and append them to the resident table.  Ids are first_id .. first_id+count-1.
 * status[i] (optional) receives 0 valid, 1 identity, or a TBG_PS_ERR_* code. */
int tbg_load_pubkeys(tbg_ctx* ctx, const uint8_t* pk48, uint32_t count, uint32_t* first_id, int32_t* status);
uint32_t tbg_pubkey_count(const tbg_ctx* ctx);

/* Enqueue a batch (copies every input); returns a ticket. */
int tbg_submit(tbg_ctx* ctx, const tbg_batch* batch, tbg_ticket* ticket);

/* Enqueue several batches (same op) as ONE device batch: they are packed
 * back to back (indices rebased) and every kernel of the chain runs once
 * over all of them, so concurrent callers' batches fill the GPU together
 * instead of queueing small launches on separate streams (the call site
 * coalesces what arrives within its window -- parsigex peers, validatorapi
 * submitters, parsigdb threshold hits).  tickets[k] names batch k: collect /
 * poll / fetch it as usual; the slot is reused once every ticket has been
 * collected.  tbg_replay / tbg_fetch_stats of any of the tickets act on the
 * whole device batch. */
int tbg_submit_group(tbg_ctx* ctx, const tbg_batch* const* batches, uint32_t n_batches, tbg_ticket* tickets);

/* Collect a batch: partial_status [n_partials], duty_status [n_duties],
 * agg96 [n_duties * 96] (any may be NULL).  block = 0 polls (TBG_E_PENDING
 * while running, nothing consumed).  A blocking collect waits WITHOUT the
 * context lock, so other threads keep submitting / polling meanwhile. */
int tbg_collect(tbg_ctx* ctx, tbg_ticket ticket, int32_t* partial_status, int32_t* duty_status,
                uint8_t* agg96, int block);

/* Non-consuming readiness check: TBG_OK when finished, TBG_E_PENDING, or an
 * error code (unknown ticket / device failure). */
int tbg_poll(tbg_ctx* ctx, tbg_ticket ticket);

/* Convenience: submit + blocking collect. */
int tbg_run(tbg_ctx* ctx, const tbg_batch* batch, int32_t* partial_status, int32_t* duty_status, uint8_t* agg96);

/* Device-resident replay: re-run the kernel chain of a collected batch whose
 * inputs are still resident in its slot's HBM arena (valid until the slot is
 * reused by a later tbg_submit), `iters` times back to back, no host copies.
 * Blocks; ms8 receives per-kernel totals as in tbg_last_timings.  tbg_fetch
 * copies that slot's current outputs back (synchronous). */
int tbg_replay(tbg_ctx* ctx, tbg_ticket ticket, uint32_t iters, float* ms8);
/* Replay several collected batches round-robin, each on its own slot's
 * streams, so up to n_tickets batches are in flight at once (the pipelined
 * throughput of back-to-back submits).  ms8[7] is the wall time. */
int tbg_replay_multi(tbg_ctx* ctx, const tbg_ticket* tickets, uint32_t n_tickets, uint32_t iters, float* ms8);
/* Replay an explicit plan: launch k re-runs the first n_parts[k] caller
 * batches (0 or NULL: all) of the resident device batch tickets[k] belongs
 * to (a prefix of a packed tbg_submit_group batch is a batch of its own), on
 * that slot's streams; launches of different slots are in flight together. */
int tbg_replay_plan(tbg_ctx* ctx, const tbg_ticket* tickets, const uint32_t* n_parts, uint32_t n_launches, float* ms8);
int tbg_fetch(tbg_ctx* ctx, tbg_ticket ticket, int32_t* partial_status, int32_t* duty_status, uint8_t* agg96);
/* Measurement hook (bench.py's roofline): replay one collected device batch
 * ALONE (the context's other slots drained first) with a HIP event pair
 * around every kernel launch on the stream it runs on; out[k] = the k-th
 * launch's kernel name (as written at the launch site) and duration in ms,
 * in launch order, at most max_entries of them.  Blocks. */
typedef struct {
  char name[64];
  float ms;
} tbg_kernel_time;
int tbg_replay_profile(tbg_ctx* ctx, tbg_ticket ticket, tbg_kernel_time* out, uint32_t max_entries,
                       uint32_t* n_entries);
/* Verification work of a collected batch's last run: out4 = [level-1 groups,
 * failed duties searched for their invalid partial (level 2b), partials
 * checked one by one (level 3), duties per group (0 = TBG_VERIFY_EACH)]. */
int tbg_fetch_stats(tbg_ctx* ctx, tbg_ticket ticket, uint32_t* out4);
/* Level 0 of a collected batch's last run: *state = TBG_L0_NOT_RUN,
 * TBG_L0_PASSED (every candidate accepted by the one batch-wide check) or
 * TBG_L0_FAILED (the group levels decided). */
int tbg_fetch_level0(tbg_ctx* ctx, tbg_ticket ticket, int32_t* state);
/* Fallback work of a collected batch's last run, per level: out8 = [level-1
 * groups, groups searched at level 1g (exponent test over a failed group's
 * partials), chunks re-checked at level 1.5, chunks searched at level 1.5b,
 * duties searched at level 2b, partials checked one by one at level 3,
 * duties per group, level 0 (TBG_L0_*)]. */
int tbg_fetch_fallback(tbg_ctx* ctx, tbg_ticket ticket, uint32_t* out8);
/* Batched subgroup test of a collected batch's last run (tbg_config.
 * subgroup_batch): out3 = [groups of consecutive partials tested by random
 * combinations (0: every signature was tested alone), groups that failed
 * (their members were then tested one by one), partials per group]. */
int tbg_fetch_subgroup(tbg_ctx* ctx, tbg_ticket ticket, uint32_t* out3);
/* Verification shape of a collected batch's last submit: out4 = [duties per
 * group G, duties per Miller chunk C, level 0 on (1) or off, Miller P-chunk
 * hexads G x C cut the batch into].  A level-0 launch with neither G nor C
 * configured picks (G, C) by the device's wave slots. */
int tbg_fetch_shape(tbg_ctx* ctx, tbg_ticket ticket, uint32_t* out4);
/* Host-side work of the context's submit / collect calls since the last
 * reset (reset != 0 zeroes the counters after reading): out8 = [submit
 * calls, partials submitted, ns packing the callers' arrays into pinned
 * staging, ns enqueueing (H2D, the kernel chain, D2H), collect calls,
 * partials collected, ns gathering (copy-out of statuses / aggregates and
 * the adaptive policies' counts), ns waiting for the device]. */
int tbg_host_stats(tbg_ctx* ctx, uint64_t* out8, int reset);
/* Footprint of the slot holding the ticket's batch: device bytes (input
 * arena + work arena) and pinned host bytes (staging both ways). */
int tbg_slot_bytes(tbg_ctx* ctx, tbg_ticket ticket, uint64_t* device_bytes, uint64_t* pinned_bytes);

/* Plain BLS aggregation (every coefficient 1) for the DKG / cluster-lock
 * multi-signatures: AggregatePublicKeys / AggregateSignatures of
 * aggLockHashSig (reference dkg/dkg.go:466-476) and FastAggregateVerify of
 * Lock.VerifySignatures (cluster/lock.go:155-177).  Set k covers items
 * [off[k], off[k+1]); off[0] = 0.
 * tbg_sum_pubkeys: sum of resident public keys (ids from tbg_load_pubkeys);
 *   out48[k] the compressed sum, status[k] TBG_DS_OK, TBG_DS_AGG_IDENTITY
 *   (empty set or identity sum; out48 = the identity encoding) or
 *   TBG_DS_DECODE (an unknown id or a key that failed to decode; out48 zero).
 * tbg_sum_sigs: decode (flags, field, curve, subgroup) and sum 96-byte
 *   signatures; status as above (the identity encoding decodes and adds
 *   nothing); sig_status (optional) per signature: TBG_PS_NOT_VERIFIED, or
 *   its decode code (TBG_PS_ERR_IDENTITY for the identity).
 * tbg_fast_aggregate_verify: per set, CoreVerify(sum of its keys, msg k,
 *   sig k) on the GPU; status[k] TBG_PS_VALID / TBG_PS_INVALID / a signature
 *   decode code / TBG_PS_ERR_PUBKEY (the key sum failed or is the identity). */
int tbg_sum_pubkeys(tbg_ctx* ctx, const uint32_t* pubkey_ids, const uint32_t* off, uint32_t n_sets, uint8_t* out48,
                    int32_t* status);
int tbg_sum_sigs(tbg_ctx* ctx, const uint8_t* sigs96, const uint32_t* off, uint32_t n_sets, uint8_t* out96,
                 int32_t* status, int32_t* sig_status);
int tbg_fast_aggregate_verify(tbg_ctx* ctx, const uint32_t* pubkey_ids, const uint32_t* key_off, uint32_t n_sets,
                              const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* sigs96, int32_t* status);

/* Test-vector / benchmark-input generation on the GPU (not on the hot path):
 * tbls.Sign / PartialSign (reference tbls/tss.go:200-217) and
 * SecretKey.GetPublicKey.  sk32: 32-byte big-endian secret scalars (< r).
 * tbg_sign signs item i with sk32[i] over message item_msg[i].
 * TEST-ONLY: the scalar multiplication by sk is a plain double-and-add whose
 * timing depends on the key, so these entry points are not side-channel safe
 * and must not hold a production validator key (the Z inversions of the
 * results use the constant-time Fermat inversion, but that alone does not
 * make the path constant time). */
int tbg_sk_to_pk(tbg_ctx* ctx, const uint8_t* sk32, uint32_t n, uint8_t* pk48);
int tbg_sign(tbg_ctx* ctx, const uint8_t* sk32, uint32_t n, const uint8_t* msgs, const uint32_t* msg_off,
             uint32_t n_msgs, const uint32_t* item_msg, uint8_t* sig96);

/* Last kernel timings of the context (milliseconds, HIP events on the
 * engine's streams): [decode, hash, combine (RLC sums + group lines),
 * H lines, verify (all check levels), lagrange, aggregate, total]. */
int tbg_last_timings(const tbg_ctx* ctx, float* ms8);

/* ---- one process, several GPUs (BASELINE config 4) -----------------------
 * A Charon node is one process: a multi-context owns one tbg_ctx per entry of
 * devices[] (entries may repeat, e.g. several contexts on one GPU in tests)
 * and shards every batch across them with no cross-device math.  Duties are
 * independent, so a batch is cut into contiguous duty ranges
 * of about equal partial counts, each range is submitted to its context
 * concurrently (host packing on one thread per context), and tbg_multi_collect
 * gathers partial_status / duty_status / agg96 straight into the caller's
 * arrays at the range offsets -- caller order is preserved by construction.
 * The gathered loops are the per-DV loops of core/parsigex/parsigex.go:101-107
 * and core/parsigdb/memory.go:96-134 -> core/sigagg/sigagg.go:53-103; the
 * engine is initialised from the app wiring (app/app.go:321-488).
 *
 * Public keys are replicated: tbg_multi_load_pubkeys decodes the table on
 * every device (1 M DVs x 4 shares x 1,124 B ~ 4.5 GB, 1.6 % of a GPU's 288
 * GB: pk, [x]pk and the RLC products' 8-entry window table, 10 x 112 B of
 * affine G1, + status), so any shard can reference any id and the ids are the same as for a
 * single context.  Replication is the chosen design: the cut follows the
 * partial counts of whatever batches arrive (a burst of one committee's
 * duties still spreads over every GPU), where key-owned shards would route
 * each duty to its keys' GPU and leave the others idle for a skewed burst
 * (DESIGN.md section 5).  cfg->device is ignored (devices[] is used).
 * Thread-safe. */
typedef struct tbg_multi tbg_multi;
int tbg_multi_init(const tbg_config* cfg, const int32_t* devices, uint32_t n_devices, tbg_multi** out);
void tbg_multi_destroy(tbg_multi* m);
uint32_t tbg_multi_size(const tbg_multi* m);
/* The context of shard i (0 <= i < tbg_multi_size), for timings / stats. */
tbg_ctx* tbg_multi_context(tbg_multi* m, uint32_t i);
int tbg_multi_load_pubkeys(tbg_multi* m, const uint8_t* pk48, uint32_t count, uint32_t* first_id, int32_t* status);
int tbg_multi_submit(tbg_multi* m, const tbg_batch* batch, tbg_ticket* ticket);
/* Several caller batches (same op) as ONE multi-device launch: the batches
 * taken back to back are cut into n contiguous ranges of about equal partial
 * counts, and each context's pieces are packed into one device batch
 * (tbg_submit_group), so concurrent callers' batches fill every GPU together
 * instead of each batch being cut into n small launches.  tickets[k] names
 * batch k for tbg_multi_collect / tbg_multi_layout (its cut points in its own
 * duties).  tbg_multi_submit(b) is tbg_multi_submit_group(&b, 1). */
int tbg_multi_submit_group(tbg_multi* m, const tbg_batch* const* batches, uint32_t n_batches, tbg_ticket* tickets);
/* Same contract as tbg_collect; block = 0 returns TBG_E_PENDING until EVERY
 * shard has finished (nothing is consumed before that). */
int tbg_multi_collect(tbg_multi* m, tbg_ticket ticket, int32_t* partial_status, int32_t* duty_status,
                      uint8_t* agg96, int block);
/* Host-side work of the multi-context's calls since the last reset (reset
 * != 0 zeroes every counter, the contexts' too): out16 = [submit calls,
 * partials submitted, ns building the per-context sub-batches (summed over
 * the host workers), submit wall ns, collect calls, collect wall ns, then
 * the 8 tbg_host_stats counters summed over the contexts (pack ns and
 * gather ns are CPU time of the context's own thread), context count, 0].
 * The cut / pack / gather run on persistent per-context host workers. */
int tbg_multi_host_stats(tbg_multi* m, uint64_t* out16, int reset);
/* Shard layout of a submitted (not yet collected) ticket: for shard i,
 * duty range [duty_lo[i], duty_lo[i+1]); arrays of tbg_multi_size()+1. */
int tbg_multi_layout(tbg_multi* m, tbg_ticket ticket, uint32_t* duty_lo);

#ifdef __cplusplus
}
#endif
#endif /* TBLS_GPU_H */
