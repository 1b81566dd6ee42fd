/*
 * cabi_threads.c -- drives libtbls_gpu.so from 8 threads the way the cgo
 * binding of INTEGRATION.md does: every goroutine submits its own batch and
 * polls tbg_collect(block = 0) (half of them block instead), several batches
 * in flight per context, plus one multi-context (tbg_multi_*) shared by all
 * threads.  Every result is checked:
 *
 *   OP_VERIFY_AGGREGATE over 3-of-4 DVs whose shares are f(1..4) of a small
 *   integer polynomial f(x) = s + c1 x + c2 x^2 (no reduction mod r needed),
 *   so the aggregate must equal tbg_sign(s, msg); one partial per DV is a
 *   wrong-message signature (must be TBG_PS_INVALID, aggregate unchanged).
 *
 * Plain C (the cgo side is C); built here by tests/cabi/Makefile (also with
 * AddressSanitizer on the host code), run on the GPU box.
 * Exit 0 and "cabi_threads: PASS" on success.
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "tbls_gpu.h"

#define NTHREADS 8
#define ITERS 6
#define NDV 96
#define NP (NDV * 4)

static tbg_ctx* g_ctx;
static tbg_multi* g_multi;
static uint8_t g_sig[NP * 96], g_wrong[NP * 96], g_group[NDV * 96];
static uint32_t g_pkid[NP], g_pkid_multi[NP];
static uint8_t g_msgs[NDV * 32];
static int g_fail;

static void fail(const char* what, int rc) {
  fprintf(stderr, "FAIL %s: %d (%s)\n", what, rc, tbg_strerror(rc));
  __atomic_store_n(&g_fail, 1, __ATOMIC_SEQ_CST);
}

/* big-endian 32-byte scalar from a small integer */
static void scalar32(uint64_t v, uint8_t* out) {
  memset(out, 0, 32);
  for (int i = 0; i < 8; ++i) out[31 - i] = (uint8_t)(v >> (8 * i));
}

static int setup(void) {
  uint8_t sk[NP * 32], gsk[NDV * 32], pk[NP * 48];
  uint32_t off[NDV + 1], item[NP], gitem[NDV];
  for (int d = 0; d < NDV; ++d) {
    uint64_t s = 1000 + 7919 * (uint64_t)d, c1 = 31 + d, c2 = 17 * (d + 3);
    scalar32(s, gsk + 32 * d);
    gitem[d] = d;
    for (int x = 1; x <= 4; ++x) {
      uint64_t f = s + c1 * x + c2 * x * x;
      scalar32(f, sk + 32 * (4 * d + x - 1));
      item[4 * d + x - 1] = d;
    }
    for (int j = 0; j < 32; ++j) g_msgs[32 * d + j] = (uint8_t)(d * 131 + j * 7 + 1);
    off[d] = 32 * d;
  }
  off[NDV] = 32 * NDV;
  int rc;
  if ((rc = tbg_sign(g_ctx, sk, NP, g_msgs, off, NDV, item, g_sig))) return rc;
  if ((rc = tbg_sign(g_ctx, gsk, NDV, g_msgs, off, NDV, gitem, g_group))) return rc;
  uint8_t wrong_msgs[NDV * 32];
  memcpy(wrong_msgs, g_msgs, sizeof(wrong_msgs));
  for (int d = 0; d < NDV; ++d) wrong_msgs[32 * d] ^= 0x80;
  if ((rc = tbg_sign(g_ctx, sk, NP, wrong_msgs, off, NDV, item, g_wrong))) return rc;
  if ((rc = tbg_sk_to_pk(g_ctx, sk, NP, pk))) return rc;
  uint32_t first = 0;
  int32_t st[NP];
  if ((rc = tbg_load_pubkeys(g_ctx, pk, NP, &first, st))) return rc;
  for (int i = 0; i < NP; ++i) {
    if (st[i] != 0) return -100;
    g_pkid[i] = first + i;
  }
  if ((rc = tbg_multi_load_pubkeys(g_multi, pk, NP, &first, st))) return rc;
  for (int i = 0; i < NP; ++i) g_pkid_multi[i] = first + i;
  return 0;
}

struct job {
  int tid;
  int use_multi;
};

static void* worker(void* arg) {
  struct job* j = (struct job*)arg;
  uint32_t duty_first[NDV + 1], duty_msg[NDV], thr[NDV], off[NDV + 1];
  uint8_t ids[NP];
  uint8_t* sigs = malloc(NP * 96);
  int32_t* ps = malloc(sizeof(int32_t) * NP);
  int32_t* ds = malloc(sizeof(int32_t) * NDV);
  uint8_t* agg = malloc(NDV * 96);
  for (int d = 0; d <= NDV; ++d) { duty_first[d] = 4 * d; off[d] = 32 * d; }
  for (int d = 0; d < NDV; ++d) { duty_msg[d] = d; thr[d] = 3; }
  for (int i = 0; i < NP; ++i) ids[i] = (uint8_t)(i % 4 + 1);
  for (int it = 0; it < ITERS && !g_fail; ++it) {
    /* partial (d, k) with k = (d + tid + it) % 4 is a wrong-message signature */
    memcpy(sigs, g_sig, NP * 96);
    for (int d = 0; d < NDV; ++d) {
      int k = (d + j->tid + it) % 4;
      memcpy(sigs + 96 * (4 * d + k), g_wrong + 96 * (4 * d + k), 96);
    }
    tbg_batch b;
    memset(&b, 0, sizeof(b));
    b.op = TBG_OP_VERIFY_AGGREGATE;
    b.n_duties = NDV;
    b.n_partials = NP;
    b.n_msgs = NDV;
    b.msgs = g_msgs;
    b.msg_off = off;
    b.duty_msg = duty_msg;
    b.duty_first = duty_first;
    b.duty_threshold = thr;
    b.sigs = sigs;
    b.identifiers = ids;
    b.pubkey_ids = j->use_multi ? g_pkid_multi : g_pkid;
    tbg_ticket t;
    int rc;
    for (;;) {  /* TBG_E_BUSY: every slot in flight -- back off like the Go side */
      rc = j->use_multi ? tbg_multi_submit(g_multi, &b, &t) : tbg_submit(g_ctx, &b, &t);
      if (rc != TBG_E_BUSY) break;
      struct timespec ts = {0, 200000};
      nanosleep(&ts, NULL);
    }
    if (rc) { fail("submit", rc); break; }
    memset(sigs, 0, NP * 96);  /* the library copied everything: the caller may reuse its buffers */
    int block = j->tid & 1;
    for (;;) {
      rc = j->use_multi ? tbg_multi_collect(g_multi, t, ps, ds, agg, block)
                        : tbg_collect(g_ctx, t, ps, ds, agg, block);
      if (rc != TBG_E_PENDING) break;
      struct timespec ts = {0, 100000};
      nanosleep(&ts, NULL);
    }
    if (rc) { fail("collect", rc); break; }
    for (int d = 0; d < NDV; ++d) {
      int k = (d + j->tid + it) % 4;
      for (int x = 0; x < 4; ++x) {
        int want = x == k ? TBG_PS_INVALID : TBG_PS_VALID;
        if (ps[4 * d + x] != want) { fail("partial status", ps[4 * d + x]); goto out; }
      }
      if (ds[d] != TBG_DS_OK) { fail("duty status", ds[d]); goto out; }
      if (memcmp(agg + 96 * d, g_group + 96 * d, 96) != 0) { fail("aggregate bytes", d); goto out; }
    }
  }
out:
  free(sigs);
  free(ps);
  free(ds);
  free(agg);
  return NULL;
}

int main(void) {
  if (tbg_device_count() < 1) { fprintf(stderr, "no device\n"); return 2; }
  tbg_config cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.slots = 4;
  int rc = tbg_init(&cfg, &g_ctx);
  if (rc) { fail("tbg_init", rc); return 1; }
  cfg.slots = TBG_MAX_SLOTS + 1;
  tbg_ctx* bad = NULL;
  if (tbg_init(&cfg, &bad) != TBG_E_INVALID_ARG) { fail("slots above TBG_MAX_SLOTS accepted", 0); return 1; }
  cfg.slots = 2;
  int32_t devs[2] = {0, 0};
  if ((rc = tbg_multi_init(&cfg, devs, 2, &g_multi))) { fail("tbg_multi_init", rc); return 1; }
  if ((rc = setup())) { fail("setup", rc); return 1; }
  pthread_t th[NTHREADS];
  struct job jobs[NTHREADS];
  for (int i = 0; i < NTHREADS; ++i) {
    jobs[i].tid = i;
    jobs[i].use_multi = i >= NTHREADS - 2; /* two goroutines share the multi-context */
    pthread_create(&th[i], NULL, worker, &jobs[i]);
  }
  for (int i = 0; i < NTHREADS; ++i) pthread_join(th[i], NULL);
  /* unknown / consumed tickets */
  int32_t ps[1];
  if (tbg_collect(g_ctx, 999999, ps, NULL, NULL, 1) != TBG_E_TICKET) fail("unknown ticket accepted", 0);
  tbg_multi_destroy(g_multi);
  tbg_destroy(g_ctx);
  if (g_fail) return 1;
  printf("cabi_threads: PASS (%d threads x %d batches of %d DVs, %d through tbg_multi)\n", NTHREADS, ITERS, NDV,
         2 * ITERS);
  return 0;
}
