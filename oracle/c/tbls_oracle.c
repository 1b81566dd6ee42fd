/*
 * oracle/c/tbls_oracle.c -- C restatement of the reference tbls hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/ (differential checks of the HIP
 * engine at sizes the Python oracle cannot reach), __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg (the timed CPU port).  The product path
 * (charon_amd/) never loads it.
 *
 * Restates, independently of the engine's code (64-bit limbs, CIOS
 * Montgomery, projective Miller loop, affine-inversion SSWU):
 *   tbls.Verify              reference tbls/tss.go:190-197
 *   tbls.Aggregate           reference tbls/tss.go:142-149
 *   tbls.VerifyAndAggregate  reference tbls/tss.go:153-187
 *   tblsconv.SigFromCore / SigToCore / KeyFromBytes
 *                            reference tbls/tblsconv/tblsconv.go:30-37,119-132
 * through the published algorithms kryptology's SigEth2 implements (the IETF
 * BLS draft POP ciphersuite named at tss.go:28-31, RFC 9380 hash-to-G2,
 * ZCash point encoding, Lagrange recombination at 0).  Per item it follows
 * the reference schedule: decompress + subgroup check, hash_to_G2, one
 * two-pair pairing check per partial, one Lagrange combination per duty.
 * Status codes and their precedence match include/tbls_gpu.h.
 *
 * Pinned through oracle/bls12_381.py (itself pinned by the reference KATs):
 * tests/test_oracle_c.py checks this library against it and against the
 * golden fixtures.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

#define NP 6 /* Fp limbs */
#define NR 4 /* Fr limbs */

/* ===================================================================== */
/* multiprecision helpers (little-endian 64-bit limbs)                   */
/* ===================================================================== */
static const u64 P_MOD[NP] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                              0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const u64 R_MOD[NR] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                              0x73eda753299d7d48ULL};
static const u64 X_ABS = 0xd201000000010000ULL; /* |x|, x < 0 */

static int mp_cmp(const u64* a, const u64* b, int n) {
  for (int i = n - 1; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  }
  return 0;
}
static u64 mp_add(u64* r, const u64* a, const u64* b, int n) {
  u64 c = 0;
  for (int i = 0; i < n; ++i) {
    u128 s = (u128)a[i] + b[i] + c;
    r[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  return c;
}
static u64 mp_sub(u64* r, const u64* a, const u64* b, int n) {
  u64 br = 0;
  for (int i = 0; i < n; ++i) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
  return br;
}
static void mp_shr(u64* r, const u64* a, int n, int s) {
  for (int i = 0; i < n; ++i) r[i] = (a[i] >> s) | (i + 1 < n && s ? a[i + 1] << (64 - s) : 0);
}
static void mp_small(u64* r, u64 v, int n) {
  memset(r, 0, 8 * n);
  r[0] = v;
}
/* r = a / d for a small d (exact or floor) */
static void mp_divsmall(u64* r, const u64* a, u64 d, int n) {
  u128 rem = 0;
  for (int i = n - 1; i >= 0; --i) {
    u128 cur = (rem << 64) | a[i];
    r[i] = (u64)(cur / d);
    rem = cur % d;
  }
}
static void mp_mulsmall(u64* r, const u64* a, u64 k, int n) {
  u128 c = 0;
  for (int i = 0; i < n; ++i) {
    c += (u128)a[i] * k;
    r[i] = (u64)c;
    c >>= 64;
  }
}
static int mp_bit(const u64* e, int i) { return (int)((e[i >> 6] >> (i & 63)) & 1); }
static int mp_bits(const u64* e, int n) {
  for (int i = n * 64 - 1; i >= 0; --i)
    if (mp_bit(e, i)) return i + 1;
  return 0;
}

/* CIOS Montgomery product mod m (n limbs), inputs < m, output < m. */
static inline __attribute__((always_inline)) void mont_mul(u64* r, const u64* a, const u64* b, const u64* m, u64 minv, int n) {
  u64 t[NP + 2];
  memset(t, 0, sizeof(t));
  for (int i = 0; i < n; ++i) {
    u128 c = 0;
    for (int j = 0; j < n; ++j) {
      c += (u128)a[j] * b[i] + t[j];
      t[j] = (u64)c;
      c >>= 64;
    }
    u128 s = (u128)t[n] + (u64)c;
    t[n] = (u64)s;
    t[n + 1] = (u64)(s >> 64);
    u64 q = t[0] * minv;
    c = ((u128)q * m[0] + t[0]) >> 64;
    for (int j = 1; j < n; ++j) {
      c += (u128)q * m[j] + t[j];
      t[j - 1] = (u64)c;
      c >>= 64;
    }
    s = (u128)t[n] + (u64)c;
    t[n - 1] = (u64)s;
    t[n] = t[n + 1] + (u64)(s >> 64);
  }
  u64 d[NP];
  u64 br = mp_sub(d, t, m, n);
  if (t[n] || !br) memcpy(r, d, 8 * n);
  else memcpy(r, t, 8 * n);
}

/* ===================================================================== */
/* Fp                                                                     */
/* ===================================================================== */
typedef struct { u64 v[NP]; } fp;

static u64 P_MINV;
static fp FP_ONE, FP_R2, FP_ZERO;
static u64 E_P_MINUS_2[NP], E_SQRT[NP], E_PM3D4[NP], E_PM1D2[NP];

static void fp_add(fp* r, const fp* a, const fp* b) {
  u64 s[NP];
  u64 c = mp_add(s, a->v, b->v, NP);
  u64 d[NP];
  u64 br = mp_sub(d, s, P_MOD, NP);
  if (c || !br) memcpy(r->v, d, sizeof(d));
  else memcpy(r->v, s, sizeof(s));
}
static void fp_sub(fp* r, const fp* a, const fp* b) {
  u64 d[NP];
  u64 br = mp_sub(d, a->v, b->v, NP);
  if (br) mp_add(d, d, P_MOD, NP);
  memcpy(r->v, d, sizeof(d));
}
static void fp_neg(fp* r, const fp* a) { fp_sub(r, &FP_ZERO, a); }
static void fp_mul(fp* r, const fp* a, const fp* b) { mont_mul(r->v, a->v, b->v, P_MOD, P_MINV, NP); }
static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static int fp_is_zero(const fp* a) {
  u64 o = 0;
  for (int i = 0; i < NP; ++i) o |= a->v[i];
  return o == 0;
}
static int fp_eq(const fp* a, const fp* b) { return memcmp(a->v, b->v, sizeof(a->v)) == 0; }
static void fp_pow(fp* r, const fp* a, const u64* e) {
  fp acc = FP_ONE;
  for (int i = mp_bits(e, NP) - 1; i >= 0; --i) {
    fp_sqr(&acc, &acc);
    if (mp_bit(e, i)) fp_mul(&acc, &acc, a);
  }
  *r = acc;
}
static void fp_inv(fp* r, const fp* a) { fp_pow(r, a, E_P_MINUS_2); }
static void fp_to_mont(fp* r, const u64* plain) {
  fp t;
  memcpy(t.v, plain, sizeof(t.v));
  fp_mul(r, &t, &FP_R2);
}
static void fp_from_mont(u64* plain, const fp* a) {
  fp one;
  mp_small(one.v, 1, NP);
  fp t;
  fp_mul(&t, a, &one);
  memcpy(plain, t.v, sizeof(t.v));
}
static void fp_from_u64(fp* r, u64 v) {
  u64 t[NP];
  mp_small(t, v, NP);
  fp_to_mont(r, t);
}
/* 48 big-endian bytes -> plain limbs */
static void be48_to_limbs(u64* r, const uint8_t* b) {
  for (int i = 0; i < NP; ++i) {
    u64 w = 0;
    for (int k = 0; k < 8; ++k) w = (w << 8) | b[(NP - 1 - i) * 8 + k];
    r[i] = w;
  }
}
static void limbs_to_be48(uint8_t* b, const u64* a) {
  for (int i = 0; i < NP; ++i)
    for (int k = 0; k < 8; ++k) b[(NP - 1 - i) * 8 + k] = (uint8_t)(a[i] >> (56 - 8 * k));
}
static int fp_lex_largest(const fp* a) { /* value > (p-1)/2 */
  u64 v[NP];
  fp_from_mont(v, a);
  return mp_cmp(v, E_PM1D2, NP) > 0;
}

/* ===================================================================== */
/* Fp2 = Fp[u] / (u^2 + 1)                                                */
/* ===================================================================== */
typedef struct { fp c0, c1; } fp2;
static fp2 FP2_ONE, FP2_ZERO;

static void fp2_add(fp2* r, const fp2* a, const fp2* b) { fp_add(&r->c0, &a->c0, &b->c0); fp_add(&r->c1, &a->c1, &b->c1); }
static void fp2_sub(fp2* r, const fp2* a, const fp2* b) { fp_sub(&r->c0, &a->c0, &b->c0); fp_sub(&r->c1, &a->c1, &b->c1); }
static void fp2_neg(fp2* r, const fp2* a) { fp_neg(&r->c0, &a->c0); fp_neg(&r->c1, &a->c1); }
static void fp2_dbl(fp2* r, const fp2* a) { fp2_add(r, a, a); }
static void fp2_conj(fp2* r, const fp2* a) { r->c0 = a->c0; fp_neg(&r->c1, &a->c1); }
static void fp2_mul(fp2* r, const fp2* a, const fp2* b) {
  fp t0, t1, s0, s1, t2;
  fp_mul(&t0, &a->c0, &b->c0);
  fp_mul(&t1, &a->c1, &b->c1);
  fp_add(&s0, &a->c0, &a->c1);
  fp_add(&s1, &b->c0, &b->c1);
  fp_mul(&t2, &s0, &s1);
  fp_sub(&r->c0, &t0, &t1);
  fp_sub(&t2, &t2, &t0);
  fp_sub(&r->c1, &t2, &t1);
}
static void fp2_sqr(fp2* r, const fp2* a) {
  fp s, d, m;
  fp_add(&s, &a->c0, &a->c1);
  fp_sub(&d, &a->c0, &a->c1);
  fp_mul(&m, &a->c0, &a->c1);
  fp_mul(&r->c0, &s, &d);
  fp_add(&r->c1, &m, &m);
}
static void fp2_mul_fp(fp2* r, const fp2* a, const fp* s) { fp_mul(&r->c0, &a->c0, s); fp_mul(&r->c1, &a->c1, s); }
static void fp2_mul_xi(fp2* r, const fp2* a) { /* (1 + u) a */
  fp t0, t1;
  fp_sub(&t0, &a->c0, &a->c1);
  fp_add(&t1, &a->c0, &a->c1);
  r->c0 = t0;
  r->c1 = t1;
}
static int fp2_is_zero(const fp2* a) { return fp_is_zero(&a->c0) && fp_is_zero(&a->c1); }
static int fp2_eq(const fp2* a, const fp2* b) { return fp_eq(&a->c0, &b->c0) && fp_eq(&a->c1, &b->c1); }
static void fp2_inv(fp2* r, const fp2* a) {
  fp n, t;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  fp_inv(&n, &n);
  fp_mul(&r->c0, &a->c0, &n);
  fp_mul(&t, &a->c1, &n);
  fp_neg(&r->c1, &t);
}
static void fp2_pow(fp2* r, const fp2* a, const u64* e, int n) {
  fp2 acc = FP2_ONE;
  for (int i = mp_bits(e, n) - 1; i >= 0; --i) {
    fp2_sqr(&acc, &acc);
    if (mp_bit(e, i)) fp2_mul(&acc, &acc, a);
  }
  *r = acc;
}
/* square root (Adj-Rodriguez-Henriquez, p = 3 mod 4); 0 when not a square */
static int fp2_sqrt(fp2* r, const fp2* a) {
  if (fp2_is_zero(a)) {
    *r = FP2_ZERO;
    return 1;
  }
  fp2 a1, alpha, x0, x, t;
  fp2_pow(&a1, a, E_PM3D4, NP);
  fp2_sqr(&alpha, &a1);
  fp2_mul(&alpha, &alpha, a);
  fp2_mul(&x0, &a1, a);
  fp2 minus_one;
  fp2_neg(&minus_one, &FP2_ONE);
  if (fp2_eq(&alpha, &minus_one)) {
    fp_neg(&x.c0, &x0.c1); /* u * x0 */
    x.c1 = x0.c0;
  } else {
    fp2 b;
    fp2_add(&t, &FP2_ONE, &alpha);
    fp2_pow(&b, &t, E_PM1D2, NP);
    fp2_mul(&x, &b, &x0);
  }
  fp2_sqr(&t, &x);
  if (!fp2_eq(&t, a)) return 0;
  *r = x;
  return 1;
}
static int fp2_is_square(const fp2* a) {
  fp n, t, l;
  fp_sqr(&n, &a->c0);
  fp_sqr(&t, &a->c1);
  fp_add(&n, &n, &t);
  if (fp_is_zero(&n)) return 1;
  fp_pow(&l, &n, E_PM1D2);
  return fp_eq(&l, &FP_ONE);
}
static int fp2_sgn0(const fp2* a) {
  u64 c0[NP], c1[NP];
  fp_from_mont(c0, &a->c0);
  fp_from_mont(c1, &a->c1);
  int s0 = (int)(c0[0] & 1), z0 = 1;
  for (int i = 0; i < NP; ++i) z0 &= c0[i] == 0;
  return s0 | (z0 & (int)(c1[0] & 1));
}
static int fp2_lex_largest(const fp2* a) {
  if (!fp_is_zero(&a->c1)) return fp_lex_largest(&a->c1);
  return fp_lex_largest(&a->c0);
}

/* ===================================================================== */
/* Fp6 = Fp2[v] / (v^3 - xi), Fp12 = Fp6[w] / (w^2 - v)                   */
/* ===================================================================== */
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;
static fp12 FP12_ONE;
static fp2 FROB_GAMMA[6];
static fp2 PSI_CX, PSI_CY; /* psi(x, y) = (conj(x) PSI_CX, conj(y) PSI_CY) */

static void fp6_add(fp6* r, const fp6* a, const fp6* b) { fp2_add(&r->c0, &a->c0, &b->c0); fp2_add(&r->c1, &a->c1, &b->c1); fp2_add(&r->c2, &a->c2, &b->c2); }
static void fp6_sub(fp6* r, const fp6* a, const fp6* b) { fp2_sub(&r->c0, &a->c0, &b->c0); fp2_sub(&r->c1, &a->c1, &b->c1); fp2_sub(&r->c2, &a->c2, &b->c2); }
static void fp6_neg(fp6* r, const fp6* a) { fp2_neg(&r->c0, &a->c0); fp2_neg(&r->c1, &a->c1); fp2_neg(&r->c2, &a->c2); }
static void fp6_mul(fp6* r, const fp6* a, const fp6* b) {
  fp2 t0, t1, t2, s, u, c0, c1, c2;
  fp2_mul(&t0, &a->c0, &b->c0);
  fp2_mul(&t1, &a->c1, &b->c1);
  fp2_mul(&t2, &a->c2, &b->c2);
  fp2_add(&s, &a->c1, &a->c2);
  fp2_add(&u, &b->c1, &b->c2);
  fp2_mul(&c0, &s, &u);
  fp2_sub(&c0, &c0, &t1);
  fp2_sub(&c0, &c0, &t2);
  fp2_mul_xi(&c0, &c0);
  fp2_add(&c0, &c0, &t0);
  fp2_add(&s, &a->c0, &a->c1);
  fp2_add(&u, &b->c0, &b->c1);
  fp2_mul(&c1, &s, &u);
  fp2_sub(&c1, &c1, &t0);
  fp2_sub(&c1, &c1, &t1);
  fp2_mul_xi(&s, &t2);
  fp2_add(&c1, &c1, &s);
  fp2_add(&s, &a->c0, &a->c2);
  fp2_add(&u, &b->c0, &b->c2);
  fp2_mul(&c2, &s, &u);
  fp2_sub(&c2, &c2, &t0);
  fp2_sub(&c2, &c2, &t2);
  fp2_add(&c2, &c2, &t1);
  r->c0 = c0;
  r->c1 = c1;
  r->c2 = c2;
}
static void fp6_mul_v(fp6* r, const fp6* a) {
  fp2 t;
  fp2_mul_xi(&t, &a->c2);
  r->c2 = a->c1;
  r->c1 = a->c0;
  r->c0 = t;
}
/* a * (b0 + b1 v) */
static void fp6_mul_by_01(fp6* r, const fp6* a, const fp2* b0, const fp2* b1) {
  fp2 aa, bb, t1, t2, t3, s, u;
  fp2_mul(&aa, &a->c0, b0);
  fp2_mul(&bb, &a->c1, b1);
  fp2_mul(&t1, &a->c2, b1);
  fp2_mul_xi(&t1, &t1);
  fp2_add(&t1, &t1, &aa);
  fp2_add(&s, b0, b1);
  fp2_add(&u, &a->c0, &a->c1);
  fp2_mul(&t2, &s, &u);
  fp2_sub(&t2, &t2, &aa);
  fp2_sub(&t2, &t2, &bb);
  fp2_mul(&t3, &a->c2, b0);
  fp2_add(&t3, &t3, &bb);
  r->c0 = t1;
  r->c1 = t2;
  r->c2 = t3;
}
/* a * (b1 v) */
static void fp6_mul_by_1(fp6* r, const fp6* a, const fp2* b1) {
  fp2 t0, t1, t2;
  fp2_mul(&t0, &a->c2, b1);
  fp2_mul_xi(&t0, &t0);
  fp2_mul(&t1, &a->c0, b1);
  fp2_mul(&t2, &a->c1, b1);
  r->c0 = t0;
  r->c1 = t1;
  r->c2 = t2;
}
static void fp6_inv(fp6* r, const fp6* a) {
  fp2 c0, c1, c2, t, u;
  fp2_sqr(&c0, &a->c0);
  fp2_mul(&t, &a->c1, &a->c2);
  fp2_mul_xi(&t, &t);
  fp2_sub(&c0, &c0, &t);
  fp2_sqr(&c1, &a->c2);
  fp2_mul_xi(&c1, &c1);
  fp2_mul(&t, &a->c0, &a->c1);
  fp2_sub(&c1, &c1, &t);
  fp2_sqr(&c2, &a->c1);
  fp2_mul(&t, &a->c0, &a->c2);
  fp2_sub(&c2, &c2, &t);
  fp2_mul(&t, &a->c2, &c1);
  fp2_mul(&u, &a->c1, &c2);
  fp2_add(&t, &t, &u);
  fp2_mul_xi(&t, &t);
  fp2_mul(&u, &a->c0, &c0);
  fp2_add(&t, &t, &u);
  fp2_inv(&t, &t);
  fp2_mul(&r->c0, &c0, &t);
  fp2_mul(&r->c1, &c1, &t);
  fp2_mul(&r->c2, &c2, &t);
}
static void fp12_mul(fp12* r, const fp12* a, const fp12* b) {
  fp6 t0, t1, s, u, c1;
  fp6_mul(&t0, &a->c0, &b->c0);
  fp6_mul(&t1, &a->c1, &b->c1);
  fp6_add(&s, &a->c0, &a->c1);
  fp6_add(&u, &b->c0, &b->c1);
  fp6_mul(&c1, &s, &u);
  fp6_sub(&c1, &c1, &t0);
  fp6_sub(&c1, &c1, &t1);
  fp6_mul_v(&t1, &t1);
  fp6_add(&r->c0, &t0, &t1);
  r->c1 = c1;
}
static void fp12_sqr(fp12* r, const fp12* a) { fp12_mul(r, a, a); }
static void fp12_conj(fp12* r, const fp12* a) { r->c0 = a->c0; fp6_neg(&r->c1, &a->c1); }
static void fp12_inv(fp12* r, const fp12* a) {
  fp6 t, u;
  fp6_mul(&t, &a->c0, &a->c0);
  fp6_mul(&u, &a->c1, &a->c1);
  fp6_mul_v(&u, &u);
  fp6_sub(&t, &t, &u);
  fp6_inv(&t, &t);
  fp6_mul(&r->c0, &a->c0, &t);
  fp6_mul(&u, &a->c1, &t);
  fp6_neg(&r->c1, &u);
}
/* f^p: a_k w^k -> conj(a_k) gamma_k w^k, a_0 = c0.c0, a_1 = c1.c0, a_2 = c0.c1,
 * a_3 = c1.c1, a_4 = c0.c2, a_5 = c1.c2 */
static void fp12_frob(fp12* r, const fp12* a) {
  fp2 t;
  fp2_conj(&r->c0.c0, &a->c0.c0);
  fp2_conj(&t, &a->c0.c1); fp2_mul(&r->c0.c1, &t, &FROB_GAMMA[2]);
  fp2_conj(&t, &a->c0.c2); fp2_mul(&r->c0.c2, &t, &FROB_GAMMA[4]);
  fp2_conj(&t, &a->c1.c0); fp2_mul(&r->c1.c0, &t, &FROB_GAMMA[1]);
  fp2_conj(&t, &a->c1.c1); fp2_mul(&r->c1.c1, &t, &FROB_GAMMA[3]);
  fp2_conj(&t, &a->c1.c2); fp2_mul(&r->c1.c2, &t, &FROB_GAMMA[5]);
}
/* f * (c0 + c1 v + c4 v w): sparse Miller-loop line */
static void fp12_mul_by_014(fp12* f, const fp2* c0, const fp2* c1, const fp2* c4) {
  fp6 aa, bb, s;
  fp2 o;
  fp6_mul_by_01(&aa, &f->c0, c0, c1);
  fp6_mul_by_1(&bb, &f->c1, c4);
  fp2_add(&o, c1, c4);
  fp6_add(&s, &f->c1, &f->c0);
  fp6_mul_by_01(&s, &s, c0, &o);
  fp6_sub(&s, &s, &aa);
  fp6_sub(&f->c1, &s, &bb);
  fp6_mul_v(&bb, &bb);
  fp6_add(&f->c0, &bb, &aa);
}
/* Granger-Scott squaring in the cyclotomic subgroup (after the easy part) */
static void fp4_square(fp2* t0, fp2* t1, const fp2* a, const fp2* b) {
  fp2 ab, s, u, xb;
  fp2_mul(&ab, a, b);
  fp2_mul_xi(&xb, b);
  fp2_add(&s, a, b);
  fp2_add(&u, a, &xb);
  fp2_mul(&s, &s, &u);
  fp2_mul_xi(&u, &ab);
  fp2_sub(&s, &s, &ab);
  fp2_sub(t0, &s, &u);
  fp2_dbl(t1, &ab);
}
static void fp12_cyc_sqr(fp12* r, const fp12* f) {
  fp2 z0 = f->c0.c0, z4 = f->c0.c1, z3 = f->c0.c2, z2 = f->c1.c0, z1 = f->c1.c1, z5 = f->c1.c2;
  fp2 t0, t1, t2, t3, t4, t5, x;
  fp4_square(&t0, &t1, &z0, &z1);
  fp4_square(&t2, &t3, &z2, &z3);
  fp4_square(&t4, &t5, &z4, &z5);
  fp2_sub(&z0, &t0, &z0); fp2_dbl(&z0, &z0); fp2_add(&z0, &z0, &t0);   /* 3 t0 - 2 z0 */
  fp2_add(&z1, &t1, &z1); fp2_dbl(&z1, &z1); fp2_add(&z1, &z1, &t1);   /* 3 t1 + 2 z1 */
  fp2_mul_xi(&x, &t5);
  fp2_add(&z2, &x, &z2); fp2_dbl(&z2, &z2); fp2_add(&z2, &z2, &x);     /* 3 xi t5 + 2 z2 */
  fp2_sub(&z3, &t4, &z3); fp2_dbl(&z3, &z3); fp2_add(&z3, &z3, &t4);   /* 3 t4 - 2 z3 */
  fp2_sub(&z4, &t2, &z4); fp2_dbl(&z4, &z4); fp2_add(&z4, &z4, &t2);   /* 3 t2 - 2 z4 */
  fp2_add(&z5, &t3, &z5); fp2_dbl(&z5, &z5); fp2_add(&z5, &z5, &t3);   /* 3 t3 + 2 z5 */
  r->c0.c0 = z0; r->c0.c1 = z4; r->c0.c2 = z3;
  r->c1.c0 = z2; r->c1.c1 = z1; r->c1.c2 = z5;
}
static int fp12_is_one(const fp12* a) {
  if (!fp_eq(&a->c0.c0.c0, &FP_ONE) || !fp_is_zero(&a->c0.c0.c1)) return 0;
  return fp2_is_zero(&a->c0.c1) && fp2_is_zero(&a->c0.c2) && fp2_is_zero(&a->c1.c0) && fp2_is_zero(&a->c1.c1) &&
         fp2_is_zero(&a->c1.c2);
}

/* ===================================================================== */
/* G1 / G2 (Jacobian; Z = 0 is the point at infinity)                     */
/* ===================================================================== */
typedef struct { fp x, y; int inf; } g1a;
typedef struct { fp X, Y, Z; } g1j;
typedef struct { fp2 x, y; int inf; } g2a;
typedef struct { fp2 X, Y, Z; } g2j;

#define DEFINE_CURVE(PT, AFF, F, ADD, SUB, MUL, SQR, DBLF, ISZ, INV, ONE, ZERO, EQ, NEG)                  \
  static void PT##_inf(PT* r) { r->X = ONE; r->Y = ONE; r->Z = ZERO; }                                   \
  static int PT##_is_inf(const PT* p) { return ISZ(&p->Z); }                                             \
  static void PT##_from_aff(PT* r, const AFF* a) {                                                       \
    if (a->inf) { PT##_inf(r); return; }                                                                \
    r->X = a->x; r->Y = a->y; r->Z = ONE;                                                                \
  }                                                                                                      \
  static void PT##_dbl(PT* r, const PT* p) { /* dbl-2009-l, a = 0 */                                   \
    if (PT##_is_inf(p)) { *r = *p; return; }                                                            \
    F A, B, C, D, E, G, t, X3, Y3, Z3;                                                                   \
    SQR(&A, &p->X); SQR(&B, &p->Y); SQR(&C, &B);                                                         \
    ADD(&t, &p->X, &B); SQR(&t, &t); SUB(&t, &t, &A); SUB(&t, &t, &C); DBLF(&D, &t);                    \
    DBLF(&E, &A); ADD(&E, &E, &A); SQR(&G, &E);                                                          \
    DBLF(&t, &D); SUB(&X3, &G, &t);                                                                      \
    SUB(&t, &D, &X3); MUL(&Y3, &E, &t);                                                                  \
    DBLF(&t, &C); DBLF(&t, &t); DBLF(&t, &t); SUB(&Y3, &Y3, &t);                                        \
    MUL(&Z3, &p->Y, &p->Z); DBLF(&Z3, &Z3);                                                              \
    r->X = X3; r->Y = Y3; r->Z = Z3;                                                                     \
  }                                                                                                      \
  static void PT##_add(PT* r, const PT* p, const PT* q) { /* add-2007-bl */                           \
    if (PT##_is_inf(p)) { *r = *q; return; }                                                            \
    if (PT##_is_inf(q)) { *r = *p; return; }                                                            \
    F Z1Z1, Z2Z2, U1, U2, S1, S2, H, I, J, Rr, V, t, X3, Y3, Z3;                                         \
    SQR(&Z1Z1, &p->Z); SQR(&Z2Z2, &q->Z);                                                                \
    MUL(&U1, &p->X, &Z2Z2); MUL(&U2, &q->X, &Z1Z1);                                                      \
    MUL(&S1, &p->Y, &q->Z); MUL(&S1, &S1, &Z2Z2);                                                        \
    MUL(&S2, &q->Y, &p->Z); MUL(&S2, &S2, &Z1Z1);                                                        \
    SUB(&H, &U2, &U1); SUB(&Rr, &S2, &S1);                                                               \
    if (ISZ(&H)) {                                                                                       \
      if (ISZ(&Rr)) { PT##_dbl(r, p); return; }                                                         \
      PT##_inf(r); return;                                                                               \
    }                                                                                                    \
    DBLF(&I, &H); SQR(&I, &I); MUL(&J, &H, &I);                                                          \
    DBLF(&Rr, &Rr); MUL(&V, &U1, &I);                                                                    \
    SQR(&X3, &Rr); SUB(&X3, &X3, &J); SUB(&X3, &X3, &V); SUB(&X3, &X3, &V);                             \
    SUB(&t, &V, &X3); MUL(&Y3, &Rr, &t); MUL(&t, &S1, &J); DBLF(&t, &t); SUB(&Y3, &Y3, &t);              \
    ADD(&t, &p->Z, &q->Z); SQR(&t, &t); SUB(&t, &t, &Z1Z1); SUB(&t, &t, &Z2Z2); MUL(&Z3, &t, &H);       \
    r->X = X3; r->Y = Y3; r->Z = Z3;                                                                     \
  }                                                                                                      \
  static void PT##_neg(PT* r, const PT* p) { r->X = p->X; NEG(&r->Y, &p->Y); r->Z = p->Z; }             \
  static void PT##_to_aff(AFF* r, const PT* p) {                                                         \
    if (PT##_is_inf(p)) { r->inf = 1; r->x = ZERO; r->y = ZERO; return; }                               \
    F zi, zi2, zi3;                                                                                      \
    INV(&zi, &p->Z); SQR(&zi2, &zi); MUL(&zi3, &zi2, &zi);                                               \
    MUL(&r->x, &p->X, &zi2); MUL(&r->y, &p->Y, &zi3); r->inf = 0;                                        \
  }                                                                                                      \
  static int PT##_eq(const PT* p, const PT* q) {                                                         \
    int pi = PT##_is_inf(p), qi = PT##_is_inf(q);                                                        \
    if (pi || qi) return pi && qi;                                                                       \
    F Z1Z1, Z2Z2, a, b;                                                                                  \
    SQR(&Z1Z1, &p->Z); SQR(&Z2Z2, &q->Z);                                                                \
    MUL(&a, &p->X, &Z2Z2); MUL(&b, &q->X, &Z1Z1);                                                        \
    if (!EQ(&a, &b)) return 0;                                                                           \
    MUL(&a, &p->Y, &q->Z); MUL(&a, &a, &Z2Z2); MUL(&b, &q->Y, &p->Z); MUL(&b, &b, &Z1Z1);               \
    return EQ(&a, &b);                                                                                   \
  }                                                                                                      \
  /* [e] P, e a little-endian limb array of n limbs */                                                  \
  static void PT##_mul(PT* r, const PT* p, const u64* e, int n) {                                       \
    PT acc;                                                                                              \
    PT##_inf(&acc);                                                                                      \
    for (int i = mp_bits(e, n) - 1; i >= 0; --i) {                                                       \
      PT##_dbl(&acc, &acc);                                                                              \
      if (mp_bit(e, i)) PT##_add(&acc, &acc, p);                                                         \
    }                                                                                                    \
    *r = acc;                                                                                            \
  }

static void fp_dbl_(fp* r, const fp* a) { fp_add(r, a, a); }
DEFINE_CURVE(g1j, g1a, fp, fp_add, fp_sub, fp_mul, fp_sqr, fp_dbl_, fp_is_zero, fp_inv, FP_ONE, FP_ZERO, fp_eq, fp_neg)
DEFINE_CURVE(g2j, g2a, fp2, fp2_add, fp2_sub, fp2_mul, fp2_sqr, fp2_dbl, fp2_is_zero, fp2_inv, FP2_ONE, FP2_ZERO,
             fp2_eq, fp2_neg)

static fp FP_B1;     /* 4 */
static fp2 FP2_B2;   /* 4 (1 + u) */
static g1a G1_GEN;
static fp INV_TWO;

static void g2_psi(g2j* r, const g2j* p) {
  fp2 t;
  fp2_conj(&t, &p->X); fp2_mul(&r->X, &t, &PSI_CX);
  fp2_conj(&t, &p->Y); fp2_mul(&r->Y, &t, &PSI_CY);
  fp2_conj(&r->Z, &p->Z);
}
static void g2_mul_x(g2j* r, const g2j* p) { /* [x] P, x = -X_ABS */
  u64 e[1] = {X_ABS};
  g2j t;
  g2j_mul(&t, p, e, 1);
  g2j_neg(r, &t);
}
/* P in G2 <=> psi(P) == [x] P (Scott, "A note on group membership tests") */
static int g2_in_subgroup(const g2j* p) {
  if (g2j_is_inf(p)) return 1;
  g2j a, b;
  g2_psi(&a, p);
  g2_mul_x(&b, p);
  return g2j_eq(&a, &b);
}
/* P in G1 <=> [r] P == O */
static int g1_in_subgroup(const g1j* p) {
  g1j t;
  g1j_mul(&t, p, R_MOD, NR);
  return g1j_is_inf(&t);
}

/* ===================================================================== */
/* ZCash serialisation                                                    */
/* ===================================================================== */
enum { ST_OK = 0, ST_IDENTITY = 1, ST_ERR_FLAGS = -1, ST_ERR_FIELD = -2, ST_ERR_CURVE = -3, ST_ERR_SUBGROUP = -4 };

static int g1_decompress(g1a* out, const uint8_t* b) {
  int c = (b[0] >> 7) & 1, inf = (b[0] >> 6) & 1, s = (b[0] >> 5) & 1;
  if (!c) return ST_ERR_FLAGS;
  uint8_t xb[48];
  memcpy(xb, b, 48);
  xb[0] &= 0x1f;
  u64 x[NP];
  be48_to_limbs(x, xb);
  if (inf) {
    u64 o = 0;
    for (int i = 0; i < NP; ++i) o |= x[i];
    if (s || o) return ST_ERR_FLAGS;
    out->inf = 1;
    return ST_IDENTITY;
  }
  if (mp_cmp(x, P_MOD, NP) >= 0) return ST_ERR_FIELD;
  fp X, y2, y, t;
  fp_to_mont(&X, x);
  fp_sqr(&y2, &X);
  fp_mul(&y2, &y2, &X);
  fp_add(&y2, &y2, &FP_B1);
  fp_pow(&y, &y2, E_SQRT);
  fp_sqr(&t, &y);
  if (!fp_eq(&t, &y2)) return ST_ERR_CURVE;
  if (fp_lex_largest(&y) != s) fp_neg(&y, &y);
  out->x = X;
  out->y = y;
  out->inf = 0;
  g1j j;
  g1j_from_aff(&j, out);
  if (!g1_in_subgroup(&j)) return ST_ERR_SUBGROUP;
  return ST_OK;
}
static int g2_decompress(g2a* out, const uint8_t* b) {
  int c = (b[0] >> 7) & 1, inf = (b[0] >> 6) & 1, s = (b[0] >> 5) & 1;
  if (!c) return ST_ERR_FLAGS;
  uint8_t hb[48];
  memcpy(hb, b, 48);
  hb[0] &= 0x1f;
  u64 x1[NP], x0[NP];
  be48_to_limbs(x1, hb);
  be48_to_limbs(x0, b + 48);
  if (inf) {
    u64 o = 0;
    for (int i = 0; i < NP; ++i) o |= x0[i] | x1[i];
    if (s || o) return ST_ERR_FLAGS;
    out->inf = 1;
    return ST_IDENTITY;
  }
  if (mp_cmp(x0, P_MOD, NP) >= 0 || mp_cmp(x1, P_MOD, NP) >= 0) return ST_ERR_FIELD;
  fp2 X, y2, y;
  fp_to_mont(&X.c0, x0);
  fp_to_mont(&X.c1, x1);
  fp2_sqr(&y2, &X);
  fp2_mul(&y2, &y2, &X);
  fp2_add(&y2, &y2, &FP2_B2);
  if (!fp2_sqrt(&y, &y2)) return ST_ERR_CURVE;
  if (fp2_lex_largest(&y) != s) fp2_neg(&y, &y);
  out->x = X;
  out->y = y;
  out->inf = 0;
  g2j j;
  g2j_from_aff(&j, out);
  if (!g2_in_subgroup(&j)) return ST_ERR_SUBGROUP;
  return ST_OK;
}
static void g2_compress(uint8_t* out, const g2a* a) {
  if (a->inf) {
    memset(out, 0, 96);
    out[0] = 0xc0;
    return;
  }
  u64 c0[NP], c1[NP];
  fp_from_mont(c0, &a->x.c0);
  fp_from_mont(c1, &a->x.c1);
  limbs_to_be48(out, c1);
  limbs_to_be48(out + 48, c0);
  out[0] |= 0x80;
  if (fp2_lex_largest(&a->y)) out[0] |= 0x20;
}
static void g1_compress(uint8_t* out, const g1a* a) {
  if (a->inf) {
    memset(out, 0, 48);
    out[0] = 0xc0;
    return;
  }
  u64 c0[NP];
  fp_from_mont(c0, &a->x);
  limbs_to_be48(out, c0);
  out[0] |= 0x80;
  if (fp_lex_largest(&a->y)) out[0] |= 0x20;
}

/* ===================================================================== */
/* SHA-256 and hash_to_G2 (RFC 9380, BLS12381G2_XMD:SHA-256_SSWU_RO_)      */
/* ===================================================================== */
typedef struct { uint32_t h[8]; uint8_t buf[64]; uint32_t nbuf; u64 total; } sha256_ctx;
static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98, 0x12835b01,
    0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc,
    0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147,
    0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08,
    0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208,
    0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static void sha256_compress(uint32_t* h, const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t t1 = hh + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + w[i];
    uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha256_init(sha256_ctx* s) {
  static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(s->h, iv, sizeof(iv));
  s->nbuf = 0;
  s->total = 0;
}
static void sha256_update(sha256_ctx* s, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    s->buf[s->nbuf++] = p[i];
    if (s->nbuf == 64) {
      sha256_compress(s->h, s->buf);
      s->nbuf = 0;
    }
  }
  s->total += n;
}
static void sha256_final(sha256_ctx* s, uint8_t* out) {
  u64 bits = s->total * 8;
  uint8_t one = 0x80, zero = 0;
  sha256_update(s, &one, 1);
  while (s->nbuf != 56) sha256_update(s, &zero, 1);
  uint8_t len[8];
  for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha256_update(s, len, 8);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)(s->h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(s->h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(s->h[i] >> 8);
    out[4 * i + 3] = (uint8_t)s->h[i];
  }
}

static const char DST_POP[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";

static void expand_message_xmd(uint8_t* out, size_t len_out, const uint8_t* msg, size_t msg_len) {
  const size_t dlen = sizeof(DST_POP) - 1;
  uint8_t dst_prime_len = (uint8_t)dlen;
  uint8_t zpad[64] = {0};
  uint8_t lib[3] = {(uint8_t)(len_out >> 8), (uint8_t)len_out, 0};
  uint8_t b0[32], bi[32], tmp[32];
  sha256_ctx s;
  sha256_init(&s);
  sha256_update(&s, zpad, 64);
  sha256_update(&s, msg, msg_len);
  sha256_update(&s, lib, 3);
  sha256_update(&s, (const uint8_t*)DST_POP, dlen);
  sha256_update(&s, &dst_prime_len, 1);
  sha256_final(&s, b0);
  size_t ell = (len_out + 31) / 32;
  for (size_t i = 1; i <= ell; ++i) {
    for (int k = 0; k < 32; ++k) tmp[k] = (uint8_t)(i == 1 ? b0[k] : (b0[k] ^ bi[k]));
    uint8_t ib = (uint8_t)i;
    sha256_init(&s);
    if (i == 1) sha256_update(&s, b0, 32);
    else sha256_update(&s, tmp, 32);
    sha256_update(&s, &ib, 1);
    sha256_update(&s, (const uint8_t*)DST_POP, dlen);
    sha256_update(&s, &dst_prime_len, 1);
    sha256_final(&s, bi);
    size_t n = len_out - 32 * (i - 1) < 32 ? len_out - 32 * (i - 1) : 32;
    memcpy(out + 32 * (i - 1), bi, n);
  }
}

/* 64 big-endian bytes mod p (Montgomery form) */
static void fp_from_be64(fp* r, const uint8_t* b) {
  uint8_t hi48[48] = {0}, lo48[48] = {0};
  memcpy(hi48 + 16, b, 32);
  memcpy(lo48 + 16, b + 32, 32);
  u64 hi[NP], lo[NP];
  be48_to_limbs(hi, hi48);
  be48_to_limbs(lo, lo48);
  fp H, L, T;
  fp_to_mont(&H, hi);
  fp_to_mont(&L, lo);
  u64 two256[NP] = {0, 0, 0, 0, 1, 0};
  fp_to_mont(&T, two256);
  fp_mul(&H, &H, &T);
  fp_add(r, &H, &L);
}

static fp2 SSWU_A, SSWU_B, SSWU_Z, ISO_K[4][4];
static const char* ISO_HEX[15][2] = {
    /* (1, 0..3) */
    {"5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6",
     "5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6"},
    {"0", "11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A"},
    {"11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E",
     "8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D"},
    {"171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1", "0"},
    /* (2, 0..1) */
    {"0", "1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63"},
    {"C", "1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F"},
    /* (3, 0..3) */
    {"1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706",
     "1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706"},
    {"0", "5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE"},
    {"11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C",
     "8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F"},
    {"124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10", "0"},
    /* (4, 0..2) */
    {"1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB",
     "1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB"},
    {"0", "1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3"},
    {"12", "1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99"},
    {NULL, NULL},
    {NULL, NULL}};

static void hex_to_limbs(u64* r, const char* h) {
  memset(r, 0, 8 * NP);
  size_t n = strlen(h);
  for (size_t i = 0; i < n; ++i) {
    char c = h[n - 1 - i];
    u64 v = (c >= '0' && c <= '9') ? (u64)(c - '0') : (c >= 'A' && c <= 'F') ? (u64)(c - 'A' + 10) : (u64)(c - 'a' + 10);
    r[i / 16] |= v << (4 * (i % 16));
  }
}
static void fp2_from_hex(fp2* r, const char* h0, const char* h1) {
  u64 a[NP], b[NP];
  hex_to_limbs(a, h0);
  hex_to_limbs(b, h1);
  fp_to_mont(&r->c0, a);
  fp_to_mont(&r->c1, b);
}

/* simplified SWU on E2': y^2 = x^3 + A' x + B' (reference form of RFC 9380 6.6.2) */
static void sswu(fp2* xo, fp2* yo, const fp2* u) {
  fp2 u2, zu2, den, x1, gx1, t, x, y;
  fp2_sqr(&u2, u);
  fp2_mul(&zu2, &SSWU_Z, &u2);
  fp2_sqr(&den, &zu2);
  fp2_add(&den, &den, &zu2);
  if (fp2_is_zero(&den)) {
    fp2_mul(&t, &SSWU_Z, &SSWU_A);
    fp2_inv(&t, &t);
    fp2_mul(&x1, &SSWU_B, &t);
  } else {
    fp2 nb, ai;
    fp2_neg(&nb, &SSWU_B);
    fp2_inv(&ai, &SSWU_A);
    fp2_mul(&nb, &nb, &ai);
    fp2_inv(&t, &den);
    fp2_add(&t, &t, &FP2_ONE);
    fp2_mul(&x1, &nb, &t);
  }
  fp2_sqr(&gx1, &x1);
  fp2_mul(&gx1, &gx1, &x1);
  fp2_mul(&t, &SSWU_A, &x1);
  fp2_add(&gx1, &gx1, &t);
  fp2_add(&gx1, &gx1, &SSWU_B);
  if (fp2_is_square(&gx1)) {
    x = x1;
    fp2_sqrt(&y, &gx1);
  } else {
    fp2 gx2;
    fp2_mul(&x, &zu2, &x1);
    fp2_sqr(&gx2, &x);
    fp2_mul(&gx2, &gx2, &x);
    fp2_mul(&t, &SSWU_A, &x);
    fp2_add(&gx2, &gx2, &t);
    fp2_add(&gx2, &gx2, &SSWU_B);
    fp2_sqrt(&y, &gx2);
  }
  if (fp2_sgn0(u) != fp2_sgn0(&y)) fp2_neg(&y, &y);
  *xo = x;
  *yo = y;
}
static void poly_eval(fp2* r, const fp2* coeffs, int n, const fp2* x) { /* Horner, coeffs[0] constant */
  fp2 acc = coeffs[n - 1];
  for (int i = n - 2; i >= 0; --i) {
    fp2_mul(&acc, &acc, x);
    fp2_add(&acc, &acc, &coeffs[i]);
  }
  *r = acc;
}
static void iso3(g2a* out, const fp2* xp, const fp2* yp) {
  fp2 xn, xd, yn, yd, c[4], t;
  poly_eval(&xn, ISO_K[0], 4, xp);
  c[0] = ISO_K[1][0]; c[1] = ISO_K[1][1]; c[2] = FP2_ONE;
  poly_eval(&xd, c, 3, xp);
  poly_eval(&yn, ISO_K[2], 4, xp);
  c[0] = ISO_K[3][0]; c[1] = ISO_K[3][1]; c[2] = ISO_K[3][2]; c[3] = FP2_ONE;
  poly_eval(&yd, c, 4, xp);
  if (fp2_is_zero(&xd) || fp2_is_zero(&yd)) {
    out->inf = 1;
    return;
  }
  fp2_inv(&t, &xd);
  fp2_mul(&out->x, &xn, &t);
  fp2_inv(&t, &yd);
  fp2_mul(&t, &yn, &t);
  fp2_mul(&out->y, yp, &t);
  out->inf = 0;
}
/* Budroni-Pintore (RFC 9380 G.3): h(P) = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P) */
static void g2_clear_cofactor(g2j* r, const g2j* p) {
  g2j t1, t2, t3, u;
  g2_mul_x(&t1, p);             /* [x]P */
  g2_psi(&t2, p);               /* psi(P) */
  g2j_dbl(&t3, p);
  g2_psi(&t3, &t3);
  g2_psi(&t3, &t3);             /* psi^2(2P) */
  g2j_neg(&u, &t2);
  g2j_add(&t3, &t3, &u);        /* psi^2(2P) - psi(P) */
  g2j_add(&t2, &t1, &t2);       /* [x]P + psi(P) */
  g2_mul_x(&t2, &t2);           /* [x^2]P + [x]psi(P) */
  g2j_add(&t3, &t3, &t2);
  g2j_neg(&u, &t1);
  g2j_add(&t3, &t3, &u);
  g2j_neg(&u, p);
  g2j_add(r, &t3, &u);
}
static void hash_to_g2(g2a* out, const uint8_t* msg, size_t len) {
  uint8_t uni[256];
  expand_message_xmd(uni, 256, msg, len);
  fp2 u0, u1, x, y;
  fp_from_be64(&u0.c0, uni);
  fp_from_be64(&u0.c1, uni + 64);
  fp_from_be64(&u1.c0, uni + 128);
  fp_from_be64(&u1.c1, uni + 192);
  g2a q0, q1;
  sswu(&x, &y, &u0);
  iso3(&q0, &x, &y);
  sswu(&x, &y, &u1);
  iso3(&q1, &x, &y);
  g2j j0, j1, s;
  g2j_from_aff(&j0, &q0);
  g2j_from_aff(&j1, &q1);
  g2j_add(&s, &j0, &j1);
  g2_clear_cofactor(&s, &s);
  g2j_to_aff(out, &s);
}

/* ===================================================================== */
/* Pairing: projective Miller loop (M-type twist) + final exponentiation  */
/* ===================================================================== */
typedef struct { fp2 X, Y, Z; } g2p; /* homogeneous projective */
static fp2 TWIST_B3;                  /* 3 b' */

static void miller_dbl(g2p* R, fp2* c0, fp2* c1, fp2* c2) {
  fp2 a, b, c, e, f, g, h, i, j, es, t;
  fp2_mul(&a, &R->X, &R->Y);
  fp2_mul_fp(&a, &a, &INV_TWO);
  fp2_sqr(&b, &R->Y);
  fp2_sqr(&c, &R->Z);
  fp2_mul(&e, &TWIST_B3, &c);
  fp2_dbl(&f, &e);
  fp2_add(&f, &f, &e);
  fp2_add(&g, &b, &f);
  fp2_mul_fp(&g, &g, &INV_TWO);
  fp2_add(&h, &R->Y, &R->Z);
  fp2_sqr(&h, &h);
  fp2_add(&t, &b, &c);
  fp2_sub(&h, &h, &t);
  fp2_sub(&i, &e, &b);
  fp2_sqr(&j, &R->X);
  fp2_sqr(&es, &e);
  fp2_sub(&t, &b, &f);
  fp2_mul(&R->X, &a, &t);
  fp2_sqr(&R->Y, &g);
  fp2_dbl(&t, &es);
  fp2_add(&t, &t, &es);
  fp2_sub(&R->Y, &R->Y, &t);
  fp2_mul(&R->Z, &b, &h);
  *c0 = i;
  fp2_dbl(c1, &j);
  fp2_add(c1, c1, &j);
  fp2_neg(c2, &h);
}
/* R <- R + Q (Q affine); line through R and Q */
static void miller_add(g2p* R, const g2a* Q, fp2* c0, fp2* c1, fp2* c2) {
  fp2 theta, lambda, c, d, e, f, g, h, t, Y0 = R->Y;
  fp2_mul(&t, &Q->y, &R->Z);
  fp2_sub(&theta, &R->Y, &t);
  fp2_mul(&t, &Q->x, &R->Z);
  fp2_sub(&lambda, &R->X, &t);
  fp2_sqr(&c, &theta);
  fp2_sqr(&d, &lambda);
  fp2_mul(&e, &lambda, &d);
  fp2_mul(&f, &R->Z, &c);
  fp2_mul(&g, &R->X, &d);
  fp2_add(&h, &e, &f);
  fp2_dbl(&t, &g);
  fp2_sub(&h, &h, &t);
  fp2_mul(&R->X, &lambda, &h);
  fp2_sub(&t, &g, &h);
  fp2_mul(&R->Y, &theta, &t);
  fp2_mul(&t, &e, &Y0);
  fp2_sub(&R->Y, &R->Y, &t);
  fp2_mul(&R->Z, &R->Z, &e);
  fp2 j, u;
  fp2_mul(&j, &theta, &Q->x);
  fp2_mul(&u, &lambda, &Q->y);
  fp2_sub(c0, &j, &u);
  fp2_neg(c1, &theta);
  *c2 = lambda;
}
static void ell(fp12* f, const fp2* c0, const fp2* c1, const fp2* c2, const g1a* P) {
  fp2 a = *c1, b = *c2;
  fp2_mul_fp(&a, &a, &P->x);
  fp2_mul_fp(&b, &b, &P->y);
  fp12_mul_by_014(f, c0, &a, &b);
}
/* prod_k f_{|x|, Q_k}(P_k), conjugated (x < 0); every point non-infinity */
static void miller_loop(fp12* out, const g1a* P, const g2a* Q, int n) {
  g2p R[2];
  for (int k = 0; k < n; ++k) {
    R[k].X = Q[k].x;
    R[k].Y = Q[k].y;
    R[k].Z = FP2_ONE;
  }
  fp12 f = FP12_ONE;
  fp2 c0, c1, c2;
  for (int i = 62; i >= 0; --i) {
    fp12_sqr(&f, &f);
    for (int k = 0; k < n; ++k) {
      miller_dbl(&R[k], &c0, &c1, &c2);
      ell(&f, &c0, &c1, &c2, &P[k]);
    }
    if ((X_ABS >> i) & 1) {
      for (int k = 0; k < n; ++k) {
        miller_add(&R[k], &Q[k], &c0, &c1, &c2);
        ell(&f, &c0, &c1, &c2, &P[k]);
      }
    }
  }
  fp12_conj(out, &f);
}
static void cyc_pow_x(fp12* r, const fp12* a) { /* a^x, x < 0, a cyclotomic */
  fp12 acc = *a;
  for (int i = 62; i >= 0; --i) {
    fp12_cyc_sqr(&acc, &acc);
    if ((X_ABS >> i) & 1) fp12_mul(&acc, &acc, a);
  }
  fp12_conj(r, &acc);
}
/* f^(3 (p^12 - 1) / r): easy part, then (x-1)^2 (x+p) (x^2+p^2-1) + 3 */
static void final_exp(fp12* r, const fp12* f_in) {
  fp12 f, t, a, b, c, u;
  fp12_conj(&t, f_in);
  fp12_inv(&u, f_in);
  fp12_mul(&f, &t, &u);
  fp12_frob(&t, &f);
  fp12_frob(&t, &t);
  fp12_mul(&f, &t, &f);
  cyc_pow_x(&t, &f);
  fp12_conj(&u, &f);
  fp12_mul(&t, &t, &u);        /* f^(x-1) */
  cyc_pow_x(&a, &t);
  fp12_conj(&u, &t);
  fp12_mul(&a, &a, &u);        /* f^((x-1)^2) */
  cyc_pow_x(&b, &a);
  fp12_frob(&u, &a);
  fp12_mul(&b, &b, &u);        /* a^(x+p) */
  cyc_pow_x(&c, &b);
  cyc_pow_x(&c, &c);
  fp12_frob(&u, &b);
  fp12_frob(&u, &u);
  fp12_mul(&c, &c, &u);
  fp12_conj(&u, &b);
  fp12_mul(&c, &c, &u);        /* b^(x^2+p^2-1) */
  fp12_cyc_sqr(&u, &f);
  fp12_mul(&u, &u, &f);        /* f^3 */
  fp12_mul(r, &c, &u);
}

/* ===================================================================== */
/* Fr and Lagrange recombination (kryptology CombineSignatures semantics)  */
/* ===================================================================== */
static u64 R_MINV, E_R_MINUS_2[NR];
static u64 FR_ONE[NR], FR_R2[NR];
static void fr_mul(u64* r, const u64* a, const u64* b) { mont_mul(r, a, b, R_MOD, R_MINV, NR); }
static void fr_from_u64(u64* r, u64 v) {
  u64 t[NR];
  mp_small(t, v, NR);
  fr_mul(r, t, FR_R2);
}
static void fr_sub(u64* r, const u64* a, const u64* b) {
  if (mp_sub(r, a, b, NR)) mp_add(r, r, R_MOD, NR);
}
static void fr_inv(u64* r, const u64* a) {
  u64 acc[NR];
  memcpy(acc, FR_ONE, sizeof(acc));
  for (int i = mp_bits(E_R_MINUS_2, NR) - 1; i >= 0; --i) {
    fr_mul(acc, acc, acc);
    if (mp_bit(E_R_MINUS_2, i)) fr_mul(acc, acc, a);
  }
  memcpy(r, acc, sizeof(acc));
}
static void fr_to_plain(u64* r, const u64* a) {
  u64 one[NR];
  mp_small(one, 1, NR);
  fr_mul(r, a, one);
}
/* lambda_i(0) = prod_{j != i} x_j / (x_j - x_i); 0 on duplicate identifiers */
static int lagrange(u64* lam_plain, const uint8_t* ids, int k, int i) {
  u64 num[NR], den[NR], xi[NR], xj[NR], d[NR];
  memcpy(num, FR_ONE, sizeof(num));
  memcpy(den, FR_ONE, sizeof(den));
  fr_from_u64(xi, ids[i]);
  for (int j = 0; j < k; ++j) {
    if (j == i) continue;
    if (ids[j] == ids[i]) return 0;
    fr_from_u64(xj, ids[j]);
    fr_mul(num, num, xj);
    fr_sub(d, xj, xi);
    fr_mul(den, den, d);
  }
  fr_inv(den, den);
  fr_mul(num, num, den);
  fr_to_plain(lam_plain, num);
  return 1;
}

/* ===================================================================== */
/* init                                                                   */
/* ===================================================================== */
static u64 newton_minv(u64 m0) {
  u64 inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - m0 * inv;
  return (u64)0 - inv;
}
/* 2^k mod m as plain limbs, by doubling */
static void pow2_mod(u64* r, int k, const u64* m, int n) {
  mp_small(r, 1, n);
  for (int i = 0; i < k; ++i) {
    u64 c = mp_add(r, r, r, n);
    u64 d[NP];
    u64 br = mp_sub(d, r, m, n);
    if (c || !br) memcpy(r, d, 8 * n);
  }
}
static int g_inited = 0;
static pthread_mutex_t g_init_mu = PTHREAD_MUTEX_INITIALIZER;

int orc_init(void) {
  pthread_mutex_lock(&g_init_mu);
  if (g_inited) {
    pthread_mutex_unlock(&g_init_mu);
    return 0;
  }
  P_MINV = newton_minv(P_MOD[0]);
  R_MINV = newton_minv(R_MOD[0]);
  memset(&FP_ZERO, 0, sizeof(FP_ZERO));
  pow2_mod(FP_ONE.v, 384, P_MOD, NP);
  pow2_mod(FP_R2.v, 768, P_MOD, NP);
  pow2_mod(FR_ONE, 256, R_MOD, NR);
  pow2_mod(FR_R2, 512, R_MOD, NR);
  u64 two[NP], t[NP];
  mp_small(two, 2, NP);
  mp_sub(E_P_MINUS_2, P_MOD, two, NP);
  mp_small(t, 1, NP);
  mp_add(t, P_MOD, t, NP);
  mp_shr(E_SQRT, t, NP, 2);                 /* (p + 1) / 4 */
  mp_small(t, 3, NP);
  mp_sub(t, P_MOD, t, NP);
  mp_shr(E_PM3D4, t, NP, 2);                /* (p - 3) / 4 */
  mp_small(t, 1, NP);
  mp_sub(t, P_MOD, t, NP);
  mp_shr(E_PM1D2, t, NP, 1);                /* (p - 1) / 2 */
  u64 two_r[NR];
  mp_small(two_r, 2, NR);
  mp_sub(E_R_MINUS_2, R_MOD, two_r, NR);
  FP2_ZERO.c0 = FP_ZERO;
  FP2_ZERO.c1 = FP_ZERO;
  FP2_ONE.c0 = FP_ONE;
  FP2_ONE.c1 = FP_ZERO;
  memset(&FP12_ONE, 0, sizeof(FP12_ONE));
  FP12_ONE.c0.c0 = FP2_ONE;
  fp_from_u64(&FP_B1, 4);
  FP2_B2.c0 = FP_B1;
  FP2_B2.c1 = FP_B1;
  fp2 three;
  fp_from_u64(&three.c0, 3);
  three.c1 = FP_ZERO;
  fp2_mul(&TWIST_B3, &three, &FP2_B2);
  fp_from_u64(&INV_TWO, 2);
  fp_inv(&INV_TWO, &INV_TWO);
  /* Frobenius and psi constants: gamma_k = xi^(k (p-1)/6); psi = 1/xi^((p-1)/3), 1/xi^((p-1)/2) */
  fp2 xi;
  xi.c0 = FP_ONE;
  xi.c1 = FP_ONE;
  u64 pm1[NP], e6[NP], ek[NP];
  mp_small(t, 1, NP);
  mp_sub(pm1, P_MOD, t, NP);
  mp_divsmall(e6, pm1, 6, NP);
  for (int k = 0; k < 6; ++k) {
    mp_mulsmall(ek, e6, (u64)k, NP);
    fp2_pow(&FROB_GAMMA[k], &xi, ek, NP);
  }
  mp_divsmall(ek, pm1, 3, NP);
  fp2_pow(&PSI_CX, &xi, ek, NP);
  fp2_inv(&PSI_CX, &PSI_CX);
  mp_divsmall(ek, pm1, 2, NP);
  fp2_pow(&PSI_CY, &xi, ek, NP);
  fp2_inv(&PSI_CY, &PSI_CY);
  /* SSWU and isogeny constants (RFC 9380 8.8.2, appendix E.3) */
  fp2_from_hex(&SSWU_A, "0", "F0");
  fp2_from_hex(&SSWU_B, "3F4", "3F4");
  u64 two_p[NP];
  mp_small(t, 2, NP);
  mp_sub(two_p, P_MOD, t, NP);
  mp_small(t, 1, NP);
  u64 one_p[NP];
  mp_sub(one_p, P_MOD, t, NP);
  fp_to_mont(&SSWU_Z.c0, two_p);            /* -2 */
  fp_to_mont(&SSWU_Z.c1, one_p);            /* -1 */
  int idx = 0;
  static const int counts[4] = {4, 2, 4, 3};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < counts[i]; ++j, ++idx) fp2_from_hex(&ISO_K[i][j], ISO_HEX[idx][0], ISO_HEX[idx][1]);
  /* G1 generator */
  u64 gx[NP], gy[NP];
  hex_to_limbs(gx, "17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB");
  hex_to_limbs(gy, "08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1");
  fp_to_mont(&G1_GEN.x, gx);
  fp_to_mont(&G1_GEN.y, gy);
  G1_GEN.inf = 0;
  g_inited = 1;
  pthread_mutex_unlock(&g_init_mu);
  return 0;
}

/* ===================================================================== */
/* exported API (statuses as include/tbls_gpu.h)                          */
/* ===================================================================== */
#define PS_INVALID 0
#define PS_VALID 1
#define PS_NOT_VERIFIED 2
#define PS_ERR_IDENTITY (-5)
#define PS_ERR_PUBKEY (-6)
#define DS_OK 0
#define DS_INSUFFICIENT (-20)
#define DS_INSUFFICIENT_VALID (-21)
#define DS_AGG_TOO_FEW (-22)
#define DS_AGG_DUPLICATE_ID (-23)
#define DS_AGG_IDENTITY (-24)
#define DS_DECODE (-25)
#define DS_NOT_AGGREGATED 1
#define OP_VERIFY 1
#define OP_AGGREGATE 2
#define OP_VERIFY_AGGREGATE 3

/* e(pk, H(m)) * e(-g1, sig) == 1 */
static int core_verify(const g1a* pk, const g2a* h, const g2a* sig) {
  if (pk->inf || sig->inf || h->inf) return 0;
  g1a P[2];
  g2a Q[2];
  P[0] = *pk;
  Q[0] = *h;
  P[1] = G1_GEN;
  fp_neg(&P[1].y, &P[1].y);
  Q[1] = *sig;
  fp12 f, e;
  miller_loop(&f, P, Q, 2);
  final_exp(&e, &f);
  return fp12_is_one(&e);
}

typedef struct {
  g1a pk;
  int32_t status; /* 0 valid, 1 identity, < 0 decode error */
} orc_pk;

void* orc_pk_table(const uint8_t* pk48, uint32_t n, int32_t* status) {
  orc_init();
  orc_pk* t = (orc_pk*)calloc(n ? n : 1, sizeof(orc_pk));
  if (!t) return NULL;
  for (uint32_t i = 0; i < n; ++i) {
    t[i].status = g1_decompress(&t[i].pk, pk48 + 48ull * i);
    if (status) status[i] = t[i].status;
  }
  return t;
}
void orc_pk_table_free(void* t) { free(t); }

/* field order as tbg_batch */
typedef struct {
  uint32_t op, n_duties, n_partials, n_msgs;
  const uint8_t* msgs;
  const uint32_t* msg_off;
  const uint32_t* duty_msg;
  const uint32_t* duty_first;
  const uint32_t* duty_threshold;
  const uint8_t* sigs;
  const uint8_t* identifiers;
  const uint32_t* pubkey_ids;
} orc_batch;

static void run_duty(const orc_batch* b, const orc_pk* pks, uint32_t n_pk, uint32_t d, int32_t* ps, int32_t* ds,
                     uint8_t* agg) {
  uint32_t first = b->duty_first[d], last = b->duty_first[d + 1], n = last - first;
  g2a* sig = (g2a*)calloc(n ? n : 1, sizeof(g2a));
  memset(agg + 96ull * d, 0, 96);
  int decode_err = 0, identity = 0;
  for (uint32_t j = 0; j < n; ++j) {
    int st = g2_decompress(&sig[j], b->sigs + 96ull * (first + j));
    if (st == ST_IDENTITY) st = PS_ERR_IDENTITY;
    ps[first + j] = st == ST_OK ? PS_NOT_VERIFIED : st;
    if (st == PS_ERR_IDENTITY) identity = 1;
    else if (st < 0) decode_err = 1;
  }
  if (b->op != OP_AGGREGATE) {
    g2a h;
    uint32_t m = b->duty_msg[d];
    hash_to_g2(&h, b->msgs + b->msg_off[m], b->msg_off[m + 1] - b->msg_off[m]);
    for (uint32_t j = 0; j < n; ++j) {
      if (ps[first + j] != PS_NOT_VERIFIED) continue;
      uint32_t pid = b->pubkey_ids[first + j];
      if (pid >= n_pk || pks[pid].status != ST_OK) {
        ps[first + j] = PS_ERR_PUBKEY;
        continue;
      }
      ps[first + j] = core_verify(&pks[pid].pk, &h, &sig[j]) ? PS_VALID : PS_INVALID;
    }
  }
  if (b->op == OP_VERIFY) {
    ds[d] = DS_NOT_AGGREGATED;
    free(sig);
    return;
  }
  int want = b->op == OP_VERIFY_AGGREGATE ? PS_VALID : PS_NOT_VERIFIED;
  int k = 0;
  for (uint32_t j = 0; j < n; ++j) k += ps[first + j] == want;
  if (b->op == OP_VERIFY_AGGREGATE) {
    uint32_t t = b->duty_threshold[d];
    if (n < t) { ds[d] = DS_INSUFFICIENT; free(sig); return; }
    if ((uint32_t)k < t) { ds[d] = DS_INSUFFICIENT_VALID; free(sig); return; }
  } else {
    if (decode_err) { ds[d] = DS_DECODE; free(sig); return; }
    if (identity) { ds[d] = DS_AGG_IDENTITY; free(sig); return; }
  }
  if (k < 2) { ds[d] = DS_AGG_TOO_FEW; free(sig); return; }
  uint8_t ids[256];
  g2a pts[256];
  int kk = 0;
  for (uint32_t j = 0; j < n; ++j)
    if (ps[first + j] == want) {
      ids[kk] = b->identifiers[first + j];
      pts[kk] = sig[j];
      ++kk;
    }
  g2j acc;
  g2j_inf(&acc);
  for (int i = 0; i < kk; ++i) {
    u64 lam[NR];
    if (!lagrange(lam, ids, kk, i)) { ds[d] = DS_AGG_DUPLICATE_ID; free(sig); return; }
    g2j p, q;
    g2j_from_aff(&p, &pts[i]);
    g2j_mul(&q, &p, lam, NR);
    g2j_add(&acc, &acc, &q);
  }
  g2a a;
  g2j_to_aff(&a, &acc);
  if (a.inf) { ds[d] = DS_AGG_IDENTITY; free(sig); return; }
  g2_compress(agg + 96ull * d, &a);
  ds[d] = DS_OK;
  free(sig);
}

typedef struct {
  const orc_batch* b;
  const orc_pk* pks;
  uint32_t n_pk;
  int32_t *ps, *ds;
  uint8_t* agg;
  uint32_t next;
  pthread_mutex_t mu;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    uint32_t d = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (d >= j->b->n_duties) return NULL;
    run_duty(j->b, j->pks, j->n_pk, d, j->ps, j->ds, j->agg);
  }
}

/* Run a batch on `threads` host threads (tbg_run semantics). */
int orc_run(const orc_batch* b, const void* pk_table, uint32_t n_pk, int threads, int32_t* ps, int32_t* ds,
            uint8_t* agg) {
  orc_init();
  if (!b || !ps || !ds || !agg) return -1;
  job_t j;
  j.b = b;
  j.pks = (const orc_pk*)pk_table;
  j.n_pk = n_pk;
  j.ps = ps;
  j.ds = ds;
  j.agg = agg;
  j.next = 0;
  pthread_mutex_init(&j.mu, NULL);
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, worker, &j);
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  pthread_mutex_destroy(&j.mu);
  return 0;
}

/* single-item helpers (tests, fixture cross-checks) */
int orc_verify(const uint8_t* pk48, const uint8_t* msg, uint32_t len, const uint8_t* sig96) {
  orc_init();
  g1a pk;
  g2a sig, h;
  int s = g1_decompress(&pk, pk48);
  if (s != ST_OK) return PS_ERR_PUBKEY;
  s = g2_decompress(&sig, sig96);
  if (s == ST_IDENTITY) return PS_ERR_IDENTITY;
  if (s != ST_OK) return s;
  hash_to_g2(&h, msg, len);
  return core_verify(&pk, &h, &sig) ? PS_VALID : PS_INVALID;
}
void orc_hash_to_g2(const uint8_t* msg, uint32_t len, uint8_t* out96) {
  orc_init();
  g2a h;
  hash_to_g2(&h, msg, len);
  g2_compress(out96, &h);
}
/* sk: 32 big-endian bytes (< r) */
static void sk_limbs(u64* e, const uint8_t* sk32) {
  for (int i = 0; i < NR; ++i) {
    u64 w = 0;
    for (int k = 0; k < 8; ++k) w = (w << 8) | sk32[(NR - 1 - i) * 8 + k];
    e[i] = w;
  }
}
void orc_sign(const uint8_t* sk32, const uint8_t* msg, uint32_t len, uint8_t* out96) {
  orc_init();
  g2a h, s;
  hash_to_g2(&h, msg, len);
  u64 e[NR];
  sk_limbs(e, sk32);
  g2j p, q;
  g2j_from_aff(&p, &h);
  g2j_mul(&q, &p, e, NR);
  g2j_to_aff(&s, &q);
  g2_compress(out96, &s);
}
void orc_sk_to_pk(const uint8_t* sk32, uint8_t* out48) {
  orc_init();
  u64 e[NR];
  sk_limbs(e, sk32);
  g1j p, q;
  g1a a;
  g1j_from_aff(&p, &G1_GEN);
  g1j_mul(&q, &p, e, NR);
  g1j_to_aff(&a, &q);
  g1_compress(out48, &a);
}
int orc_g2_decode_status(const uint8_t* sig96) {
  orc_init();
  g2a a;
  int s = g2_decompress(&a, sig96);
  return s == ST_IDENTITY ? PS_ERR_IDENTITY : s;
}
