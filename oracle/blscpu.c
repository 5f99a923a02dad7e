/* blscpu.c -- TEST INFRASTRUCTURE ONLY (see blscpu.h): CPU oracle + cpu_baseline of the BLS12-381
 * signature-set verification path.
 *
 * A restatement from the specifications (ZCash BLS12-381 encoding, RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_
 * with the Eth2 POP DST, optimal-ate pairing) of what @chainsafe/blst computes for the reference's
 * IBlsVerifier path, written for host CPUs: 6 x 64-bit limbs, Montgomery (R = 2^384, CIOS with unsigned
 * __int128 products), one shared-squaring multi-Miller loop per batch chunk (as blst's miller_loop_n), the
 * same final-exponentiation chain as the device (oracle/bls12_381.py final_exp), and the reference pool's
 * scheduling: calls split into <= 128-set jobs (multithread/index.ts:156), jobs packed into worker requests
 * of >= 128 sets (prepareWork, index.ts:386-401), batchable jobs verified in chunks of >= 16 jobs with a
 * per-job re-verification when a chunk fails or throws (worker.ts:17,32-108), verifySignatureSetsMaybeBatch
 * per chunk / job (maybeBatch.ts:16-39).  Checked against oracle/bls12_381.py and the reference KATs in
 * tests/test_cpu_oracle.py.
 */
#include "blscpu.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

typedef unsigned __int128 u128;

/* ============================================================================================ Fp */
typedef struct {
  uint64_t l[6];
} fp;

static const fp P = {{0xB9FEFFFFFFFFAAABull, 0x1EABFFFEB153FFFFull, 0x6730D2A0F6B0F624ull, 0x64774B84F38512BFull,
                      0x4B1BA7B6434BACD7ull, 0x1A0111EA397FE69Aull}};
static uint64_t N0;           /* -p^-1 mod 2^64 */
static fp R1, R2, R3;         /* R, R^2, R^3 mod p (plain) -- R1 is Montgomery one */
static __thread uint64_t g_count __attribute__((tls_model("initial-exec")));
#define COUNT() (g_count++)

static inline fp fp_zero(void) {
  fp r;
  memset(&r, 0, sizeof r);
  return r;
}
static inline int fp_is_zero(fp a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3] | a.l[4] | a.l[5]) == 0; }
static inline int fp_eq(fp a, fp b) { return memcmp(&a, &b, sizeof a) == 0; }

/* r = a - b over 6 limbs, returns borrow */
static inline uint64_t sub6(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
  return br;
}
static inline uint64_t add6(uint64_t* r, const uint64_t* a, const uint64_t* b) {
  u128 c = 0;
  for (int i = 0; i < 6; i++) {
    c += (u128)a[i] + b[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
static inline int geq6(const uint64_t* a, const uint64_t* b) {
  for (int i = 5; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 1;
}

static inline fp fp_add(fp a, fp b) {
  fp r, t;
  add6(r.l, a.l, b.l); /* < 2p < 2^382: no carry out */
  return sub6(t.l, r.l, P.l) ? r : t;
}
static inline fp fp_sub(fp a, fp b) {
  fp r, t;
  if (sub6(r.l, a.l, b.l)) {
    add6(t.l, r.l, P.l);
    return t;
  }
  return r;
}
static inline fp fp_neg(fp a) {
  if (fp_is_zero(a)) return a;
  fp r;
  sub6(r.l, P.l, a.l);
  return r;
}
static inline fp fp_dbl(fp a) { return fp_add(a, a); }

/* Montgomery product, CIOS, unrolled; operands < p.  p < 2^381 leaves 3 spare bits in the top limb, so the running
 * value t (< 2p) never needs a 7th word: each row is 6 products + 6 reduction products. */
#define MAC(t, a, b, c)                 \
  do {                                  \
    u128 _m = (u128)(a) * (b) + (t) + (c); \
    (t) = (uint64_t)_m;                 \
    (c) = (uint64_t)(_m >> 64);         \
  } while (0)
static fp fp_mul(fp a, fp b) {
  COUNT();
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
#pragma GCC unroll 6
  for (int i = 0; i < 6; i++) {
    const uint64_t bi = b.l[i];
    uint64_t c = 0;
    MAC(t0, a.l[0], bi, c);
    MAC(t1, a.l[1], bi, c);
    MAC(t2, a.l[2], bi, c);
    MAC(t3, a.l[3], bi, c);
    MAC(t4, a.l[4], bi, c);
    MAC(t5, a.l[5], bi, c);
    const uint64_t hi = c;
    const uint64_t m = t0 * N0;
    c = 0;
    uint64_t d = t0;
    MAC(d, m, P.l[0], c);
    MAC(t1, m, P.l[1], c);
    MAC(t2, m, P.l[2], c);
    MAC(t3, m, P.l[3], c);
    MAC(t4, m, P.l[4], c);
    MAC(t5, m, P.l[5], c);
    t0 = t1;
    t1 = t2;
    t2 = t3;
    t3 = t4;
    t4 = t5;
    t5 = hi + c;
  }
  fp r = {{t0, t1, t2, t3, t4, t5}}, s;
  return sub6(s.l, r.l, P.l) ? r : s;
}
static inline fp fp_sqr(fp a) { return fp_mul(a, a); }
static inline fp fp_to_mont(fp plain) { return fp_mul(plain, R2); }
static inline fp fp_from_mont(fp a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_mul(a, one);
}
static inline fp fp_one(void) { return R1; }
static inline fp fp_small(uint64_t v) {
  fp r = fp_zero();
  r.l[0] = v;
  return fp_to_mont(r);
}

/* exponentiation by a public little-endian 64-bit-word exponent, 4-bit fixed window */
static fp fp_pow(fp a, const uint64_t* e, int nwords) {
  fp tab[16];
  tab[0] = fp_one();
  for (int i = 1; i < 16; i++) tab[i] = fp_mul(tab[i - 1], a);
  fp r = fp_one();
  int started = 0;
  for (int w = nwords - 1; w >= 0; w--) {
    for (int k = 60; k >= 0; k -= 4) {
      unsigned d = (unsigned)(e[w] >> k) & 15u;
      if (started) {
        r = fp_sqr(fp_sqr(fp_sqr(fp_sqr(r))));
        if (d) r = fp_mul(r, tab[d]);
      } else if (d) {
        r = tab[d];
        started = 1;
      }
    }
  }
  return r;
}
static uint64_t E_PM2[6], E_P14[6], E_P34[6], E_PM1_2[6]; /* p-2, (p+1)/4, (p-3)/4, (p-1)/2 */
static fp HALF; /* 1/2 */
static inline fp fp_inv(fp a) { return fp_pow(a, E_PM2, 6); }
/* sqrt for p = 3 mod 4; returns 0 when a is not a square */
static int fp_sqrt(fp a, fp* out) {
  fp s = fp_pow(a, E_P14, 6);
  *out = s;
  return fp_eq(fp_sqr(s), a);
}
static int fp_is_square(fp a) {
  if (fp_is_zero(a)) return 1;
  return fp_eq(fp_pow(a, E_PM1_2, 6), fp_one());
}

/* big-endian 48 bytes -> plain value; returns 0 if >= p */
static int fp_from_be(const uint8_t* b, fp* out, uint8_t top_mask) {
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) {
      uint8_t byte = b[47 - 8 * i - k];
      if (8 * i + k == 47) byte &= top_mask;
      v |= (uint64_t)byte << (8 * k);
    }
    out->l[i] = v;
  }
  return !geq6(out->l, P.l);
}
static void fp_to_be(fp mont, uint8_t* b) {
  fp v = fp_from_mont(mont);
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) b[47 - 8 * i - k] = (uint8_t)(v.l[i] >> (8 * k));
}
/* canonical value > (p-1)/2 ("lexicographically largest") */
static int fp_lex_largest(fp mont) {
  fp v = fp_from_mont(mont), h;
  memcpy(h.l, E_PM1_2, sizeof h.l);
  return !geq6(h.l, v.l); /* v > (p-1)/2 */
}
static int fp_sgn0(fp mont) { return (int)(fp_from_mont(mont).l[0] & 1); }

/* ============================================================================================ Fp2 */
typedef struct {
  fp c0, c1;
} fp2;
static inline fp2 fp2_make(fp a, fp b) {
  fp2 r = {a, b};
  return r;
}
static inline fp2 fp2_zero(void) { return fp2_make(fp_zero(), fp_zero()); }
static inline fp2 fp2_one(void) { return fp2_make(fp_one(), fp_zero()); }
static inline fp2 fp2_add(fp2 a, fp2 b) { return fp2_make(fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)); }
static inline fp2 fp2_sub(fp2 a, fp2 b) { return fp2_make(fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)); }
static inline fp2 fp2_neg(fp2 a) { return fp2_make(fp_neg(a.c0), fp_neg(a.c1)); }
static inline fp2 fp2_dbl(fp2 a) { return fp2_add(a, a); }
static inline fp2 fp2_conj(fp2 a) { return fp2_make(a.c0, fp_neg(a.c1)); }
static inline int fp2_is_zero(fp2 a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
static inline int fp2_eq(fp2 a, fp2 b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
static fp2 fp2_mul(fp2 a, fp2 b) {
  fp t0 = fp_mul(a.c0, b.c0), t1 = fp_mul(a.c1, b.c1);
  fp t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return fp2_make(fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1));
}
static fp2 fp2_sqr(fp2 a) {
  fp c0 = fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1));
  fp c1 = fp_mul(fp_dbl(a.c0), a.c1);
  return fp2_make(c0, c1);
}
static inline fp2 fp2_mul_fp(fp2 a, fp s) { return fp2_make(fp_mul(a.c0, s), fp_mul(a.c1, s)); }
static inline fp2 fp2_mul_xi(fp2 a) { return fp2_make(fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)); } /* (1+u) a */
static inline fp fp2_norm(fp2 a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }
static fp2 fp2_inv(fp2 a) {
  fp ni = fp_inv(fp2_norm(a));
  return fp2_make(fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni)));
}
static fp2 fp2_pow(fp2 a, const uint64_t* e, int nwords) {
  fp2 r = fp2_one();
  for (int w = nwords - 1; w >= 0; w--)
    for (int k = 63; k >= 0; k--) {
      r = fp2_sqr(r);
      if ((e[w] >> k) & 1) r = fp2_mul(r, a);
    }
  return r;
}
/* sqrt in Fp2 through the norm (p = 3 mod 4), two Fp exponentiations by (p-3)/4; 0 if not a square.
 * Root sign unspecified (callers fix it). */
static int fp2_sqrt(fp2 a, fp2* out) {
  fp n = fp2_norm(a);
  fp s = fp_mul(n, fp_pow(n, E_P34, 6)); /* n^((p+1)/4) */
  if (!fp_eq(fp_sqr(s), n)) return 0;
  fp t = fp_mul(fp_add(a.c0, s), HALF);
  if (fp_is_zero(t)) t = fp_mul(fp_sub(a.c0, s), HALF);
  fp y = fp_pow(t, E_P34, 6); /* t^((p-3)/4): x0 = t y, 1/x0 = y when t is a square */
  fp x0 = fp_mul(t, y);
  fp2 r;
  if (fp_eq(fp_sqr(x0), t)) {
    r = fp2_make(x0, fp_mul(fp_mul(a.c1, y), HALF));
  } else { /* t non-residue: (a0 - s)/2 = -t' ... use sqrt(-t) u as the Fp part */
    r = fp2_make(fp_mul(fp_mul(a.c1, y), HALF), fp_neg(x0));
  }
  if (!fp2_eq(fp2_sqr(r), a)) return 0;
  *out = r;
  return 1;
}
static int fp2_sgn0(fp2 a) {
  int s0 = fp_sgn0(a.c0), z0 = fp_is_zero(a.c0), s1 = fp_sgn0(a.c1);
  return s0 | (z0 & s1);
}
static int fp2_lex_largest(fp2 y) { return fp_is_zero(y.c1) ? fp_lex_largest(y.c0) : fp_lex_largest(y.c1); }

/* ============================================================================================ Fp6/Fp12 */
typedef struct {
  fp2 c0, c1, c2;
} fp6;
typedef struct {
  fp6 c0, c1;
} fp12;
static inline fp6 fp6_make(fp2 a, fp2 b, fp2 c) {
  fp6 r = {a, b, c};
  return r;
}
static inline fp6 fp6_zero(void) { return fp6_make(fp2_zero(), fp2_zero(), fp2_zero()); }
static inline fp6 fp6_add(fp6 a, fp6 b) { return fp6_make(fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)); }
static inline fp6 fp6_sub(fp6 a, fp6 b) { return fp6_make(fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)); }
static inline fp6 fp6_neg(fp6 a) { return fp6_make(fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)); }
static inline fp6 fp6_mul_v(fp6 a) { return fp6_make(fp2_mul_xi(a.c2), a.c0, a.c1); }
static fp6 fp6_mul(fp6 a, fp6 b) {
  fp2 t0 = fp2_mul(a.c0, b.c0), t1 = fp2_mul(a.c1, b.c1), t2 = fp2_mul(a.c2, b.c2);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), fp2_add(t1, t2))));
  fp2 c1 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), fp2_add(t0, t1)), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), fp2_add(t0, t2)), t1);
  return fp6_make(c0, c1, c2);
}
static fp6 fp6_mul_by_01(fp6 x, fp2 l0, fp2 l1) {
  fp2 t0 = fp2_mul(x.c0, l0), t1 = fp2_mul(x.c1, l1);
  fp2 c0 = fp2_add(t0, fp2_mul_xi(fp2_mul(x.c2, l1)));
  fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add(x.c0, x.c1), fp2_add(l0, l1)), t0), t1);
  fp2 c2 = fp2_add(fp2_mul(x.c2, l0), t1);
  return fp6_make(c0, c1, c2);
}
static fp6 fp6_mul_by_1(fp6 x, fp2 l1) {
  return fp6_make(fp2_mul_xi(fp2_mul(x.c2, l1)), fp2_mul(x.c0, l1), fp2_mul(x.c1, l1));
}
static fp6 fp6_inv(fp6 a) {
  fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2 di = fp2_inv(d);
  return fp6_make(fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di));
}
static inline fp12 fp12_make(fp6 a, fp6 b) {
  fp12 r = {a, b};
  return r;
}
static inline fp12 fp12_one(void) { return fp12_make(fp6_make(fp2_one(), fp2_zero(), fp2_zero()), fp6_zero()); }
static fp12 fp12_mul(fp12 a, fp12 b) {
  fp6 t0 = fp6_mul(a.c0, b.c0), t1 = fp6_mul(a.c1, b.c1);
  fp6 c1 = fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), fp6_add(t0, t1));
  return fp12_make(fp6_add(t0, fp6_mul_v(t1)), c1);
}
static fp12 fp12_sqr(fp12 a) {
  fp6 t = fp6_mul(a.c0, a.c1);
  fp6 s = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  return fp12_make(fp6_sub(fp6_sub(s, t), fp6_mul_v(t)), fp6_add(t, t));
}
static inline fp12 fp12_conj(fp12 a) { return fp12_make(a.c0, fp6_neg(a.c1)); }
static fp12 fp12_inv(fp12 a) {
  fp6 t = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6 ti = fp6_inv(t);
  return fp12_make(fp6_mul(a.c0, ti), fp6_neg(fp6_mul(a.c1, ti)));
}
static fp12 fp12_mul_by_014(fp12 f, fp2 l0, fp2 l1, fp2 l4) {
  fp6 a0 = fp6_mul_by_01(f.c0, l0, l1), a1 = fp6_mul_by_1(f.c1, l4);
  fp6 s = fp6_mul_by_01(fp6_add(f.c0, f.c1), l0, fp2_add(l1, l4));
  return fp12_make(fp6_add(a0, fp6_mul_v(a1)), fp6_sub(fp6_sub(s, a0), a1));
}
static void fp4_sqr(fp2 a, fp2 b, fp2* c0, fp2* c1) {
  fp2 t0 = fp2_sqr(a), t1 = fp2_sqr(b);
  *c0 = fp2_add(fp2_mul_xi(t1), t0);
  *c1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}
static inline fp2 cyc_sub(fp2 t, fp2 z) { return fp2_add(fp2_dbl(fp2_sub(t, z)), t); }
static inline fp2 cyc_add(fp2 t, fp2 z) { return fp2_add(fp2_dbl(fp2_add(t, z)), t); }
/* Granger-Scott squaring in the cyclotomic subgroup */
static fp12 fp12_cyc_sqr(fp12 f) {
  fp2 t0, t1, t2, t3, u0, u1;
  fp12 r;
  fp4_sqr(f.c0.c0, f.c1.c1, &t0, &t1);
  r.c0.c0 = cyc_sub(t0, f.c0.c0);
  r.c1.c1 = cyc_add(t1, f.c1.c1);
  fp4_sqr(f.c1.c0, f.c0.c2, &u0, &u1);
  fp4_sqr(f.c0.c1, f.c1.c2, &t2, &t3);
  r.c0.c1 = cyc_sub(u0, f.c0.c1);
  r.c1.c2 = cyc_add(u1, f.c1.c2);
  r.c1.c0 = cyc_add(fp2_mul_xi(t3), f.c1.c0);
  r.c0.c2 = cyc_sub(t2, f.c0.c2);
  return r;
}
static fp2 GAMMA1[6], GAMMA2[6]; /* xi^(k (p-1)/6), xi^(k (p^2-1)/6) */
static fp12 fp12_frob(fp12 a, int e) {
  const fp2* g = e == 1 ? GAMMA1 : GAMMA2;
  fp2* c[6] = {&a.c0.c0, &a.c1.c0, &a.c0.c1, &a.c1.c1, &a.c0.c2, &a.c1.c2}; /* w^0 .. w^5 */
  for (int k = 0; k < 6; k++) {
    fp2 v = e == 1 ? fp2_conj(*c[k]) : *c[k];
    *c[k] = k ? fp2_mul(v, g[k]) : v;
  }
  return a;
}
static int fp12_is_one(fp12 a) {
  fp12 o = fp12_one();
  return memcmp(&a, &o, sizeof a) == 0;
}

/* ============================================================================================ curves */
static fp B1;         /* 4 */
static fp2 B2;        /* 4 (1 + u) */
static fp2 PSI_X, PSI_Y, PSI2_X, PSI2_Y;
static fp G1X, G1Y;
static const uint64_t Z_ABS = 0xD201000000010000ull;

#define DEFINE_JAC(G, F, PFX)                                                                             \
  typedef struct {                                                                                        \
    F x, y, z;                                                                                            \
  } G##j;                                                                                                 \
  typedef struct {                                                                                        \
    F x, y;                                                                                               \
    int inf;                                                                                              \
  } G##a;                                                                                                 \
  static inline G##j G##_inf(void) {                                                                      \
    G##j r = {PFX##_one(), PFX##_one(), PFX##_zero()};                                                    \
    return r;                                                                                             \
  }                                                                                                       \
  static inline int G##_is_inf(G##j p) { return PFX##_is_zero(p.z); }                                    \
  static inline G##j G##_from_aff(G##a a) {                                                               \
    if (a.inf) return G##_inf();                                                                          \
    G##j r = {a.x, a.y, PFX##_one()};                                                                     \
    return r;                                                                                             \
  }                                                                                                       \
  static G##j G##_dbl(G##j p) {                                                                           \
    F A = PFX##_sqr(p.x), B = PFX##_sqr(p.y), C = PFX##_sqr(B);                                           \
    F D = PFX##_dbl(PFX##_sub(PFX##_sub(PFX##_sqr(PFX##_add(p.x, B)), A), C));                            \
    F E = PFX##_add(PFX##_dbl(A), A), Fv = PFX##_sqr(E);                                                  \
    G##j r;                                                                                               \
    r.x = PFX##_sub(Fv, PFX##_dbl(D));                                                                    \
    r.y = PFX##_sub(PFX##_mul(E, PFX##_sub(D, r.x)), PFX##_dbl(PFX##_dbl(PFX##_dbl(C))));                 \
    r.z = PFX##_mul(PFX##_dbl(p.y), p.z);                                                                 \
    return r;                                                                                             \
  }                                                                                                       \
  static inline G##j G##_neg(G##j p) {                                                                    \
    p.y = PFX##_neg(p.y);                                                                                 \
    return p;                                                                                             \
  }                                                                                                       \
  static G##j G##_add(G##j p, G##j q) {                                                                   \
    if (G##_is_inf(p)) return q;                                                                          \
    if (G##_is_inf(q)) return p;                                                                          \
    F Z1Z1 = PFX##_sqr(p.z), Z2Z2 = PFX##_sqr(q.z);                                                       \
    F U1 = PFX##_mul(p.x, Z2Z2), U2 = PFX##_mul(q.x, Z1Z1);                                               \
    F S1 = PFX##_mul(p.y, PFX##_mul(q.z, Z2Z2)), S2 = PFX##_mul(q.y, PFX##_mul(p.z, Z1Z1));               \
    F H = PFX##_sub(U2, U1), rr = PFX##_dbl(PFX##_sub(S2, S1));                                           \
    if (PFX##_is_zero(H)) return PFX##_is_zero(rr) ? G##_dbl(p) : G##_inf();                              \
    F I = PFX##_sqr(PFX##_dbl(H)), J = PFX##_mul(H, I), V = PFX##_mul(U1, I);                             \
    G##j r;                                                                                               \
    r.x = PFX##_sub(PFX##_sub(PFX##_sqr(rr), J), PFX##_dbl(V));                                           \
    r.y = PFX##_sub(PFX##_mul(rr, PFX##_sub(V, r.x)), PFX##_dbl(PFX##_mul(S1, J)));                       \
    r.z = PFX##_mul(PFX##_sub(PFX##_sub(PFX##_sqr(PFX##_add(p.z, q.z)), Z1Z1), Z2Z2), H);                 \
    return r;                                                                                             \
  }                                                                                                       \
  static G##j G##_add_aff(G##j p, G##a q) {                                                               \
    if (q.inf) return p;                                                                                  \
    if (G##_is_inf(p)) return G##_from_aff(q);                                                            \
    F Z1Z1 = PFX##_sqr(p.z), U2 = PFX##_mul(q.x, Z1Z1), S2 = PFX##_mul(q.y, PFX##_mul(p.z, Z1Z1));        \
    F H = PFX##_sub(U2, p.x), rr = PFX##_dbl(PFX##_sub(S2, p.y));                                         \
    if (PFX##_is_zero(H)) return PFX##_is_zero(rr) ? G##_dbl(p) : G##_inf();                              \
    F HH = PFX##_sqr(H), I = PFX##_dbl(PFX##_dbl(HH)), J = PFX##_mul(H, I), V = PFX##_mul(p.x, I);        \
    G##j r;                                                                                               \
    r.x = PFX##_sub(PFX##_sub(PFX##_sqr(rr), J), PFX##_dbl(V));                                           \
    r.y = PFX##_sub(PFX##_mul(rr, PFX##_sub(V, r.x)), PFX##_dbl(PFX##_mul(p.y, J)));                      \
    r.z = PFX##_sub(PFX##_sub(PFX##_sqr(PFX##_add(p.z, H)), Z1Z1), HH);                                   \
    return r;                                                                                             \
  }                                                                                                       \
  /* [k]P, k little-endian 64-bit words, 4-bit fixed window */                                            \
  static G##j G##_mul(G##j p, const uint64_t* k, int nwords) {                                            \
    G##j tab[16];                                                                                         \
    tab[0] = G##_inf();                                                                                   \
    tab[1] = p;                                                                                           \
    for (int i = 2; i < 16; i++) tab[i] = (i & 1) ? G##_add(tab[i - 1], p) : G##_dbl(tab[i / 2]);         \
    G##j r = G##_inf();                                                                                   \
    for (int w = nwords - 1; w >= 0; w--)                                                                 \
      for (int s = 60; s >= 0; s -= 4) {                                                                  \
        r = G##_dbl(G##_dbl(G##_dbl(G##_dbl(r))));                                                        \
        unsigned d = (unsigned)(k[w] >> s) & 15u;                                                         \
        if (d) r = G##_add(r, tab[d]);                                                                    \
      }                                                                                                   \
    return r;                                                                                             \
  }                                                                                                       \
  static G##j G##_mul_zabs(G##j p) {                                                                      \
    G##j r = p;                                                                                           \
    for (int i = 62; i >= 0; i--) {                                                                       \
      r = G##_dbl(r);                                                                                     \
      if ((Z_ABS >> i) & 1) r = G##_add(r, p);                                                            \
    }                                                                                                     \
    return r;                                                                                             \
  }                                                                                                       \
  static G##a G##_to_aff(G##j p) {                                                                        \
    G##a a;                                                                                               \
    if (G##_is_inf(p)) {                                                                                  \
      a.x = PFX##_zero();                                                                                 \
      a.y = PFX##_zero();                                                                                 \
      a.inf = 1;                                                                                          \
      return a;                                                                                           \
    }                                                                                                     \
    F zi = PFX##_inv(p.z), zi2 = PFX##_sqr(zi);                                                           \
    a.x = PFX##_mul(p.x, zi2);                                                                            \
    a.y = PFX##_mul(p.y, PFX##_mul(zi2, zi));                                                             \
    a.inf = 0;                                                                                            \
    return a;                                                                                             \
  }                                                                                                       \
  static int G##_eq(G##j p, G##j q) {                                                                     \
    int pi = G##_is_inf(p), qi = G##_is_inf(q);                                                           \
    if (pi || qi) return pi && qi;                                                                        \
    F Z1Z1 = PFX##_sqr(p.z), Z2Z2 = PFX##_sqr(q.z);                                                       \
    if (!PFX##_eq(PFX##_mul(p.x, Z2Z2), PFX##_mul(q.x, Z1Z1))) return 0;                                  \
    return PFX##_eq(PFX##_mul(p.y, PFX##_mul(q.z, Z2Z2)), PFX##_mul(q.y, PFX##_mul(p.z, Z1Z1)));          \
  }

DEFINE_JAC(g1, fp, fp)
DEFINE_JAC(g2, fp2, fp2)

static uint64_t R_ORDER[4] = {0xFFFFFFFF00000001ull, 0x53BDA402FFFE5BFEull, 0x3339D80809A1D805ull,
                              0x73EDA753299D7D48ull};

static g2j g2_psi(g2j p) {
  g2j r = {fp2_mul(fp2_conj(p.x), PSI_X), fp2_mul(fp2_conj(p.y), PSI_Y), fp2_conj(p.z)};
  return r;
}
static g2j g2_psi2(g2j p) {
  g2j r = {fp2_mul(p.x, PSI2_X), fp2_mul(p.y, PSI2_Y), p.z};
  return r;
}
/* psi(P) == [z]P (Scott, eprint 2021/1130) */
static int g2_in_group(g2a a) {
  if (a.inf) return 1;
  g2j P = g2_from_aff(a);
  return g2_eq(g2_psi(P), g2_neg(g2_mul_zabs(P)));
}
/* definitional [r]P == O (KeyValidate) */
static int g1_in_group(g1a a) {
  if (a.inf) return 1;
  return g1_is_inf(g1_mul(g1_from_aff(a), R_ORDER, 4));
}
static int g1_on_curve(g1a a) { return fp_eq(fp_sqr(a.y), fp_add(fp_mul(fp_sqr(a.x), a.x), B1)); }
static int g2_on_curve(g2a a) { return fp2_eq(fp2_sqr(a.y), fp2_add(fp2_mul(fp2_sqr(a.x), a.x), B2)); }

/* ============================================================================================ codecs */
enum {
  C_OK = BLSGPU_OK,
  C_BAD = BLSGPU_BAD_ENCODING,
  C_NOC = BLSGPU_POINT_NOT_ON_CURVE,
  C_NIG = BLSGPU_POINT_NOT_IN_GROUP,
  C_PKINF = BLSGPU_PK_IS_INFINITY,
  C_SIZE = BLSGPU_INVALID_SIZE,
  C_EAGG = BLSGPU_EMPTY_AGGREGATE,
  C_ESET = BLSGPU_EMPTY_SET
};

static int all_zero(const uint8_t* b, int n) {
  uint8_t o = 0;
  for (int i = 0; i < n; i++) o |= b[i];
  return o == 0;
}

/* G1: 96-byte uncompressed (blst_p1_deserialize) or 48-byte compressed (POINTonE1_Uncompress); no
 * subgroup check */
static int g1_decode(const uint8_t* b, uint32_t len, g1a* out) {
  memset(out, 0, sizeof *out);
  if (len != 48 && len != 96) return C_SIZE;
  uint8_t b0 = b[0];
  int compressed = (b0 & 0x80) != 0;
  if (compressed != (len == 48)) return C_BAD;
  if (b0 & 0x40) {
    if ((b0 & 0x3f) == 0 && all_zero(b + 1, (int)len - 1)) {
      out->inf = 1;
      return C_OK;
    }
    return C_BAD;
  }
  fp x, y;
  if (compressed) {
    if (!fp_from_be(b, &x, 0x1f)) return C_BAD;
    x = fp_to_mont(x);
    if (!fp_sqrt(fp_add(fp_mul(fp_sqr(x), x), B1), &y)) return C_NOC;
    if (fp_lex_largest(y) != ((b0 & 0x20) != 0)) y = fp_neg(y);
  } else {
    if (b0 & 0x20) return C_BAD;
    if (!fp_from_be(b, &x, 0xff) || !fp_from_be(b + 48, &y, 0xff)) return C_BAD;
    x = fp_to_mont(x);
    y = fp_to_mont(y);
    out->x = x;
    out->y = y;
    if (!g1_on_curve(*out)) return C_NOC;
  }
  out->x = x;
  out->y = y;
  return C_OK;
}
static void g1_encode96(g1a a, uint8_t* b) {
  if (a.inf) {
    memset(b, 0, 96);
    b[0] = 0x40;
    return;
  }
  fp_to_be(a.x, b);
  fp_to_be(a.y, b + 48);
}
static void g1_encode48(g1a a, uint8_t* b) {
  if (a.inf) {
    memset(b, 0, 48);
    b[0] = 0xc0;
    return;
  }
  fp_to_be(a.x, b);
  b[0] |= 0x80 | (fp_lex_largest(a.y) ? 0x20 : 0);
}

/* Signature.fromBytes(sig, affine, validate = true) */
static int sig_decode(const uint8_t* b, uint32_t len, g2a* out) {
  memset(out, 0, sizeof *out);
  if (len != 96 && len != 192) return C_SIZE;
  uint8_t b0 = b[0];
  int compressed = (b0 & 0x80) != 0;
  if (compressed != (len == 96)) return C_BAD;
  if (b0 & 0x40) {
    if ((b0 & 0x3f) == 0 && all_zero(b + 1, (int)len - 1)) {
      out->inf = 1;
      return C_OK;
    }
    return C_BAD;
  }
  fp x1, x0;
  int ok1 = fp_from_be(b, &x1, 0x1f), ok0 = fp_from_be(b + 48, &x0, 0xff);
  g2a p;
  p.inf = 0;
  if (compressed) {
    if (!ok1 || !ok0) return C_BAD;
    p.x = fp2_make(fp_to_mont(x0), fp_to_mont(x1));
    fp2 y;
    if (!fp2_sqrt(fp2_add(fp2_mul(fp2_sqr(p.x), p.x), B2), &y)) return C_NOC;
    if (fp2_lex_largest(y) != ((b0 & 0x20) != 0)) y = fp2_neg(y);
    p.y = y;
  } else {
    if (b0 & 0x20) return C_BAD;
    fp y1, y0;
    int ok3 = fp_from_be(b + 96, &y1, 0xff), ok2 = fp_from_be(b + 144, &y0, 0xff);
    if (!ok1 || !ok0 || !ok2 || !ok3) return C_BAD;
    p.x = fp2_make(fp_to_mont(x0), fp_to_mont(x1));
    p.y = fp2_make(fp_to_mont(y0), fp_to_mont(y1));
    if (!g2_on_curve(p)) return C_NOC;
  }
  if (!g2_in_group(p)) return C_NIG;
  *out = p;
  return C_OK;
}
static void g2_encode192(g2a a, uint8_t* b) {
  if (a.inf) {
    memset(b, 0, 192);
    b[0] = 0x40;
    return;
  }
  fp_to_be(a.x.c1, b);
  fp_to_be(a.x.c0, b + 48);
  fp_to_be(a.y.c1, b + 96);
  fp_to_be(a.y.c0, b + 144);
}
static void g2_encode96(g2a a, uint8_t* b) {
  if (a.inf) {
    memset(b, 0, 96);
    b[0] = 0xc0;
    return;
  }
  fp_to_be(a.x.c1, b);
  fp_to_be(a.x.c0, b + 48);
  b[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0);
}

/* ============================================================================================ SHA-256 */
static const uint32_t SK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_blocks(uint32_t st[8], const uint8_t* p, size_t nblk) {
  for (size_t bk = 0; bk < nblk; bk++, p += 64) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
      uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
      uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SK[i] + w[i];
      uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      h = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
    st[5] += f;
    st[6] += g;
    st[7] += h;
  }
}
static void sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t full = len / 64;
  sha256_blocks(st, msg, full);
  uint8_t tail[128];
  size_t rem = len - full * 64;
  memset(tail, 0, sizeof tail);
  memcpy(tail, msg + full * 64, rem);
  tail[rem] = 0x80;
  size_t tl = rem + 9 <= 64 ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha256_blocks(st, tail, tl / 64);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8);
    out[4 * i + 3] = (uint8_t)st[i];
  }
}

/* ============================================================================================ hash_to_G2 */
static const char DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";
#define DST_LEN 43

/* expand_message_xmd(msg, DST, 256) (RFC 9380 5.3.1) */
static void expand_xmd(const uint8_t* msg, size_t mlen, uint8_t out[256]) {
  uint8_t buf[64 + 256 + 2 + 1 + DST_LEN + 1];
  size_t o = 0;
  memset(buf, 0, 64);
  o = 64;
  memcpy(buf + o, msg, mlen);
  o += mlen;
  buf[o++] = 1; /* I2OSP(256, 2) */
  buf[o++] = 0;
  buf[o++] = 0;
  memcpy(buf + o, DST, DST_LEN);
  o += DST_LEN;
  buf[o++] = DST_LEN;
  uint8_t b0[32], bi[32];
  sha256(buf, o, b0);
  uint8_t blk[32 + 1 + DST_LEN + 1];
  for (int i = 1; i <= 8; i++) {
    for (int k = 0; k < 32; k++) blk[k] = i == 1 ? b0[k] : (uint8_t)(b0[k] ^ bi[k]);
    blk[32] = (uint8_t)i;
    memcpy(blk + 33, DST, DST_LEN);
    blk[33 + DST_LEN] = DST_LEN;
    sha256(blk, sizeof blk, bi);
    memcpy(out + 32 * (i - 1), bi, 32);
  }
}
/* 64 big-endian bytes mod p, Montgomery */
static fp fp_from_be64(const uint8_t* b) {
  fp lo, hi = fp_zero();
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)b[63 - 8 * i - k] << (8 * k);
    lo.l[i] = v;
  }
  for (int i = 0; i < 2; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)b[15 - 8 * i - k] << (8 * k);
    hi.l[i] = v;
  }
  while (geq6(lo.l, P.l)) sub6(lo.l, lo.l, P.l); /* fp_mul needs operands < p (no 7th word) */
  return fp_add(fp_mul(lo, R2), fp_mul(hi, R3));
}

static fp2 SSWU_A, SSWU_B, SSWU_Z, SSWU_MB_A, SSWU_B_ZA; /* -B/A, B/(Z A) */
static fp2 ISO_XNUM[4], ISO_XDEN[3], ISO_YNUM[4], ISO_YDEN[4];

/* RFC 9380 6.6.2 simplified SWU on E2' (non-constant-time restatement, as oracle map_to_curve_sswu) */
static g2a map_sswu(fp2 u) {
  fp2 Zu2 = fp2_mul(SSWU_Z, fp2_sqr(u));
  fp2 tv = fp2_add(fp2_sqr(Zu2), Zu2);
  fp2 x1 = fp2_is_zero(tv) ? SSWU_B_ZA : fp2_mul(SSWU_MB_A, fp2_add(fp2_one(), fp2_inv(tv)));
  fp2 gx1 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x1), SSWU_A), x1), SSWU_B);
  g2a r;
  r.inf = 0;
  fp2 y;
  if (fp2_sqrt(gx1, &y)) {
    r.x = x1;
  } else {
    fp2 x2 = fp2_mul(Zu2, x1);
    fp2 gx2 = fp2_add(fp2_mul(fp2_add(fp2_sqr(x2), SSWU_A), x2), SSWU_B);
    fp2_sqrt(gx2, &y);
    r.x = x2;
  }
  if (fp2_sgn0(u) != fp2_sgn0(y)) y = fp2_neg(y);
  r.y = y;
  return r;
}
static fp2 poly(const fp2* c, int n, fp2 x) {
  fp2 acc = fp2_zero();
  for (int i = n - 1; i >= 0; i--) acc = fp2_add(fp2_mul(acc, x), c[i]);
  return acc;
}
/* 3-isogeny E2' -> E2 into Jacobian coordinates (no inversion) */
static g2j iso3(g2a p) {
  fp2 xn = poly(ISO_XNUM, 4, p.x), xd = poly(ISO_XDEN, 3, p.x);
  fp2 yn = poly(ISO_YNUM, 4, p.x), yd = poly(ISO_YDEN, 4, p.x);
  if (fp2_is_zero(xd) || fp2_is_zero(yd)) return g2_inf();
  g2j r;
  fp2 dd = fp2_mul(xd, yd);
  r.z = dd;
  r.x = fp2_mul(fp2_mul(xn, yd), dd);
  r.y = fp2_mul(fp2_mul(fp2_mul(p.y, yn), fp2_mul(fp2_sqr(xd), xd)), fp2_sqr(yd));
  return r;
}
/* RFC 9380 G.3 h_eff P (Budroni-Pintore) */
static g2j clear_cofactor(g2j P) {
  g2j t1 = g2_neg(g2_mul_zabs(P));
  g2j t2 = g2_psi(P);
  g2j t3 = g2_psi2(g2_dbl(P));
  t3 = g2_add(t3, g2_neg(t2));
  t2 = g2_add(t1, t2);
  t2 = g2_neg(g2_mul_zabs(t2));
  t3 = g2_add(t3, t2);
  t3 = g2_add(t3, g2_neg(t1));
  return g2_add(t3, g2_neg(P));
}
static g2j hash_to_g2(const uint8_t* msg, size_t len) {
  uint8_t ub[256];
  expand_xmd(msg, len, ub);
  fp2 u0 = fp2_make(fp_from_be64(ub), fp_from_be64(ub + 64));
  fp2 u1 = fp2_make(fp_from_be64(ub + 128), fp_from_be64(ub + 192));
  g2j Q = g2_add(iso3(map_sswu(u0)), iso3(map_sswu(u1)));
  return clear_cofactor(Q);
}

/* ============================================================================================ pairing */
typedef struct {
  fp2 x, y, z;
} g2p;
static void dbl_line(g2p* T, fp xP, fp yP, fp2* l0, fp2* l1, fp2* l4) {
  fp2 A = fp2_mul_fp(fp2_mul(T->x, T->y), HALF);
  fp2 B = fp2_sqr(T->y), C = fp2_sqr(T->z);
  fp2 E = fp2_mul_xi(C);
  E = fp2_add(fp2_dbl(E), E);
  E = fp2_dbl(fp2_dbl(E)); /* 12 xi C = 3 b' C */
  fp2 F = fp2_add(fp2_dbl(E), E);
  fp2 G = fp2_mul_fp(fp2_add(B, F), HALF);
  fp2 H = fp2_sub(fp2_sub(fp2_sqr(fp2_add(T->y, T->z)), B), C);
  fp2 J = fp2_sqr(T->x), E2 = fp2_sqr(E);
  T->x = fp2_mul(A, fp2_sub(B, F));
  T->y = fp2_sub(fp2_sqr(G), fp2_add(fp2_dbl(E2), E2));
  T->z = fp2_mul(B, H);
  *l0 = fp2_sub(E, B);
  *l1 = fp2_mul_fp(fp2_add(fp2_dbl(J), J), xP);
  *l4 = fp2_mul_fp(fp2_neg(H), yP);
}
static void add_line(g2p* T, g2a Q, fp xP, fp yP, fp2* l0, fp2* l1, fp2* l4) {
  fp2 theta = fp2_sub(T->y, fp2_mul(Q.y, T->z)), lam = fp2_sub(T->x, fp2_mul(Q.x, T->z));
  fp2 C = fp2_sqr(theta), D = fp2_sqr(lam), E = fp2_mul(lam, D), F = fp2_mul(T->z, C), G = fp2_mul(T->x, D);
  fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  fp2 X3 = fp2_mul(lam, H);
  fp2 Y3 = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), fp2_mul(T->y, E));
  fp2 Z3 = fp2_mul(T->z, E);
  *l0 = fp2_sub(fp2_mul(theta, Q.x), fp2_mul(lam, Q.y));
  *l1 = fp2_mul_fp(fp2_neg(theta), xP);
  *l4 = fp2_mul_fp(lam, yP);
  T->x = X3;
  T->y = Y3;
  T->z = Z3;
}
/* prod_i conj(f_{|z|,Q_i}(P_i)) with one shared squaring per step (multi-Miller loop); pairs with an
 * infinity point contribute 1 */
static fp12 miller_loop_n(const g1a* Pp, const g2a* Qp, int n) {
  g2p* T = (g2p*)malloc(sizeof(g2p) * (n ? n : 1));
  for (int i = 0; i < n; i++) {
    T[i].x = Qp[i].x;
    T[i].y = Qp[i].y;
    T[i].z = fp2_one();
  }
  fp12 f = fp12_one();
  for (int b = 62; b >= 0; b--) {
    if (b != 62) f = fp12_sqr(f);
    for (int i = 0; i < n; i++) {
      if (Pp[i].inf || Qp[i].inf) continue;
      fp2 l0, l1, l4;
      dbl_line(&T[i], Pp[i].x, Pp[i].y, &l0, &l1, &l4);
      f = fp12_mul_by_014(f, l0, l1, l4);
    }
    if ((Z_ABS >> b) & 1)
      for (int i = 0; i < n; i++) {
        if (Pp[i].inf || Qp[i].inf) continue;
        fp2 l0, l1, l4;
        add_line(&T[i], Qp[i], Pp[i].x, Pp[i].y, &l0, &l1, &l4);
        f = fp12_mul_by_014(f, l0, l1, l4);
      }
  }
  free(T);
  return fp12_conj(f);
}
static fp12 cyc_pow_z(fp12 f) { /* f^z, z < 0, cyclotomic */
  fp12 r = f;
  for (int i = 62; i >= 0; i--) {
    r = fp12_cyc_sqr(r);
    if ((Z_ABS >> i) & 1) r = fp12_mul(r, f);
  }
  return fp12_conj(r);
}
/* returns e^3 (same "== 1" answer): easy part, then (z-1)^2 (z+p)(z^2+p^2-1) + 3 */
static fp12 final_exp(fp12 f) {
  fp12 f1 = fp12_mul(fp12_conj(f), fp12_inv(f));
  fp12 m = fp12_mul(fp12_frob(f1, 2), f1);
  fp12 t = fp12_mul(cyc_pow_z(m), fp12_conj(m));
  t = fp12_mul(cyc_pow_z(t), fp12_conj(t));
  t = fp12_mul(cyc_pow_z(t), fp12_frob(t, 1));
  t = fp12_mul(fp12_mul(cyc_pow_z(cyc_pow_z(t)), fp12_frob(t, 2)), fp12_conj(t));
  return fp12_mul(t, fp12_mul(fp12_sqr(m), m));
}

/* ============================================================================================ init */
static void hex_to_fp(const char* h, fp* out) { /* plain big-endian hex -> Montgomery */
  fp v = fp_zero();
  size_t n = strlen(h);
  for (size_t i = 0; i < n; i++) {
    char c = h[i];
    uint64_t d = (c >= '0' && c <= '9') ? (uint64_t)(c - '0') : (uint64_t)((c | 32) - 'a' + 10);
    /* v = v * 16 + d */
    uint64_t carry = d;
    for (int k = 0; k < 6; k++) {
      u128 t = ((u128)v.l[k] << 4) + carry;
      v.l[k] = (uint64_t)t;
      carry = (uint64_t)(t >> 64);
    }
  }
  *out = fp_to_mont(v);
}
static fp2 hex2(const char* a, const char* b) {
  fp2 r;
  hex_to_fp(a, &r.c0);
  hex_to_fp(b, &r.c1);
  return r;
}
static fp2 small2(int64_t a, int64_t b) {
  fp x = a >= 0 ? fp_small((uint64_t)a) : fp_neg(fp_small((uint64_t)(-a)));
  fp y = b >= 0 ? fp_small((uint64_t)b) : fp_neg(fp_small((uint64_t)(-b)));
  return fp2_make(x, y);
}
/* 6-limb (plain) helpers for exponent constants */
static void bn_sub_small(uint64_t* r, const uint64_t* a, uint64_t s) {
  uint64_t bw = s;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)a[i] - bw;
    r[i] = (uint64_t)d;
    bw = (uint64_t)(d >> 64) & 1;
  }
}
static void bn_add_small(uint64_t* r, const uint64_t* a, uint64_t s) {
  u128 c = s;
  for (int i = 0; i < 6; i++) {
    c += a[i];
    r[i] = (uint64_t)c;
    c >>= 64;
  }
}
static void bn_div_small(uint64_t* r, const uint64_t* a, uint64_t d) {
  u128 rem = 0;
  for (int i = 5; i >= 0; i--) {
    u128 cur = (rem << 64) | a[i];
    r[i] = (uint64_t)(cur / d);
    rem = cur % d;
  }
}
static void init_once(void) {
  /* N0 = -p^-1 mod 2^64 (Newton) */
  uint64_t inv = 1;
  for (int i = 0; i < 7; i++) inv *= 2 - P.l[0] * inv;
  N0 = (uint64_t)0 - inv;
  /* R mod p, R^2 mod p by doubling */
  fp x = fp_zero();
  x.l[0] = 1;
  for (int i = 0; i < 768; i++) {
    fp t;
    uint64_t c = add6(t.l, x.l, x.l);
    fp s;
    if (c || geq6(t.l, P.l)) {
      sub6(s.l, t.l, P.l);
      t = s;
    }
    x = t;
    if (i == 383) R1 = x;
  }
  R2 = x;
  R3 = fp_mul(R2, R2);
  bn_sub_small(E_PM2, P.l, 2);
  uint64_t t6[6];
  bn_add_small(t6, P.l, 1);
  bn_div_small(E_P14, t6, 4);
  bn_sub_small(t6, P.l, 3);
  bn_div_small(E_P34, t6, 4);
  bn_sub_small(t6, P.l, 1);
  bn_div_small(E_PM1_2, t6, 2);
  HALF = fp_inv(fp_small(2));
  B1 = fp_small(4);
  B2 = small2(4, 4);
  hex_to_fp("17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB", &G1X);
  hex_to_fp("08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1", &G1Y);
  /* Frobenius and psi constants from xi = 1 + u */
  fp2 xi = small2(1, 1);
  uint64_t e6[6], e3[6], e2[6];
  bn_div_small(e6, t6, 6); /* (p-1)/6 */
  bn_div_small(e3, t6, 3);
  bn_div_small(e2, t6, 2);
  fp2 g = fp2_pow(xi, e6, 6);
  GAMMA1[0] = fp2_one();
  for (int k = 1; k < 6; k++) GAMMA1[k] = fp2_mul(GAMMA1[k - 1], g);
  for (int k = 0; k < 6; k++) GAMMA2[k] = fp2_mul(GAMMA1[k], fp2_conj(GAMMA1[k]));
  PSI_X = fp2_inv(fp2_pow(xi, e3, 6));
  PSI_Y = fp2_inv(fp2_pow(xi, e2, 6));
  PSI2_X = fp2_mul(fp2_conj(PSI_X), PSI_X);
  PSI2_Y = fp2_mul(fp2_conj(PSI_Y), PSI_Y);
  SSWU_A = small2(0, 240);
  SSWU_B = small2(1012, 1012);
  SSWU_Z = small2(-2, -1);
  SSWU_MB_A = fp2_mul(fp2_neg(SSWU_B), fp2_inv(SSWU_A));
  SSWU_B_ZA = fp2_mul(SSWU_B, fp2_inv(fp2_mul(SSWU_Z, SSWU_A)));
  /* RFC 9380 Appendix E.3 */
  ISO_XNUM[0] = hex2("5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6",
                     "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97d6");
  ISO_XNUM[1] = hex2("0", "11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71a");
  ISO_XNUM[2] = hex2("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71e",
                     "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38d");
  ISO_XNUM[3] = hex2("171d6541fa38ccfaed6dea691f5fb614cb14b4e7f4e810aa22d6108f142b85757098e38d0f671c7188e2aaaaaaaa5ed1", "0");
  ISO_XDEN[0] = small2(0, -72);
  ISO_XDEN[1] = small2(12, -12);
  ISO_XDEN[2] = small2(1, 0);
  ISO_YNUM[0] = hex2("1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706",
                     "1530477c7ab4113b59a4c18b076d11930f7da5d4a07f649bf54439d87d27e500fc8c25ebf8c92f6812cfc71c71c6d706");
  ISO_YNUM[1] = hex2("0", "5c759507e8e333ebb5b7a9a47d7ed8532c52d39fd3a042a88b58423c50ae15d5c2638e343d9c71c6238aaaaaaaa97be");
  ISO_YNUM[2] = hex2("11560bf17baa99bc32126fced787c88f984f87adf7ae0c7f9a208c6b4f20a4181472aaa9cb8d555526a9ffffffffc71c",
                     "8ab05f8bdd54cde190937e76bc3e447cc27c3d6fbd7063fcd104635a790520c0a395554e5c6aaaa9354ffffffffe38f");
  ISO_YNUM[3] = hex2("124c9ad43b6cf79bfbf7043de3811ad0761b0f37a1e26286b0e977c69aa274524e79097a56dc4bd9e1b371c71c718b10", "0");
  ISO_YDEN[0] = small2(-432, -432);
  ISO_YDEN[1] = small2(0, -216);
  ISO_YDEN[2] = small2(18, -18);
  ISO_YDEN[3] = small2(1, 0);
}
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void ensure_init(void) { pthread_once(&g_once, init_once); }

/* ============================================================================================ threads */
typedef void (*range_fn)(void* ctx, uint32_t i);
typedef struct {
  range_fn fn;
  void* ctx;
  uint32_t n;
  volatile uint32_t next;
} par_job;
static void* par_worker(void* a) {
  par_job* j = (par_job*)a;
  for (;;) {
    uint32_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
    if (i >= j->n) break;
    j->fn(j->ctx, i);
  }
  return NULL;
}
static int resolve_threads(int n_threads) {
  if (n_threads > 0) return n_threads;
  long c = sysconf(_SC_NPROCESSORS_ONLN);
  return c > 0 ? (int)c : 1;
}
static void par_for(uint32_t n, int n_threads, range_fn fn, void* ctx) {
  par_job j = {fn, ctx, n, 0};
  int nt = resolve_threads(n_threads);
  if ((uint32_t)nt > n) nt = (int)(n ? n : 1);
  if (nt <= 1) {
    par_worker(&j);
    return;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nt);
  for (int t = 0; t < nt; t++) pthread_create(&th[t], NULL, par_worker, &j);
  for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
  free(th);
}

/* ============================================================================================ keys */
static void sk_words(const uint8_t* be, uint64_t w[4]) {
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)be[31 - 8 * i - k] << (8 * k);
    w[i] = v;
  }
}
typedef struct {
  const uint8_t *sk, *msg;
  uint8_t* out;
} key_ctx;
static void do_sk_to_pk(void* c, uint32_t i) {
  key_ctx* k = (key_ctx*)c;
  uint64_t w[4];
  sk_words(k->sk + 32 * (size_t)i, w);
  g1a g = {G1X, G1Y, 0};
  g1_encode96(g1_to_aff(g1_mul(g1_from_aff(g), w, 4)), k->out + 96 * (size_t)i);
}
static void do_sign(void* c, uint32_t i) {
  key_ctx* k = (key_ctx*)c;
  uint64_t w[4];
  sk_words(k->sk + 32 * (size_t)i, w);
  g2_encode96(g2_to_aff(g2_mul(hash_to_g2(k->msg + 32 * (size_t)i, 32), w, 4)), k->out + 96 * (size_t)i);
}
static void do_hash(void* c, uint32_t i) {
  key_ctx* k = (key_ctx*)c;
  g2_encode192(g2_to_aff(hash_to_g2(k->msg + 32 * (size_t)i, 32)), k->out + 192 * (size_t)i);
}
int blscpu_sk_to_pk(uint32_t n, const uint8_t* sk, uint8_t* out, int n_threads) {
  ensure_init();
  key_ctx k = {sk, NULL, out};
  par_for(n, n_threads, do_sk_to_pk, &k);
  return 0;
}
int blscpu_sign(uint32_t n, const uint8_t* sk, const uint8_t* msg, uint8_t* out, int n_threads) {
  ensure_init();
  key_ctx k = {sk, msg, out};
  par_for(n, n_threads, do_sign, &k);
  return 0;
}
int blscpu_hash_to_g2(uint32_t n, const uint8_t* msg, uint8_t* out, int n_threads) {
  ensure_init();
  key_ctx k = {NULL, msg, out};
  par_for(n, n_threads, do_hash, &k);
  return 0;
}
int blscpu_sig_status(const uint8_t* sig, uint32_t len) {
  ensure_init();
  g2a p;
  return sig_decode(sig, len, &p);
}
int blscpu_key_validate(const uint8_t* pk, uint32_t len) {
  ensure_init();
  g1a a;
  int st = g1_decode(pk, len, &a);
  if (st) return st;
  if (a.inf) return C_PKINF;
  return g1_in_group(a) ? C_OK : C_NIG;
}
int blscpu_pk_decode(const uint8_t* pk, uint32_t len, uint8_t* out) {
  ensure_init();
  g1a a;
  int st = g1_decode(pk, len, &a);
  if (!st) g1_encode96(a, out);
  return st;
}

/* ============================================================================================ table */
struct blscpu_table {
  uint32_t n;
  g1a* pk;
};
blscpu_table* blscpu_table_create(const uint8_t* pk96, uint32_t n, uint32_t* bad) {
  ensure_init();
  blscpu_table* t = (blscpu_table*)malloc(sizeof *t);
  t->n = n;
  t->pk = (g1a*)malloc(sizeof(g1a) * (n ? n : 1));
  for (uint32_t i = 0; i < n; i++) {
    if (g1_decode(pk96 + 96 * (size_t)i, 96, &t->pk[i]) != C_OK) {
      if (bad) *bad = i;
      free(t->pk);
      free(t);
      return NULL;
    }
  }
  return t;
}
void blscpu_table_free(blscpu_table* t) {
  if (!t) return;
  free(t->pk);
  free(t);
}

/* ============================================================================================ sets */
/* the aggregated pubkey of set i (PublicKey.aggregate + fromBytes(affine)): status and affine point */
static int set_pubkey(const blsgpu_batch* b, const blscpu_table* t, uint32_t i, g1a* out) {
  if (b->pk_bytes && !b->set_pk_first) {
    int st = g1_decode(b->pk_bytes + 96 * (size_t)i, 96, out);
    if (st) return st;
    return out->inf ? C_PKINF : C_OK;
  }
  uint32_t a = b->set_pk_first[i], e = b->set_pk_first[i + 1];
  if (a == e) return C_EAGG;
  g1j acc = g1_inf();
  for (uint32_t k = a; k < e; k++) {
    g1a q;
    if (b->pk_bytes) {
      int st = g1_decode(b->pk_bytes + 96 * (size_t)k, 96, &q);
      if (st) return st;
    } else {
      uint32_t idx = b->pk_index[k];
      if (!t || idx >= t->n) return BLSGPU_ERR_ARGS;
      q = t->pk[idx];
    }
    acc = g1_add_aff(acc, q);
  }
  *out = g1_to_aff(acc);
  return out->inf ? C_PKINF : C_OK;
}

typedef struct {
  const blsgpu_batch* b;
  const blscpu_table* t;
  uint8_t* out;
  uint32_t out_len;
  int8_t* status;
} agg_ctx;
static void do_agg(void* c, uint32_t i) {
  agg_ctx* a = (agg_ctx*)c;
  g1a pk;
  int st = set_pubkey(a->b, a->t, i, &pk);
  if (st == C_PKINF) {
    st = C_OK; /* the aggregate itself may be the identity; toBytes encodes it */
    pk.inf = 1;
  }
  a->status[i] = (int8_t)st;
  uint8_t* o = a->out + (size_t)a->out_len * i;
  memset(o, 0, a->out_len);
  if (st == C_OK) {
    if (a->out_len == 48)
      g1_encode48(pk, o);
    else
      g1_encode96(pk, o);
  }
}
int blscpu_aggregate_pubkeys(const blsgpu_batch* b, const blscpu_table* t, uint8_t* out, uint32_t out_len,
                             int8_t* status, int n_threads) {
  ensure_init();
  if (out_len != 48 && out_len != 96) return BLSGPU_ERR_ARGS;
  agg_ctx a = {b, t, out, out_len, status};
  par_for(b->n_sets, n_threads, do_agg, &a);
  return 0;
}

static inline uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return z ? z : 1;
}

/* one deserialized set (SignatureSetDeserialized + the decoded signature) */
typedef struct {
  int pk_st, sig_st;
  g1a pk;
  g2a sig;
  const uint8_t* msg;
  uint32_t gidx; /* global set index (random scalar stream position) */
} dset;

/* verifySignatureSetsMaybeBatch (maybeBatch.ts:16-39) over sets already deserialized in the worker's
 * order: 1 / 0, or -code when it throws */
static int maybe_batch(dset* s, uint32_t n, uint64_t seed) {
  if (n == 0) return -C_ESET;
  for (uint32_t i = 0; i < n; i++)
    if (s[i].pk_st) return -s[i].pk_st;
  for (uint32_t i = 0; i < n; i++)
    if (s[i].sig_st) return -s[i].sig_st;
  g1a* P = (g1a*)malloc(sizeof(g1a) * (n + 1));
  g2a* Q = (g2a*)malloc(sizeof(g2a) * (n + 1));
  g2j S = g2_inf();
  for (uint32_t i = 0; i < n; i++) {
    uint64_t r = n >= 2 ? splitmix64_at(seed, s[i].gidx) : 1; /* 1 set: CoreVerify */
    g1j rp = g1_from_aff(s[i].pk);
    if (r != 1) rp = g1_mul(rp, &r, 1);
    P[i] = g1_to_aff(rp);
    Q[i] = g2_to_aff(hash_to_g2(s[i].msg, 32));
    g2j rs = g2_from_aff(s[i].sig);
    if (r != 1) rs = g2_mul(rs, &r, 1);
    S = g2_add(S, rs);
  }
  g1a ng = {G1X, fp_neg(G1Y), 0};
  P[n] = ng;
  Q[n] = g2_to_aff(S);
  int ok = fp12_is_one(final_exp(miller_loop_n(P, Q, (int)n + 1)));
  free(P);
  free(Q);
  return ok;
}

/* ---- the pool: calls -> <=128-set jobs -> worker requests of >= 128 sets -> verifyManySignatureSets */
typedef struct {
  uint32_t call;        /* blsgpu_batch job (= verifySignatureSets call) it belongs to */
  uint32_t first, end;  /* set range */
  int batchable;
  int result;
} pjob;
typedef struct {
  uint32_t first_job, end_job;
} wreq;
typedef struct {
  const blsgpu_batch* b;
  const blscpu_table* t;
  pjob* jobs;
  wreq* reqs;
  uint64_t seed;
  volatile uint32_t retries, sigs_success;
} pool_ctx;

static void deserialize(pool_ctx* c, uint32_t first, uint32_t end, dset* out) {
  const blsgpu_batch* b = c->b;
  for (uint32_t i = first; i < end; i++) {
    dset* d = &out[i - first];
    d->pk_st = set_pubkey(b, c->t, i, &d->pk);
    d->msg = b->msgs + 32 * (size_t)i;
    d->gidx = i;
    d->sig_st = C_OK;
  }
  for (uint32_t i = first; i < end; i++) {
    dset* d = &out[i - first];
    d->sig_st = sig_decode(b->sigs + (size_t)b->sig_stride * i, b->sig_len[i], &d->sig);
  }
}
/* chunkifyMaximizeChunkSize (multithread/utils.ts:4-19): items per chunk of an array of len items */
static uint32_t chunk_size(uint32_t len, uint32_t min) {
  uint32_t cc = len / min;
  return cc <= 1 ? len : (len + cc - 1) / cc;
}

/* chunkifyMaximizeChunkSize as index lists: chunk_first[0..*n_chunks] (the reference returns [arr] when
 * floor(len / min) <= 1, an empty arr included) */
int blscpu_chunkify(uint32_t len, uint32_t min, uint32_t* chunk_first, uint32_t* n_chunks) {
  if (!min || !chunk_first || !n_chunks) return BLSGPU_ERR_ARGS;
  uint32_t c = 0, per = chunk_size(len, min);
  if (len / min <= 1) {
    chunk_first[c++] = 0;
  } else {
    for (uint32_t i = 0; i < len; i += per) chunk_first[c++] = i;
  }
  chunk_first[c] = len;
  *n_chunks = c;
  return 0;
}

/* worker.ts verifyManySignatureSets over one request's jobs */
static void do_request(void* vc, uint32_t r) {
  pool_ctx* c = (pool_ctx*)vc;
  wreq q = c->reqs[r];
  uint32_t nb = 0;
  uint32_t* batchable = (uint32_t*)malloc(sizeof(uint32_t) * (q.end_job - q.first_job + 1));
  uint32_t* rest = (uint32_t*)malloc(sizeof(uint32_t) * (q.end_job - q.first_job + 1));
  uint32_t nr = 0;
  for (uint32_t j = q.first_job; j < q.end_job; j++) {
    if (c->jobs[j].result != 2) continue; /* empty call, already rejected */
    if (c->jobs[j].batchable)
      batchable[nb++] = j;
    else
      rest[nr++] = j;
  }
  if (nb) {
    uint32_t per = chunk_size(nb, 16);
    for (uint32_t k = 0; k < nb; k += per) {
      uint32_t ke = k + per < nb ? k + per : nb;
      uint32_t total = 0;
      for (uint32_t x = k; x < ke; x++) total += c->jobs[batchable[x]].end - c->jobs[batchable[x]].first;
      dset* all = (dset*)malloc(sizeof(dset) * (total ? total : 1));
      uint32_t o = 0;
      for (uint32_t x = k; x < ke; x++) {
        pjob* pj = &c->jobs[batchable[x]];
        deserialize(c, pj->first, pj->end, all + o);
        o += pj->end - pj->first;
      }
      int v = maybe_batch(all, total, c->seed);
      free(all);
      if (v == 1) {
        for (uint32_t x = k; x < ke; x++) {
          c->jobs[batchable[x]].result = 1;
          __atomic_fetch_add(&c->sigs_success, c->jobs[batchable[x]].end - c->jobs[batchable[x]].first,
                             __ATOMIC_RELAXED);
        }
      } else {
        __atomic_fetch_add(&c->retries, 1, __ATOMIC_RELAXED);
        for (uint32_t x = k; x < ke; x++) rest[nr++] = batchable[x];
      }
    }
  }
  for (uint32_t x = 0; x < nr; x++) {
    pjob* pj = &c->jobs[rest[x]];
    uint32_t n = pj->end - pj->first;
    dset* d = (dset*)malloc(sizeof(dset) * (n ? n : 1));
    deserialize(c, pj->first, pj->end, d);
    pj->result = maybe_batch(d, n, c->seed);
    free(d);
  }
  free(batchable);
  free(rest);
}

int blscpu_verify_jobs(const blsgpu_batch* b, const blscpu_table* t, int8_t* job_result, int n_threads,
                       blscpu_stats* st) {
  ensure_init();
  if (!b || !b->job_first_set) return BLSGPU_ERR_ARGS;
  /* calls -> jobs of <= 128 sets (chunkifyMaximizeChunkSize(sets, 128), index.ts:156) */
  uint32_t cap = b->n_jobs + b->n_sets / 64 + 2, nj = 0;
  pjob* jobs = (pjob*)malloc(sizeof(pjob) * cap);
  for (uint32_t call = 0; call < b->n_jobs; call++) {
    uint32_t a = b->job_first_set[call], e = b->job_first_set[call + 1], len = e - a;
    int batchable = b->job_flags && (b->job_flags[call] & 1);
    if (len == 0) { /* empty call: rejected (the reference throws on empty results / sets) */
      pjob pj = {call, a, a, batchable, -C_ESET};
      jobs[nj++] = pj;
      continue;
    }
    uint32_t per = chunk_size(len, 128);
    for (uint32_t k = a; k < e; k += per) {
      pjob pj = {call, k, k + per < e ? k + per : e, batchable, 2};
      if (nj == cap) {
        cap *= 2;
        jobs = (pjob*)realloc(jobs, sizeof(pjob) * cap);
      }
      jobs[nj++] = pj;
    }
  }
  /* prepareWork: pack queued jobs until the request holds >= 128 sets (index.ts:386-401) */
  wreq* reqs = (wreq*)malloc(sizeof(wreq) * (nj + 1));
  uint32_t nr = 0, j = 0;
  while (j < nj) {
    uint32_t total = 0, j0 = j;
    while (j < nj && total < 128) {
      total += jobs[j].end - jobs[j].first;
      j++;
    }
    reqs[nr].first_job = j0;
    reqs[nr].end_job = j;
    nr++;
  }
  pool_ctx c = {b, t, jobs, reqs, b->seed ? b->seed : 0x4C4F444553544152ull, 0, 0};
  par_for(nr, n_threads, do_request, &c);
  /* AND per call; the first rejection (in job order) rejects the call */
  for (uint32_t call = 0; call < b->n_jobs; call++) job_result[call] = 1;
  int8_t* seen_err = (int8_t*)calloc(b->n_jobs ? b->n_jobs : 1, 1);
  for (uint32_t k = 0; k < nj; k++) {
    pjob* pj = &jobs[k];
    if (seen_err[pj->call]) continue;
    if (pj->result < 0) {
      job_result[pj->call] = (int8_t)pj->result;
      seen_err[pj->call] = 1;
    } else if (pj->result == 0) {
      job_result[pj->call] = 0;
    }
  }
  free(seen_err);
  if (st) {
    st->work_requests = nr;
    st->batch_retries = c.retries;
    st->batch_sigs_success = c.sigs_success;
    st->threads = (uint32_t)resolve_threads(n_threads);
  }
  free(jobs);
  free(reqs);
  return 0;
}

void blscpu_count_reset(void) { g_count = 0; }
uint64_t blscpu_count_get(void) { return g_count; }
