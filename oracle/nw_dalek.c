/*
 * nw_dalek.c — TEST INFRASTRUCTURE ONLY: the timed CPU baseline ("dalek-equivalent
 * restatement"). Only bench.py's cpu_baseline legs and tests/ load it; the product library
 * (libnarwhal_amd.so) never links or calls it.
 *
 * nw_oracle.c is the parity checker: plain 4-bit fixed windows and full extended additions,
 * written for obviousness, not speed. Timing the checker would understate the reference's
 * CPU path ("What's missing" 4), so this file restates, with the SAME
 * ALGORITHMS, what the reference's crypto calls run on a host core:
 *
 *   crypto::Signature::verify       /root/reference/crypto/src/lib.rs:200-204
 *     -> ed25519-dalek 1.0.1 PublicKey::verify_strict [ext]: decompress A and R, small-order
 *        checks by [8]P, k = H(R||A||M) (Scalar::from_hash), then
 *        EdwardsPoint::vartime_double_scalar_mul_basepoint(k, -A, s): width-5 NAF of k over
 *        8 cached odd multiples of -A (ProjectiveNiels), width-8 NAF of s over the 64 affine
 *        odd multiples of B (AffineNiels), one shared doubling chain from the highest
 *        nonzero digit, Projective/Completed point models; R' == R by projective compare.
 *   crypto::Signature::verify_batch /root/reference/crypto/src/lib.rs:206-219
 *     -> ed25519-dalek 1.0.1 verify_batch [ext]: 128-bit z_i, B coefficient -(sum z_i s_i),
 *        EdwardsPoint::optional_multiscalar_mul = vartime Straus (NAF-5 ProjectiveNiels
 *        tables) below 190 points, else vartime Pippenger with signed radix-2^w digits,
 *        w = 6 / 7 / 8 below 500 / below 800 / from 800 points, 2^(w-1) buckets of extended
 *        points, the running-sum bucket reduction, columns combined by mul_by_pow_2(w).
 *   curve25519-dalek 3.x u64 backend [ext]: FieldElement51 (radix 2^51, u128 products,
 *        additions without reduction, subtraction/negation through 16p and a weak
 *        reduction), Scalar52 (radix 2^52, Montgomery reduction, R = 2^260).
 * [ext] = crates.io code not vendored in /root/reference (the reference's Cargo.toml pins
 * ed25519-dalek 1.0.1); restated here from the published algorithms, not copied.
 *
 * Not restated: the merlin transcript (Keccak over every hram, length and s) that seeds
 * dalek's z_i. Its cost is omitted, which makes this baseline slightly FASTER than dalek.
 * z_i come from ChaCha20 (as the checker) or are injected.
 *
 * Verdicts (status, index) are the checker's bit for bit with injected z
 * (tests/test_dalek_restatement.py: edge corpus, golden batches, random sets).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sys/random.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "nw_oracle.h"
#include "nw_dalek.h"

typedef unsigned __int128 u128;

/* ---------------------------------------------------------------------------------- */
/* FieldElement51                                                                      */
/* ---------------------------------------------------------------------------------- */
typedef struct { uint64_t l[5]; } f51;
#define M51 ((1ULL << 51) - 1)

static inline u128 mw(uint64_t a, uint64_t b) { return (u128)a * b; }

/* parallel carries, limb 4's carry folded into limb 0 times 19 */
static inline void f_weak(f51* h) {
  const uint64_t c0 = h->l[0] >> 51, c1 = h->l[1] >> 51, c2 = h->l[2] >> 51,
                 c3 = h->l[3] >> 51, c4 = h->l[4] >> 51;
  h->l[0] = (h->l[0] & M51) + 19 * c4;
  h->l[1] = (h->l[1] & M51) + c0;
  h->l[2] = (h->l[2] & M51) + c1;
  h->l[3] = (h->l[3] & M51) + c2;
  h->l[4] = (h->l[4] & M51) + c3;
}
static inline void f_zero(f51* h) { memset(h, 0, sizeof *h); }
static inline void f_one(f51* h) { f_zero(h); h->l[0] = 1; }
static inline void f_add(f51* h, const f51* a, const f51* b) {
  for (int i = 0; i < 5; ++i) h->l[i] = a->l[i] + b->l[i];
}
/* a - b through a + 16p - b */
static inline void f_sub(f51* h, const f51* a, const f51* b) {
  const uint64_t p16_0 = 16 * ((1ULL << 51) - 19), p16 = 16 * M51;
  h->l[0] = a->l[0] + p16_0 - b->l[0];
  for (int i = 1; i < 5; ++i) h->l[i] = a->l[i] + p16 - b->l[i];
  f_weak(h);
}
static inline void f_neg(f51* h, const f51* a) { f51 z; f_zero(&z); f_sub(h, &z, a); }

/* the five 128-bit columns of a product, then one carry sweep */
static inline void f_carry_cols(f51* h, u128 c0, u128 c1, u128 c2, u128 c3, u128 c4) {
  uint64_t o0, o1, o2, o3, o4;
  c1 += (uint64_t)(c0 >> 51); o0 = (uint64_t)c0 & M51;
  c2 += (uint64_t)(c1 >> 51); o1 = (uint64_t)c1 & M51;
  c3 += (uint64_t)(c2 >> 51); o2 = (uint64_t)c2 & M51;
  c4 += (uint64_t)(c3 >> 51); o3 = (uint64_t)c3 & M51;
  const uint64_t top = (uint64_t)(c4 >> 51); o4 = (uint64_t)c4 & M51;
  o0 += 19 * top;
  o1 += o0 >> 51; o0 &= M51;
  h->l[0] = o0; h->l[1] = o1; h->l[2] = o2; h->l[3] = o3; h->l[4] = o4;
}
static inline void f_mul(f51* h, const f51* a, const f51* b) {
  const uint64_t *x = a->l, *y = b->l;
  const uint64_t y1 = 19 * y[1], y2 = 19 * y[2], y3 = 19 * y[3], y4 = 19 * y[4];
  f_carry_cols(h,
               mw(x[0], y[0]) + mw(x[4], y1) + mw(x[3], y2) + mw(x[2], y3) + mw(x[1], y4),
               mw(x[1], y[0]) + mw(x[0], y[1]) + mw(x[4], y2) + mw(x[3], y3) + mw(x[2], y4),
               mw(x[2], y[0]) + mw(x[1], y[1]) + mw(x[0], y[2]) + mw(x[4], y3) + mw(x[3], y4),
               mw(x[3], y[0]) + mw(x[2], y[1]) + mw(x[1], y[2]) + mw(x[0], y[3]) + mw(x[4], y4),
               mw(x[4], y[0]) + mw(x[3], y[1]) + mw(x[2], y[2]) + mw(x[1], y[3]) + mw(x[0], y[4]));
}
/* k successive squarings (the symmetric terms doubled once) */
static inline void f_sqk(f51* h, const f51* a, int k) {
  f51 t = *a;
  while (k-- > 0) {
    const uint64_t* x = t.l;
    const uint64_t x3 = 19 * x[3], x4 = 19 * x[4];
    f_carry_cols(&t,
                 mw(x[0], x[0]) + 2 * (mw(x[1], x4) + mw(x[2], x3)),
                 mw(x[3], x3) + 2 * (mw(x[0], x[1]) + mw(x[2], x4)),
                 mw(x[1], x[1]) + 2 * (mw(x[0], x[2]) + mw(x[4], x3)),
                 mw(x[4], x4) + 2 * (mw(x[0], x[3]) + mw(x[1], x[2])),
                 mw(x[2], x[2]) + 2 * (mw(x[0], x[4]) + mw(x[1], x[3])));
  }
  *h = t;
}
static inline void f_sq(f51* h, const f51* a) { f_sqk(h, a, 1); }
static inline void f_sq2(f51* h, const f51* a) {
  f_sqk(h, a, 1);
  for (int i = 0; i < 5; ++i) h->l[i] *= 2;
}
static void f_from_bytes(f51* h, const uint8_t s[32]) {
  uint64_t w[4];
  memcpy(w, s, 32);
  h->l[0] = w[0] & M51;
  h->l[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  h->l[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  h->l[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  h->l[4] = (w[3] >> 12) & M51;
}
static void f_to_bytes(uint8_t s[32], const f51* a) {
  f51 t = *a;
  f_weak(&t);
  uint64_t q = (t.l[0] + 19) >> 51;
  for (int i = 1; i < 5; ++i) q = (t.l[i] + q) >> 51;
  t.l[0] += 19 * q;
  for (int i = 0; i < 4; ++i) { t.l[i + 1] += t.l[i] >> 51; t.l[i] &= M51; }
  t.l[4] &= M51;
  const uint64_t w[4] = {t.l[0] | (t.l[1] << 51), (t.l[1] >> 13) | (t.l[2] << 38),
                         (t.l[2] >> 26) | (t.l[3] << 25), (t.l[3] >> 39) | (t.l[4] << 12)};
  memcpy(s, w, 32);
}
static int f_eq(const f51* a, const f51* b) {
  uint8_t x[32], y[32];
  f_to_bytes(x, a);
  f_to_bytes(y, b);
  return memcmp(x, y, 32) == 0;
}
static int f_is_negative(const f51* a) {
  uint8_t x[32];
  f_to_bytes(x, a);
  return x[0] & 1;
}
/* z^(2^250 - 1) (and z^11 on the way): the shared addition chain of invert / pow_p58 */
static void f_pow22501(f51* t19, f51* t3, const f51* z) {
  f51 t0, t1, t2, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15, t16, t17, t18;
  f_sq(&t0, z);
  f_sqk(&t1, &t0, 2);
  f_mul(&t2, z, &t1);
  f_mul(t3, &t0, &t2);
  f_sq(&t4, t3);
  f_mul(&t5, &t2, &t4);
  f_sqk(&t6, &t5, 5);     f_mul(&t7, &t6, &t5);
  f_sqk(&t8, &t7, 10);    f_mul(&t9, &t8, &t7);
  f_sqk(&t10, &t9, 20);   f_mul(&t11, &t10, &t9);
  f_sqk(&t12, &t11, 10);  f_mul(&t13, &t12, &t7);
  f_sqk(&t14, &t13, 50);  f_mul(&t15, &t14, &t13);
  f_sqk(&t16, &t15, 100); f_mul(&t17, &t16, &t15);
  f_sqk(&t18, &t17, 50);  f_mul(t19, &t18, &t13);
}
static void f_invert(f51* h, const f51* z) {
  f51 t19, t3, t20;
  f_pow22501(&t19, &t3, z);
  f_sqk(&t20, &t19, 5);
  f_mul(h, &t20, &t3);
}
static void f_pow_p58(f51* h, const f51* z) {
  f51 t19, t3, t20;
  f_pow22501(&t19, &t3, z);
  f_sqk(&t20, &t19, 2);
  f_mul(h, &t20, z);
}

static f51 F_D, F_D2, F_SQRTM1;

/* sqrt_ratio_i: (u/v is a nonzero square or u == 0, the non-negative root of u/v or i u/v) */
static int f_sqrt_ratio_i(f51* r, const f51* u, const f51* v) {
  f51 v3, v7, t, uv3, uv7, check, nu, nui, rp;
  f_sq(&t, v);   f_mul(&v3, &t, v);
  f_sq(&t, &v3); f_mul(&v7, &t, v);
  f_mul(&uv3, u, &v3);
  f_mul(&uv7, u, &v7);
  f_pow_p58(&t, &uv7);
  f_mul(r, &uv3, &t);
  f_sq(&t, r);
  f_mul(&check, v, &t);
  f_neg(&nu, u);
  f_mul(&nui, &nu, &F_SQRTM1);
  const int correct = f_eq(&check, u), flipped = f_eq(&check, &nu), flipped_i = f_eq(&check, &nui);
  f_mul(&rp, &F_SQRTM1, r);
  if (flipped | flipped_i) *r = rp;
  if (f_is_negative(r)) f_neg(r, r);
  return correct | flipped;
}

/* ---------------------------------------------------------------------------------- */
/* Point models                                                                        */
/* ---------------------------------------------------------------------------------- */
typedef struct { f51 X, Y, Z, T; } ept;        /* extended                  */
typedef struct { f51 X, Y, Z; } ppt;           /* projective                */
typedef struct { f51 X, Y, Z, T; } cpt;        /* completed (P1 x P1)       */
typedef struct { f51 YpX, YmX, Z, T2d; } pnp;  /* projective Niels          */
typedef struct { f51 ypx, ymx, xy2d; } anp;    /* affine Niels              */

static void e_identity(ept* p) { f_zero(&p->X); f_one(&p->Y); f_one(&p->Z); f_zero(&p->T); }
static void p_identity(ppt* p) { f_zero(&p->X); f_one(&p->Y); f_one(&p->Z); }
static inline void c_to_p(ppt* r, const cpt* c) {
  f_mul(&r->X, &c->X, &c->T); f_mul(&r->Y, &c->Y, &c->Z); f_mul(&r->Z, &c->Z, &c->T);
}
static inline void c_to_e(ept* r, const cpt* c) {
  f51 X, Y, Z, T;
  f_mul(&X, &c->X, &c->T); f_mul(&Y, &c->Y, &c->Z); f_mul(&Z, &c->Z, &c->T); f_mul(&T, &c->X, &c->Y);
  r->X = X; r->Y = Y; r->Z = Z; r->T = T;
}
static inline void e_to_p(ppt* r, const ept* e) { r->X = e->X; r->Y = e->Y; r->Z = e->Z; }
/* (X : Y : Z) -> (XZ : YZ : Z^2 : XY) */
static inline void p_to_e(ept* r, const ppt* p) {
  f_mul(&r->X, &p->X, &p->Z); f_mul(&r->Y, &p->Y, &p->Z); f_sq(&r->Z, &p->Z);
  f_mul(&r->T, &p->X, &p->Y);
}
static inline void p_dbl(cpt* r, const ppt* p) {
  f51 XX, YY, ZZ2, XpY, XpY2, YYpXX, YYmXX;
  f_sq(&XX, &p->X);
  f_sq(&YY, &p->Y);
  f_sq2(&ZZ2, &p->Z);
  f_add(&XpY, &p->X, &p->Y);
  f_sq(&XpY2, &XpY);
  f_add(&YYpXX, &YY, &XX);
  f_sub(&YYmXX, &YY, &XX);
  f_sub(&r->X, &XpY2, &YYpXX);
  r->Y = YYpXX;
  r->Z = YYmXX;
  f_sub(&r->T, &ZZ2, &YYmXX);
}
static inline void e_to_pn(pnp* r, const ept* e) {
  f_add(&r->YpX, &e->Y, &e->X);
  f_sub(&r->YmX, &e->Y, &e->X);
  r->Z = e->Z;
  f_mul(&r->T2d, &e->T, &F_D2);
}
/* e + q (neg: e - q) */
static inline void add_pn(cpt* r, const ept* e, const pnp* q, int neg) {
  f51 YpX, YmX, PP, MM, TT2d, ZZ, ZZ2;
  f_add(&YpX, &e->Y, &e->X);
  f_sub(&YmX, &e->Y, &e->X);
  f_mul(&PP, &YpX, neg ? &q->YmX : &q->YpX);
  f_mul(&MM, &YmX, neg ? &q->YpX : &q->YmX);
  f_mul(&TT2d, &e->T, &q->T2d);
  f_mul(&ZZ, &e->Z, &q->Z);
  f_add(&ZZ2, &ZZ, &ZZ);
  f_sub(&r->X, &PP, &MM);
  f_add(&r->Y, &PP, &MM);
  if (neg) { f_sub(&r->Z, &ZZ2, &TT2d); f_add(&r->T, &ZZ2, &TT2d); }
  else { f_add(&r->Z, &ZZ2, &TT2d); f_sub(&r->T, &ZZ2, &TT2d); }
}
static inline void add_an(cpt* r, const ept* e, const anp* q, int neg) {
  f51 YpX, YmX, PP, MM, Txy2d, Z2;
  f_add(&YpX, &e->Y, &e->X);
  f_sub(&YmX, &e->Y, &e->X);
  f_mul(&PP, &YpX, neg ? &q->ymx : &q->ypx);
  f_mul(&MM, &YmX, neg ? &q->ypx : &q->ymx);
  f_mul(&Txy2d, &e->T, &q->xy2d);
  f_add(&Z2, &e->Z, &e->Z);
  f_sub(&r->X, &PP, &MM);
  f_add(&r->Y, &PP, &MM);
  if (neg) { f_sub(&r->Z, &Z2, &Txy2d); f_add(&r->T, &Z2, &Txy2d); }
  else { f_add(&r->Z, &Z2, &Txy2d); f_sub(&r->T, &Z2, &Txy2d); }
}
/* EdwardsPoint + EdwardsPoint */
static inline void e_add(ept* r, const ept* a, const ept* b) {
  pnp q; cpt c;
  e_to_pn(&q, b);
  add_pn(&c, a, &q, 0);
  c_to_e(r, &c);
}
static inline void e_dbl(ept* r, const ept* a) {
  ppt p; cpt c;
  e_to_p(&p, a);
  p_dbl(&c, &p);
  c_to_e(r, &c);
}
static void e_neg(ept* r, const ept* a) {
  f_neg(&r->X, &a->X); r->Y = a->Y; r->Z = a->Z; f_neg(&r->T, &a->T);
}
static void e_mul_pow2(ept* r, const ept* a, int k) {
  ppt s; cpt c;
  e_to_p(&s, a);
  for (int i = 0; i < k - 1; ++i) { p_dbl(&c, &s); c_to_p(&s, &c); }
  p_dbl(&c, &s);
  c_to_e(r, &c);
}
/* projective equality X1 Z2 == X2 Z1, Y1 Z2 == Y2 Z1 */
static int e_eq(const ept* a, const ept* b) {
  f51 u, v;
  f_mul(&u, &a->X, &b->Z); f_mul(&v, &b->X, &a->Z);
  if (!f_eq(&u, &v)) return 0;
  f_mul(&u, &a->Y, &b->Z); f_mul(&v, &b->Y, &a->Z);
  return f_eq(&u, &v);
}
static int e_is_identity(const ept* a) { ept id; e_identity(&id); return e_eq(a, &id); }
static int e_is_small_order(const ept* a) { ept t; e_mul_pow2(&t, a, 3); return e_is_identity(&t); }

static int e_decompress(ept* p, const uint8_t s[32]) {
  f51 one, YY, u, v, X;
  f_from_bytes(&p->Y, s);
  f_one(&one);
  f_sq(&YY, &p->Y);
  f_sub(&u, &YY, &one);
  f_mul(&v, &YY, &F_D);
  f_add(&v, &v, &one);
  if (!f_sqrt_ratio_i(&X, &u, &v)) return 0;
  if (s[31] >> 7) f_neg(&X, &X);
  p->X = X;
  p->Z = one;
  f_mul(&p->T, &X, &p->Y);
  return 1;
}

/* odd multiples P, 3P, ..., 15P as ProjectiveNiels (width-5 NAF table) */
static void naf5_table(pnp t[8], const ept* P) {
  ept P2, acc;
  cpt c;
  e_to_pn(&t[0], P);
  e_dbl(&P2, P);
  for (int i = 0; i < 7; ++i) {
    add_pn(&c, &P2, &t[i], 0);
    c_to_e(&acc, &c);
    e_to_pn(&t[i + 1], &acc);
  }
}
static anp B_ODD[64];   /* B, 3B, ..., 127B (affine Niels) */
static ept E_B;

/* ---------------------------------------------------------------------------------- */
/* Scalar52 (radix 2^52, Montgomery R = 2^260)                                         */
/* ---------------------------------------------------------------------------------- */
typedef struct { uint64_t l[5]; } s52;
#define M52 ((1ULL << 52) - 1)
static s52 S_L, S_R, S_RR;
static uint64_t S_LFACTOR;   /* -l^-1 mod 2^52 */

static void s_from_bytes(s52* r, const uint8_t b[32]) {
  uint64_t w[4];
  memcpy(w, b, 32);
  r->l[0] = w[0] & M52;
  r->l[1] = ((w[0] >> 52) | (w[1] << 12)) & M52;
  r->l[2] = ((w[1] >> 40) | (w[2] << 24)) & M52;
  r->l[3] = ((w[2] >> 28) | (w[3] << 36)) & M52;
  r->l[4] = w[3] >> 16;
}
static void s_to_bytes(uint8_t b[32], const s52* a) {
  const uint64_t w[4] = {a->l[0] | (a->l[1] << 52), (a->l[1] >> 12) | (a->l[2] << 40),
                         (a->l[2] >> 24) | (a->l[3] << 28), (a->l[3] >> 36) | (a->l[4] << 16)};
  memcpy(b, w, 32);
}
/* a - b, plus l when it went negative */
static void s_sub(s52* r, const s52* a, const s52* b) {
  uint64_t d[5], borrow = 0;
  for (int i = 0; i < 5; ++i) {
    borrow = a->l[i] - (b->l[i] + (borrow >> 63));
    d[i] = borrow & M52;
  }
  const uint64_t m = (uint64_t)0 - (borrow >> 63);
  uint64_t carry = 0;
  for (int i = 0; i < 5; ++i) {
    carry = (carry >> 52) + d[i] + (S_L.l[i] & m);
    r->l[i] = carry & M52;
  }
}
static void s_add(s52* r, const s52* a, const s52* b) {
  s52 s;
  uint64_t carry = 0;
  for (int i = 0; i < 5; ++i) {
    carry = a->l[i] + b->l[i] + (carry >> 52);
    s.l[i] = carry & M52;
  }
  s_sub(r, &s, &S_L);
}
static void s_mul_wide(u128 z[9], const s52* a, const s52* b) {
  for (int k = 0; k < 9; ++k) z[k] = 0;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) z[i + j] += mw(a->l[i], b->l[j]);
}
/* z / 2^260 mod l (z < 2^260 l) */
static void s_montgomery_reduce(s52* r, const u128 z[9]) {
  uint64_t n[5];
  u128 carry = 0;
  for (int k = 0; k < 5; ++k) {   /* clear the low five limbs */
    u128 sum = carry + z[k];
    for (int i = 0; i < k; ++i) sum += mw(n[i], S_L.l[k - i]);
    n[k] = ((uint64_t)sum * S_LFACTOR) & M52;
    sum += mw(n[k], S_L.l[0]);
    carry = sum >> 52;
  }
  s52 hi;
  for (int k = 5; k < 9; ++k) {
    u128 sum = carry + z[k];
    for (int i = k - 4; i < 5; ++i) sum += mw(n[i], S_L.l[k - i]);
    hi.l[k - 5] = (uint64_t)sum & M52;
    carry = sum >> 52;
  }
  hi.l[4] = (uint64_t)carry;
  s_sub(r, &hi, &S_L);
}
static void s_montgomery_mul(s52* r, const s52* a, const s52* b) {
  u128 z[9];
  s_mul_wide(z, a, b);
  s_montgomery_reduce(r, z);
}
/* a b mod l */
static void s_mul(s52* r, const s52* a, const s52* b) {
  s52 ab;
  s_montgomery_mul(&ab, a, b);
  s_montgomery_mul(r, &ab, &S_RR);
}
/* 64 bytes mod l (Scalar::from_bytes_mod_order_wide) */
static void s_from_wide(s52* r, const uint8_t b[64]) {
  uint64_t w[8];
  memcpy(w, b, 64);
  s52 lo, hi;
  lo.l[0] = w[0] & M52;
  lo.l[1] = ((w[0] >> 52) | (w[1] << 12)) & M52;
  lo.l[2] = ((w[1] >> 40) | (w[2] << 24)) & M52;
  lo.l[3] = ((w[2] >> 28) | (w[3] << 36)) & M52;
  lo.l[4] = ((w[3] >> 16) | (w[4] << 48)) & M52;
  hi.l[0] = (w[4] >> 4) & M52;
  hi.l[1] = ((w[4] >> 56) | (w[5] << 8)) & M52;
  hi.l[2] = ((w[5] >> 44) | (w[6] << 20)) & M52;
  hi.l[3] = ((w[6] >> 32) | (w[7] << 32)) & M52;
  hi.l[4] = w[7] >> 20;
  s_montgomery_mul(&lo, &lo, &S_R);    /* lo R / R           */
  s_montgomery_mul(&hi, &hi, &S_RR);   /* hi R^2 / R = hi R  */
  s_add(r, &hi, &lo);
}
static int s_canonical(const uint8_t s[32]) {   /* ed25519-dalek check_scalar */
  if ((s[31] & 240) == 0) return 1;
  s52 a, r;
  s_from_bytes(&a, s);
  s52 zero = {{0, 0, 0, 0, 0}};
  s_add(&r, &a, &zero);   /* reduces a < 2l by one conditional subtraction */
  uint8_t b[32];
  s_to_bytes(b, &r);
  return memcmp(b, s, 32) == 0;
}

/* width-w NAF of a 256-bit scalar: odd digits |d| < 2^(w-1), each followed by >= w-1 zeros */
static void naf(int8_t out[256], const uint8_t s[32], int w) {
  uint64_t x[5] = {0};
  memcpy(x, s, 32);
  memset(out, 0, 256);
  const uint64_t width = 1ULL << w, mask = width - 1;
  uint64_t carry = 0;
  int pos = 0;
  while (pos < 256) {
    const int wi = pos / 64, bi = pos % 64;
    uint64_t buf = x[wi] >> bi;
    if (bi > 64 - w) buf |= x[wi + 1] << (64 - bi);
    const uint64_t win = carry + (buf & mask);
    if (!(win & 1)) { ++pos; continue; }
    if (win < width / 2) { carry = 0; out[pos] = (int8_t)win; }
    else { carry = 1; out[pos] = (int8_t)((int64_t)win - (int64_t)width); }
    pos += w;
  }
}
/* signed radix-2^w digits in [-2^(w-1), 2^(w-1)]; returns the digit count */
static int radix_2w(int8_t* d, const uint8_t s[32], int w) {
  uint64_t x[4];
  memcpy(x, s, 32);
  const int cnt = (256 + w - 1) / w;
  const uint64_t radix = 1ULL << w, mask = radix - 1;
  uint64_t carry = 0;
  for (int i = 0; i < cnt; ++i) {
    const int off = i * w, wi = off / 64, bi = off % 64;
    uint64_t buf = x[wi] >> bi;
    if (bi > 64 - w && wi < 3) buf |= x[wi + 1] << (64 - bi);
    const uint64_t coef = carry + (buf & mask);
    carry = (coef + radix / 2) >> w;
    d[i] = (int8_t)((int64_t)coef - (int64_t)(carry << w));
  }
  if (w == 8) { d[cnt] = (int8_t)carry; return cnt + 1; }
  d[cnt - 1] = (int8_t)(d[cnt - 1] + (int8_t)(carry << w));
  return cnt;
}

/* ---------------------------------------------------------------------------------- */
/* Scalar multiplication                                                               */
/* ---------------------------------------------------------------------------------- */
/* [a]A + [b]B (vartime_double_scalar_mul_basepoint) */
static void double_base(ept* r, const uint8_t a[32], const ept* A, const uint8_t b[32]) {
  int8_t an[256], bn[256];
  naf(an, a, 5);
  naf(bn, b, 8);
  int i = 255;
  while (i > 0 && !an[i] && !bn[i]) --i;
  pnp ta[8];
  naf5_table(ta, A);
  ppt p; cpt c; ept e;
  p_identity(&p);
  for (;; --i) {
    p_dbl(&c, &p);
    if (an[i]) {
      c_to_e(&e, &c);
      add_pn(&c, &e, &ta[(an[i] > 0 ? an[i] : -an[i]) / 2], an[i] < 0);
    }
    if (bn[i]) {
      c_to_e(&e, &c);
      add_an(&c, &e, &B_ODD[(bn[i] > 0 ? bn[i] : -bn[i]) / 2], bn[i] < 0);
    }
    c_to_p(&p, &c);
    if (i == 0) break;
  }
  p_to_e(r, &p);
}

/* sum s_i P_i, vartime Straus (NAF-5 tables) */
static void msm_straus(ept* r, const uint8_t* sc, const ept* pts, size_t n) {
  int8_t* nafs = (int8_t*)malloc(256 * n);
  pnp* tabs = (pnp*)malloc(sizeof(pnp) * 8 * n);
  for (size_t j = 0; j < n; ++j) {
    naf(nafs + 256 * j, sc + 32 * j, 5);
    naf5_table(tabs + 8 * j, &pts[j]);
  }
  ppt p; cpt c; ept e;
  p_identity(&p);
  for (int i = 255; i >= 0; --i) {
    p_dbl(&c, &p);
    for (size_t j = 0; j < n; ++j) {
      const int d = nafs[256 * j + i];
      if (!d) continue;
      c_to_e(&e, &c);
      add_pn(&c, &e, &tabs[8 * j + (d > 0 ? d : -d) / 2], d < 0);
    }
    c_to_p(&p, &c);
  }
  p_to_e(r, &p);
  free(nafs);
  free(tabs);
}

/* sum s_i P_i, vartime Pippenger (signed radix 2^w, running-sum bucket reduction) */
static void msm_pippenger(ept* r, const uint8_t* sc, const ept* pts, size_t n) {
  const int w = n < 500 ? 6 : (n < 800 ? 7 : 8);
  const int nb = 1 << (w - 1);
  int8_t* dig = (int8_t*)malloc(64 * n);
  pnp* q = (pnp*)malloc(sizeof(pnp) * n);
  ept* bk = (ept*)malloc(sizeof(ept) * nb);
  int cnt = 0;
  for (size_t j = 0; j < n; ++j) {
    cnt = radix_2w(dig + 64 * j, sc + 32 * j, w);
    e_to_pn(&q[j], &pts[j]);
  }
  cpt c;
  for (int d = cnt - 1; d >= 0; --d) {
    for (int b = 0; b < nb; ++b) e_identity(&bk[b]);
    for (size_t j = 0; j < n; ++j) {
      const int v = dig[64 * j + d];
      if (!v) continue;
      const int b = (v > 0 ? v : -v) - 1;
      add_pn(&c, &bk[b], &q[j], v < 0);
      c_to_e(&bk[b], &c);
    }
    ept run = bk[nb - 1], sum = bk[nb - 1];
    for (int b = nb - 2; b >= 0; --b) {
      e_add(&run, &run, &bk[b]);
      e_add(&sum, &sum, &run);
    }
    if (d == cnt - 1) {
      *r = sum;
    } else {
      e_mul_pow2(r, r, w);
      e_add(r, r, &sum);
    }
  }
  free(dig);
  free(q);
  free(bk);
}

static void msm(ept* r, const uint8_t* sc, const ept* pts, size_t n) {
  if (n < 190) msm_straus(r, sc, pts, n);
  else msm_pippenger(r, sc, pts, n);
}

/* ---------------------------------------------------------------------------------- */
/* Initialisation: every constant is derived here, none is tabulated                   */
/* ---------------------------------------------------------------------------------- */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init(void) {
  f51 a, b, t;
  /* d = -121665 / 121666 */
  f_zero(&a); a.l[0] = 121665; f_neg(&a, &a);
  f_zero(&b); b.l[0] = 121666; f_invert(&t, &b);
  f_mul(&F_D, &a, &t);
  f_add(&F_D2, &F_D, &F_D);
  /* sqrt(-1) = 2^((p-1)/4) */
  f51 two; f_zero(&two); two.l[0] = 2;
  f_pow_p58(&t, &two);
  f_sq(&a, &t);
  f_mul(&F_SQRTM1, &a, &two);
  /* B: y = 4/5, x non-negative */
  f_zero(&a); a.l[0] = 4; f_zero(&b); b.l[0] = 5;
  f_invert(&t, &b);
  f_mul(&a, &a, &t);
  uint8_t by[32];
  f_to_bytes(by, &a);
  e_decompress(&E_B, by);
  /* B_ODD[i] = (2i + 1) B in affine Niels form */
  ept B2, P = E_B;
  e_dbl(&B2, &E_B);
  for (int i = 0; i < 64; ++i) {
    f51 zi, x, y, xy;
    f_invert(&zi, &P.Z);
    f_mul(&x, &P.X, &zi);
    f_mul(&y, &P.Y, &zi);
    f_add(&B_ODD[i].ypx, &y, &x);
    f_sub(&B_ODD[i].ymx, &y, &x);
    f_mul(&xy, &x, &y);
    f_mul(&B_ODD[i].xy2d, &xy, &F_D2);
    e_add(&P, &P, &B2);
  }
  /* l = 2^252 + 27742317777372353535851937790883648493 */
  static const uint8_t Lb[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58,
                                 0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9, 0xde, 0x14,
                                 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};
  s_from_bytes(&S_L, Lb);
  /* LFACTOR = -l^-1 mod 2^52 (Newton: each step doubles the correct low bits) */
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - S_L.l[0] * inv;
  S_LFACTOR = (0 - inv) & M52;
  /* R = 2^260 mod l, RR = 2^520 mod l by doubling 1 */
  s52 x = {{1, 0, 0, 0, 0}};
  for (int i = 1; i <= 520; ++i) {
    s_add(&x, &x, &x);
    if (i == 260) S_R = x;
  }
  S_RR = x;
}
static inline void ensure(void) { pthread_once(&g_once, init); }

/* ---------------------------------------------------------------------------------- */
/* Verification                                                                        */
/* ---------------------------------------------------------------------------------- */
static void from_hash3(s52* k, const uint8_t R[32], const uint8_t A[32], const uint8_t* m,
                       size_t len) {
  uint8_t buf[64 + 256], h[64];
  if (len <= 256) {
    memcpy(buf, R, 32);
    memcpy(buf + 32, A, 32);
    memcpy(buf + 64, m, len);
    nwo_sha512(buf, 64 + len, h);
  } else {
    uint8_t* big = (uint8_t*)malloc(64 + len);
    memcpy(big, R, 32);
    memcpy(big + 32, A, 32);
    memcpy(big + 64, m, len);
    nwo_sha512(big, 64 + len, h);
    free(big);
  }
  s_from_wide(k, h);
}

int nwd_verify_strict(const uint8_t* msg, size_t len, const uint8_t pk[32],
                      const uint8_t sig[64]) {
  ensure();
  if (sig[63] & 0xE0) return NWO_ERR_S_HIGH_BITS;           /* ed25519 Signature::from_bytes */
  ept A;
  if (!e_decompress(&A, pk)) return NWO_ERR_A_DECODE;       /* PublicKey::from_bytes        */
  if (!s_canonical(sig + 32)) return NWO_ERR_S_NONCANONICAL; /* InternalSignature::try_from  */
  ept R;
  if (!e_decompress(&R, sig)) return NWO_ERR_R_DECODE;
  if (e_is_small_order(&R)) return NWO_ERR_R_SMALL_ORDER;
  if (e_is_small_order(&A)) return NWO_ERR_A_SMALL_ORDER;
  s52 k;
  from_hash3(&k, sig, pk, msg, len);
  uint8_t kb[32];
  s_to_bytes(kb, &k);
  ept mA, Rp;
  e_neg(&mA, &A);
  double_base(&Rp, kb, &mA, sig + 32);
  return e_eq(&Rp, &R) ? NWO_OK : NWO_ERR_EQUATION;
}

void nwd_verify_strict_many(const uint8_t* msgs, size_t msg_stride, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, int32_t* status, int nthreads) {
  ensure();
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
#endif
  for (long i = 0; i < (long)n; ++i)
    status[i] = nwd_verify_strict(msgs + msg_stride * i, 32, pks + 32 * i, sigs + 64 * i);
  (void)nthreads;
}

int nwd_verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs,
                     size_t n, const uint8_t* z16, size_t* fail_index) {
  ensure();
  if (fail_index) *fail_index = n;
  if (n == 0) return NWO_OK;
  const size_t npts = 2 * n + 1;
  ept* pts = (ept*)malloc(sizeof(ept) * npts);
  uint8_t* sc = (uint8_t*)malloc(32 * npts);
  uint8_t* zbuf = NULL;
  int status = NWO_OK;
  size_t idx = n;
  /* crypto/src/lib.rs:214-217: per vote, Signature::from_bytes then PublicKey::from_bytes */
  for (size_t i = 0; i < n; ++i) {
    if (sigs[64 * i + 63] & 0xE0) { status = NWO_ERR_S_HIGH_BITS; idx = i; break; }
    if (!e_decompress(&pts[1 + n + i], pks + 32 * i)) { status = NWO_ERR_A_DECODE; idx = i; break; }
  }
  if (status == NWO_OK)   /* InternalSignature::try_from over all signatures */
    for (size_t i = 0; i < n; ++i)
      if (!s_canonical(sigs + 64 * i + 32)) { status = NWO_ERR_S_NONCANONICAL; idx = i; break; }
  if (status == NWO_OK)   /* Rs decompressed inside optional_multiscalar_mul */
    for (size_t i = 0; i < n; ++i)
      if (!e_decompress(&pts[1 + i], sigs + 64 * i)) { status = NWO_ERR_R_DECODE; idx = i; break; }
  if (status == NWO_OK) {
    if (!z16) {
      uint8_t key[32], nonce[8] = {0};
      size_t got = 0;
      while (got < sizeof key) {
        const ssize_t r = getrandom(key + got, sizeof key - got, 0);
        if (r > 0) got += (size_t)r;
      }
      zbuf = (uint8_t*)malloc(16 * n);
      nwo_chacha20_keystream(key, nonce, 0, zbuf, 16 * n);
      z16 = zbuf;
    }
    s52 bsum = {{0, 0, 0, 0, 0}};
    for (size_t i = 0; i < n; ++i) {
      uint8_t zb[32] = {0};
      memcpy(zb, z16 + 16 * i, 16);
      s52 z, k, s, t;
      s_from_bytes(&z, zb);
      from_hash3(&k, sigs + 64 * i, pks + 32 * i, digest, 32);
      s_from_bytes(&s, sigs + 64 * i + 32);
      memcpy(sc + 32 * (1 + i), zb, 32);              /* z_i R_i            */
      s_mul(&t, &z, &k);
      s_to_bytes(sc + 32 * (1 + n + i), &t);          /* (z_i k_i mod l) A_i */
      s_mul(&t, &z, &s);
      s_add(&bsum, &bsum, &t);
    }
    s52 zero = {{0, 0, 0, 0, 0}}, nb;
    s_sub(&nb, &zero, &bsum);
    s_to_bytes(sc, &nb);                              /* -(sum z_i s_i) B    */
    pts[0] = E_B;
    ept sum;
    msm(&sum, sc, pts, npts);
    if (!e_is_identity(&sum)) status = NWO_ERR_EQUATION;
  }
  free(pts);
  free(sc);
  free(zbuf);
  if (fail_index) *fail_index = idx;
  return status;
}

void nwd_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                           const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                           int32_t* status, int nthreads) {
  ensure();
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
  for (long b = 0; b < (long)nbatches; ++b) {
    const size_t off = offsets[b], cnt = offsets[b + 1] - offsets[b];
    status[b] = nwd_verify_batch(digests + 32 * b, pks + 32 * off, sigs + 64 * off, cnt,
                                 z16 ? z16 + 16 * off : NULL, NULL);
  }
  (void)nthreads;
}

int nwd_double_base(const uint8_t a[32], const uint8_t A[32], const uint8_t b[32],
                    uint8_t out[32]) {
  ensure();
  ept P, r;
  if (!e_decompress(&P, A)) return 0;
  double_base(&r, a, &P, b);
  f51 zi, x, y;
  f_invert(&zi, &r.Z);
  f_mul(&x, &r.X, &zi);
  f_mul(&y, &r.Y, &zi);
  f_to_bytes(out, &y);
  out[31] ^= (uint8_t)(f_is_negative(&x) << 7);
  return 1;
}
