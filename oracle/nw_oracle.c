/*
 * nw_oracle.c — CPU restatement of Narwhal's crypto hot path. TEST INFRASTRUCTURE ONLY:
 * the parity checker for the HIP engine and the bench.py cpu_baseline ("port"). Never
 * linked into the product library. See nw_oracle.h for the reference call sites it
 * follows and DESIGN.md "Oracle" for how it is pinned.
 *
 * Arithmetic follows the published curve25519-dalek 3.x u64 backend design (radix 2^51,
 * unified extended-coordinate formulas, Straus below 190 points and Pippenger above
 * with windows 6/7/8 at 500/800 points) so that as a CPU baseline it is a
 * "dalek-equivalent restatement". Constants are derived from their definitions at
 * start-up (d = -121665/121666, sqrt(-1) = 2^((p-1)/4), B.y = 4/5) rather than typed in.
 */
#include "nw_oracle.h"
#include "nw_dalek.h"

#include <stdlib.h>
#include <string.h>
#include <sys/random.h>
#include <pthread.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------------------ */
/* SHA-512 (FIPS 180-4)                                                                  */
/* ------------------------------------------------------------------------------------ */
static const uint64_t K512[80] = {
  0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
  0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
  0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
  0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
  0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
  0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
  0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
  0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
  0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
  0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
  0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
  0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
  0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
  0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
  0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
  0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
  0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

static const uint64_t H512[8] = {
  0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
  0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

typedef struct {
  uint64_t h[8];
  uint8_t buf[128];
  size_t buflen;
  uint64_t total;
} sha512_ctx;

static inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
static inline uint64_t load64_be(const uint8_t* p) {
  uint64_t r = 0;
  for (int i = 0; i < 8; ++i) r = (r << 8) | p[i];
  return r;
}
static inline void store64_be(uint8_t* p, uint64_t v) {
  for (int i = 7; i >= 0; --i) { p[i] = (uint8_t)v; v >>= 8; }
}

static void sha512_block(uint64_t h[8], const uint8_t* blk) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) w[t] = load64_be(blk + 8 * t);
  for (int t = 16; t < 80; ++t) {
    uint64_t s0 = rotr64(w[t - 15], 1) ^ rotr64(w[t - 15], 8) ^ (w[t - 15] >> 7);
    uint64_t s1 = rotr64(w[t - 2], 19) ^ rotr64(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 80; ++t) {
    uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + K512[t] + w[t];
    uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    uint64_t maj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + maj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha512_init(sha512_ctx* c) {
  memcpy(c->h, H512, sizeof(H512));
  c->buflen = 0;
  c->total = 0;
}
static void sha512_update(sha512_ctx* c, const uint8_t* m, size_t n) {
  c->total += n;
  if (c->buflen) {
    size_t take = 128 - c->buflen;
    if (take > n) take = n;
    memcpy(c->buf + c->buflen, m, take);
    c->buflen += take; m += take; n -= take;
    if (c->buflen == 128) { sha512_block(c->h, c->buf); c->buflen = 0; }
  }
  while (n >= 128) { sha512_block(c->h, m); m += 128; n -= 128; }
  if (n) { memcpy(c->buf, m, n); c->buflen = n; }
}
static void sha512_final(sha512_ctx* c, uint8_t out[64]) {
  uint64_t bits = c->total * 8;
  uint8_t pad[256];
  size_t padlen = (c->buflen < 112) ? (112 - c->buflen) : (240 - c->buflen);
  memset(pad, 0, sizeof(pad));
  pad[0] = 0x80;
  /* 128-bit length, high 64 bits zero (messages < 2^61 bytes). */
  store64_be(pad + padlen + 8, bits);
  sha512_update(c, pad, padlen + 16);
  for (int i = 0; i < 8; ++i) store64_be(out + 8 * i, c->h[i]);
}

void nwo_sha512(const uint8_t* msg, size_t len, uint8_t out[64]) {
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, msg, len);
  sha512_final(&c, out);
}

void nwo_sha512_digest32_many(const uint8_t* data, const uint64_t* offsets,
                              const uint64_t* lengths, size_t n, uint8_t* out32,
                              int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
  for (long i = 0; i < (long)n; ++i) {
    uint8_t full[64];
    nwo_sha512(data + offsets[i], lengths[i], full);
    memcpy(out32 + 32 * i, full, 32);
  }
  (void)nthreads;
}

/* ------------------------------------------------------------------------------------ */
/* ChaCha20 (DJB variant: 64-bit block counter in words 12-13, 64-bit nonce in 14-15)    */
/* rand_chacha 0.2 ChaCha20Rng::from_seed(seed) = this keystream with nonce 0, counter 0 */
/* ------------------------------------------------------------------------------------ */
static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static inline uint32_t load32_le(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
#define QR(a, b, c, d) \
  a += b; d ^= a; d = rotl32(d, 16); c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  c += d; b ^= c; b = rotl32(b, 7);

static void chacha20_block(const uint32_t in[16], uint8_t out[64]) {
  uint32_t x[16];
  memcpy(x, in, 64);
  for (int i = 0; i < 10; ++i) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
    QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
    QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; ++i) {
    uint32_t v = x[i] + in[i];
    out[4 * i] = (uint8_t)v; out[4 * i + 1] = (uint8_t)(v >> 8);
    out[4 * i + 2] = (uint8_t)(v >> 16); out[4 * i + 3] = (uint8_t)(v >> 24);
  }
}

void nwo_chacha20_keystream(const uint8_t key[32], const uint8_t nonce[8], uint64_t counter,
                            uint8_t* out, size_t len) {
  uint32_t st[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574};
  for (int i = 0; i < 8; ++i) st[4 + i] = load32_le(key + 4 * i);
  st[14] = load32_le(nonce);
  st[15] = load32_le(nonce + 4);
  uint8_t blk[64];
  while (len) {
    st[12] = (uint32_t)counter;
    st[13] = (uint32_t)(counter >> 32);
    chacha20_block(st, blk);
    size_t take = len < 64 ? len : 64;
    memcpy(out, blk, take);
    out += take; len -= take; ++counter;
  }
}

/* ------------------------------------------------------------------------------------ */
/* GF(2^255 - 19), radix 2^51                                                            */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint64_t v[5]; } fe;
#define MASK51 ((1ULL << 51) - 1)

static inline void fe_carry(fe* h) {
  uint64_t c;
  c = h->v[0] >> 51; h->v[0] &= MASK51; h->v[1] += c;
  c = h->v[1] >> 51; h->v[1] &= MASK51; h->v[2] += c;
  c = h->v[2] >> 51; h->v[2] &= MASK51; h->v[3] += c;
  c = h->v[3] >> 51; h->v[3] &= MASK51; h->v[4] += c;
  c = h->v[4] >> 51; h->v[4] &= MASK51; h->v[0] += c * 19;
}
static inline void fe_0(fe* h) { memset(h, 0, sizeof(*h)); }
static inline void fe_1(fe* h) { fe_0(h); h->v[0] = 1; }
static inline void fe_from_u64(fe* h, uint64_t x) { fe_0(h); h->v[0] = x & MASK51; h->v[1] = x >> 51; }

/* curve25519-dalek FieldElement51::from_bytes: low 255 bits, NOT reduced mod p. */
static void fe_frombytes(fe* h, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) {
    uint64_t r = 0;
    for (int j = 7; j >= 0; --j) r = (r << 8) | s[8 * i + j];
    w[i] = r;
  }
  h->v[0] = w[0] & MASK51;
  h->v[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
  h->v[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
  h->v[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
  h->v[4] = (w[3] >> 12) & MASK51;
}

/* Canonical encoding (fully reduced mod p). */
static void fe_tobytes(uint8_t s[32], const fe* f) {
  fe t = *f;
  fe_carry(&t); fe_carry(&t); fe_carry(&t);
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51;
  q = (t.v[2] + q) >> 51;
  q = (t.v[3] + q) >> 51;
  q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  t.v[1] += t.v[0] >> 51; t.v[0] &= MASK51;
  t.v[2] += t.v[1] >> 51; t.v[1] &= MASK51;
  t.v[3] += t.v[2] >> 51; t.v[2] &= MASK51;
  t.v[4] += t.v[3] >> 51; t.v[3] &= MASK51;
  t.v[4] &= MASK51;
  uint64_t w[4];
  w[0] = t.v[0] | (t.v[1] << 51);
  w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
  w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
  w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static inline void fe_add(fe* h, const fe* f, const fe* g) {
  for (int i = 0; i < 5; ++i) h->v[i] = f->v[i] + g->v[i];
  fe_carry(h);
}
/* f - g + 4p (limbwise 4p keeps every limb non-negative for carried g). */
static inline void fe_sub(fe* h, const fe* f, const fe* g) {
  h->v[0] = (f->v[0] + 0x1fffffffffffb4ULL) - g->v[0];
  h->v[1] = (f->v[1] + 0x1ffffffffffffcULL) - g->v[1];
  h->v[2] = (f->v[2] + 0x1ffffffffffffcULL) - g->v[2];
  h->v[3] = (f->v[3] + 0x1ffffffffffffcULL) - g->v[3];
  h->v[4] = (f->v[4] + 0x1ffffffffffffcULL) - g->v[4];
  fe_carry(h);
}
static inline void fe_neg(fe* h, const fe* f) { fe z; fe_0(&z); fe_sub(h, &z, f); }

static inline void fe_mul(fe* h, const fe* f, const fe* g) {
  const uint64_t f0 = f->v[0], f1 = f->v[1], f2 = f->v[2], f3 = f->v[3], f4 = f->v[4];
  const uint64_t g0 = g->v[0], g1 = g->v[1], g2 = g->v[2], g3 = g->v[3], g4 = g->v[4];
  const uint64_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4;
  u128 t0 = (u128)f0 * g0 + (u128)f1 * g4_19 + (u128)f2 * g3_19 + (u128)f3 * g2_19 + (u128)f4 * g1_19;
  u128 t1 = (u128)f0 * g1 + (u128)f1 * g0 + (u128)f2 * g4_19 + (u128)f3 * g3_19 + (u128)f4 * g2_19;
  u128 t2 = (u128)f0 * g2 + (u128)f1 * g1 + (u128)f2 * g0 + (u128)f3 * g4_19 + (u128)f4 * g3_19;
  u128 t3 = (u128)f0 * g3 + (u128)f1 * g2 + (u128)f2 * g1 + (u128)f3 * g0 + (u128)f4 * g4_19;
  u128 t4 = (u128)f0 * g4 + (u128)f1 * g3 + (u128)f2 * g2 + (u128)f3 * g1 + (u128)f4 * g0;
  t1 += (uint64_t)(t0 >> 51); uint64_t r0 = (uint64_t)t0 & MASK51;
  t2 += (uint64_t)(t1 >> 51); uint64_t r1 = (uint64_t)t1 & MASK51;
  t3 += (uint64_t)(t2 >> 51); uint64_t r2 = (uint64_t)t2 & MASK51;
  t4 += (uint64_t)(t3 >> 51); uint64_t r3 = (uint64_t)t3 & MASK51;
  uint64_t c = (uint64_t)(t4 >> 51); uint64_t r4 = (uint64_t)t4 & MASK51;
  r0 += c * 19;
  r1 += r0 >> 51; r0 &= MASK51;
  h->v[0] = r0; h->v[1] = r1; h->v[2] = r2; h->v[3] = r3; h->v[4] = r4;
}

static inline void fe_sq(fe* h, const fe* f) {
  const uint64_t f0 = f->v[0], f1 = f->v[1], f2 = f->v[2], f3 = f->v[3], f4 = f->v[4];
  const uint64_t f0_2 = 2 * f0, f1_2 = 2 * f1, f3_19 = 19 * f3, f4_19 = 19 * f4;
  u128 t0 = (u128)f0 * f0 + (u128)f1_2 * f4_19 + (u128)(2 * f2) * f3_19;
  u128 t1 = (u128)f0_2 * f1 + (u128)(2 * f2) * f4_19 + (u128)f3 * f3_19;
  u128 t2 = (u128)f0_2 * f2 + (u128)f1 * f1 + (u128)(2 * f3) * f4_19;
  u128 t3 = (u128)f0_2 * f3 + (u128)f1_2 * f2 + (u128)f4 * f4_19;
  u128 t4 = (u128)f0_2 * f4 + (u128)f1_2 * f3 + (u128)f2 * f2;
  t1 += (uint64_t)(t0 >> 51); uint64_t r0 = (uint64_t)t0 & MASK51;
  t2 += (uint64_t)(t1 >> 51); uint64_t r1 = (uint64_t)t1 & MASK51;
  t3 += (uint64_t)(t2 >> 51); uint64_t r2 = (uint64_t)t2 & MASK51;
  t4 += (uint64_t)(t3 >> 51); uint64_t r3 = (uint64_t)t3 & MASK51;
  uint64_t c = (uint64_t)(t4 >> 51); uint64_t r4 = (uint64_t)t4 & MASK51;
  r0 += c * 19;
  r1 += r0 >> 51; r0 &= MASK51;
  h->v[0] = r0; h->v[1] = r1; h->v[2] = r2; h->v[3] = r3; h->v[4] = r4;
}
static inline void fe_sqn(fe* h, const fe* f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

/* z^(2^250 - 1) and z^11, shared by invert and pow22523. */
static void fe_pow2_250_1(fe* out, fe* z11, const fe* z) {
  fe z2, z9, t, z5, z10, z20, z40, z50, z100, z200;
  fe_sq(&z2, z);              /* 2 */
  fe_sqn(&t, &z2, 2);         /* 8 */
  fe_mul(&z9, &t, z);         /* 9 */
  fe_mul(z11, &z9, &z2);      /* 11 */
  fe_sq(&t, z11);             /* 22 */
  fe_mul(&z5, &t, &z9);       /* 2^5 - 1 */
  fe_sqn(&t, &z5, 5);  fe_mul(&z10, &t, &z5);     /* 2^10 - 1 */
  fe_sqn(&t, &z10, 10); fe_mul(&z20, &t, &z10);   /* 2^20 - 1 */
  fe_sqn(&t, &z20, 20); fe_mul(&z40, &t, &z20);   /* 2^40 - 1 */
  fe_sqn(&t, &z40, 10); fe_mul(&z50, &t, &z10);   /* 2^50 - 1 */
  fe_sqn(&t, &z50, 50); fe_mul(&z100, &t, &z50);  /* 2^100 - 1 */
  fe_sqn(&t, &z100, 100); fe_mul(&z200, &t, &z100); /* 2^200 - 1 */
  fe_sqn(&t, &z200, 50); fe_mul(out, &t, &z50);   /* 2^250 - 1 */
}
static void fe_invert(fe* out, const fe* z) {
  fe t, z11;
  fe_pow2_250_1(&t, &z11, z);
  fe_sqn(&t, &t, 5);          /* 2^255 - 32 */
  fe_mul(out, &t, &z11);      /* 2^255 - 21 = p - 2 */
}
static void fe_pow22523(fe* out, const fe* z) {
  fe t, z11;
  fe_pow2_250_1(&t, &z11, z);
  fe_sqn(&t, &t, 2);          /* 2^252 - 4 */
  fe_mul(out, &t, z);         /* 2^252 - 3 = (p-5)/8 */
}
static int fe_eq(const fe* a, const fe* b) {
  uint8_t x[32], y[32];
  fe_tobytes(x, a); fe_tobytes(y, b);
  return memcmp(x, y, 32) == 0;
}
static int fe_iszero(const fe* a) {
  uint8_t x[32];
  fe_tobytes(x, a);
  for (int i = 0; i < 32; ++i) if (x[i]) return 0;
  return 1;
}
static int fe_isnegative(const fe* a) {
  uint8_t x[32];
  fe_tobytes(x, a);
  return x[0] & 1;
}

static fe FE_D, FE_D2, FE_SQRTM1;

/* curve25519-dalek FieldElement::sqrt_ratio_i. Returns was_nonzero_square; r = the
 * non-negative root of u/v (or of i*u/v). */
static int fe_sqrt_ratio_i(fe* r, const fe* u, const fe* v) {
  fe v3, v7, t, uv3, uv7, check, neg_u, neg_u_i, r_prime;
  fe_sq(&t, v); fe_mul(&v3, &t, v);
  fe_sq(&t, &v3); fe_mul(&v7, &t, v);
  fe_mul(&uv3, u, &v3);
  fe_mul(&uv7, u, &v7);
  fe_pow22523(&t, &uv7);
  fe_mul(r, &uv3, &t);
  fe_sq(&t, r); fe_mul(&check, v, &t);
  fe_neg(&neg_u, u);
  fe_mul(&neg_u_i, &neg_u, &FE_SQRTM1);
  int correct = fe_eq(&check, u);
  int flipped = fe_eq(&check, &neg_u);
  int flipped_i = fe_eq(&check, &neg_u_i);
  fe_mul(&r_prime, &FE_SQRTM1, r);
  if (flipped || flipped_i) *r = r_prime;
  if (fe_isnegative(r)) fe_neg(r, r);
  return correct || flipped;
}

/* ------------------------------------------------------------------------------------ */
/* Edwards points, extended coordinates (X:Y:Z:T), -x^2 + y^2 = 1 + d x^2 y^2            */
/* ------------------------------------------------------------------------------------ */
typedef struct { fe X, Y, Z, T; } ge;

static void ge_identity(ge* p) { fe_0(&p->X); fe_1(&p->Y); fe_1(&p->Z); fe_0(&p->T); }

/* Unified (complete) addition, add-2008-hwcd-3 with k = 2d. */
static void ge_add(ge* r, const ge* p, const ge* q) {
  fe a, b, c, d, e, f, g, h, t1, t2;
  fe_sub(&t1, &p->Y, &p->X); fe_sub(&t2, &q->Y, &q->X); fe_mul(&a, &t1, &t2);
  fe_add(&t1, &p->Y, &p->X); fe_add(&t2, &q->Y, &q->X); fe_mul(&b, &t1, &t2);
  fe_mul(&t1, &p->T, &q->T); fe_mul(&c, &t1, &FE_D2);
  fe_mul(&t1, &p->Z, &q->Z); fe_add(&d, &t1, &t1);
  fe_sub(&e, &b, &a); fe_sub(&f, &d, &c); fe_add(&g, &d, &c); fe_add(&h, &b, &a);
  fe_mul(&r->X, &e, &f); fe_mul(&r->Y, &g, &h); fe_mul(&r->T, &e, &h); fe_mul(&r->Z, &f, &g);
}

/* dbl-2008-hwcd with a = -1. */
static void ge_dbl(ge* r, const ge* p) {
  fe A, B, C, D, E, F, G, H, t;
  fe_sq(&A, &p->X);
  fe_sq(&B, &p->Y);
  fe_sq(&t, &p->Z); fe_add(&C, &t, &t);
  fe_neg(&D, &A);
  fe_add(&t, &p->X, &p->Y); fe_sq(&E, &t); fe_sub(&E, &E, &A); fe_sub(&E, &E, &B);
  fe_add(&G, &D, &B);
  fe_sub(&F, &G, &C);
  fe_sub(&H, &D, &B);
  fe_mul(&r->X, &E, &F); fe_mul(&r->Y, &G, &H); fe_mul(&r->T, &E, &H); fe_mul(&r->Z, &F, &G);
}

static void ge_neg(ge* r, const ge* p) {
  fe_neg(&r->X, &p->X); r->Y = p->Y; r->Z = p->Z; fe_neg(&r->T, &p->T);
}

/* curve25519-dalek EdwardsPoint::ct_eq: X1 Z2 == X2 Z1 and Y1 Z2 == Y2 Z1. */
static int ge_eq(const ge* p, const ge* q) {
  fe a, b;
  fe_mul(&a, &p->X, &q->Z); fe_mul(&b, &q->X, &p->Z);
  if (!fe_eq(&a, &b)) return 0;
  fe_mul(&a, &p->Y, &q->Z); fe_mul(&b, &q->Y, &p->Z);
  return fe_eq(&a, &b);
}
static int ge_is_identity(const ge* p) {
  ge id; ge_identity(&id);
  return ge_eq(p, &id);
}
static int ge_is_small_order(const ge* p) {
  ge t;
  ge_dbl(&t, p); ge_dbl(&t, &t); ge_dbl(&t, &t);
  return ge_is_identity(&t);
}

static void ge_tobytes(uint8_t s[32], const ge* p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_tobytes(s, &y);
  s[31] ^= (uint8_t)(fe_isnegative(&x) << 7);
}

/* curve25519-dalek CompressedEdwardsY::decompress (y >= p accepted, x = 0 with sign 1
 * accepted). Returns 1 on success. */
static int ge_frombytes(ge* p, const uint8_t s[32]) {
  fe one, yy, u, v, x;
  fe_frombytes(&p->Y, s);
  fe_1(&one);
  fe_sq(&yy, &p->Y);
  fe_sub(&u, &yy, &one);
  fe_mul(&v, &yy, &FE_D); fe_add(&v, &v, &one);
  if (!fe_sqrt_ratio_i(&x, &u, &v)) return 0;
  if (s[31] >> 7) fe_neg(&x, &x);
  p->X = x;
  fe_1(&p->Z);
  fe_mul(&p->T, &p->X, &p->Y);
  return 1;
}

static ge GE_B;
static ge GE_B_TABLE[16];   /* j * B, j = 0..15 */

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_constants(void);
static inline void ensure_init(void);

/* ------------------------------------------------------------------------------------ */
/* Scalars mod l = 2^252 + 27742317777372353535851937790883648493 (u32 limbs, Barrett)   */
/* ------------------------------------------------------------------------------------ */
static const uint8_t L_BYTES[32] = {
  0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9, 0xde, 0x14,
  0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x10};
static uint32_t L32[8];
static uint32_t MU32[9];    /* floor(2^512 / l) */

static void bytes_to_u32(uint32_t* w, const uint8_t* b, int nwords) {
  for (int i = 0; i < nwords; ++i) w[i] = load32_le(b + 4 * i);
}
static void u32_to_bytes(uint8_t* b, const uint32_t* w, int nwords) {
  for (int i = 0; i < nwords; ++i) {
    b[4 * i] = (uint8_t)w[i]; b[4 * i + 1] = (uint8_t)(w[i] >> 8);
    b[4 * i + 2] = (uint8_t)(w[i] >> 16); b[4 * i + 3] = (uint8_t)(w[i] >> 24);
  }
}
/* a >= b over n words */
static int bn_geq(const uint32_t* a, const uint32_t* b, int n) {
  for (int i = n - 1; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 1;
}
/* a -= b over n words, returns borrow */
static uint32_t bn_sub(uint32_t* a, const uint32_t* b, int n) {
  uint64_t borrow = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t d = (uint64_t)a[i] - b[i] - borrow;
    a[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  return (uint32_t)borrow;
}
static void bn_mul(uint32_t* r, const uint32_t* a, int na, const uint32_t* b, int nb) {
  memset(r, 0, sizeof(uint32_t) * (na + nb));
  for (int i = 0; i < na; ++i) {
    uint64_t carry = 0;
    for (int j = 0; j < nb; ++j) {
      uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + carry;
      r[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r[i + nb] = (uint32_t)carry;
  }
}

static void sc_init_constants(void) {
  bytes_to_u32(L32, L_BYTES, 8);
  /* MU = floor(2^512 / l) by binary long division. */
  uint32_t rem[9] = {0}, lw[9] = {0};
  memcpy(lw, L32, sizeof(L32));
  memset(MU32, 0, sizeof(MU32));
  for (int bit = 512; bit >= 0; --bit) {
    /* rem = 2*rem + (bit == 512) */
    uint32_t carry = (bit == 512) ? 1 : 0;
    for (int i = 0; i < 9; ++i) {
      uint32_t nc = rem[i] >> 31;
      rem[i] = (rem[i] << 1) | carry;
      carry = nc;
    }
    if (bn_geq(rem, lw, 9)) {
      bn_sub(rem, lw, 9);
      if (bit < 288) MU32[bit / 32] |= 1u << (bit % 32);
    }
  }
}

/* x (16 words, < 2^512) mod l -> out (8 words). HAC Algorithm 14.42, b = 2^32, k = 8. */
static void sc_barrett(uint32_t out[8], const uint32_t x[16]) {
  uint32_t q2[18], q3[9], r2full[17], r[9];
  bn_mul(q2, x + 7, 9, MU32, 9);
  memcpy(q3, q2 + 9, sizeof(q3));
  bn_mul(r2full, q3, 9, L32, 8);
  memcpy(r, x, sizeof(uint32_t) * 9);
  bn_sub(r, r2full, 9);   /* mod b^9 */
  uint32_t lw[9] = {0};
  memcpy(lw, L32, sizeof(L32));
  while (bn_geq(r, lw, 9)) bn_sub(r, lw, 9);
  memcpy(out, r, sizeof(uint32_t) * 8);
}

void nwo_scalar_reduce64(const uint8_t in[64], uint8_t out[32]) {
  ensure_init();
  uint32_t x[16], o[8];
  bytes_to_u32(x, in, 16);
  sc_barrett(o, x);
  u32_to_bytes(out, o, 8);
}
void nwo_scalar_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  ensure_init();
  uint32_t aw[8], bw[8], x[16], o[8];
  bytes_to_u32(aw, a, 8); bytes_to_u32(bw, b, 8);
  bn_mul(x, aw, 8, bw, 8);
  sc_barrett(o, x);
  u32_to_bytes(out, o, 8);
}
void nwo_scalar_add(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  ensure_init();
  uint32_t aw[8], bw[8], x[16] = {0}, o[8];
  bytes_to_u32(aw, a, 8); bytes_to_u32(bw, b, 8);
  uint64_t c = 0;
  for (int i = 0; i < 8; ++i) { c += (uint64_t)aw[i] + bw[i]; x[i] = (uint32_t)c; c >>= 32; }
  x[8] = (uint32_t)c;
  sc_barrett(o, x);
  u32_to_bytes(out, o, 8);
}
static void sc_neg(uint8_t out[32], const uint8_t a[32]) {
  /* (l - (a mod l)) mod l */
  uint32_t x[16] = {0}, am[8], lw[8];
  bytes_to_u32(x, a, 8);
  sc_barrett(am, x);
  memcpy(lw, L32, sizeof(lw));
  int zero = 1;
  for (int i = 0; i < 8; ++i) if (am[i]) zero = 0;
  if (zero) { memset(out, 0, 32); return; }
  bn_sub(lw, am, 8);
  u32_to_bytes(out, lw, 8);
}
/* s < l ? (dalek Scalar::from_canonical_bytes / check_scalar) */
static int sc_is_canonical(const uint8_t s[32]) {
  uint32_t w[8];
  bytes_to_u32(w, s, 8);
  return !bn_geq(w, L32, 8);
}

/* ------------------------------------------------------------------------------------ */
/* Scalar multiplication                                                                 */
/* ------------------------------------------------------------------------------------ */
static inline int nibble(const uint8_t s[32], int i) { return (s[i >> 1] >> ((i & 1) * 4)) & 15; }

static void ge_table16(ge t[16], const ge* p) {
  ge_identity(&t[0]);
  t[1] = *p;
  for (int j = 2; j < 16; ++j) ge_add(&t[j], &t[j - 1], p);
}

/* [a]B + [b]P (Straus, 4-bit fixed windows, full 256-bit scalars). */
static void ge_double_scalarmult_vartime(ge* r, const uint8_t a[32], const uint8_t b[32],
                                         const ge* P) {
  ge tp[16];
  ge_table16(tp, P);
  ge_identity(r);
  for (int i = 63; i >= 0; --i) {
    if (i != 63) { ge_dbl(r, r); ge_dbl(r, r); ge_dbl(r, r); ge_dbl(r, r); }
    int na = nibble(a, i), nb = nibble(b, i);
    if (na) ge_add(r, r, &GE_B_TABLE[na]);
    if (nb) ge_add(r, r, &tp[nb]);
  }
}
static void ge_scalarmult(ge* r, const uint8_t s[32], const ge* P) {
  ge tp[16];
  ge_table16(tp, P);
  ge_identity(r);
  for (int i = 63; i >= 0; --i) {
    if (i != 63) { ge_dbl(r, r); ge_dbl(r, r); ge_dbl(r, r); ge_dbl(r, r); }
    int n = nibble(s, i);
    if (n) ge_add(r, r, &tp[n]);
  }
}

/* Multi-scalar multiplication sum s_i P_i. Straus (4-bit windows) below 190 points,
 * Pippenger above (window 6/7/8 at <500/<800/>=800), the thresholds dalek uses [ext]. */
static void ge_msm(ge* r, const uint8_t* scalars, const ge* pts, size_t n) {
  ge_identity(r);
  if (n == 0) return;
  if (n < 190) {
    ge* tabs = (ge*)malloc(sizeof(ge) * 16 * n);
    for (size_t i = 0; i < n; ++i) ge_table16(tabs + 16 * i, &pts[i]);
    for (int w = 63; w >= 0; --w) {
      if (w != 63) { ge_dbl(r, r); ge_dbl(r, r); ge_dbl(r, r); ge_dbl(r, r); }
      for (size_t i = 0; i < n; ++i) {
        int d = nibble(scalars + 32 * i, w);
        if (d) ge_add(r, r, &tabs[16 * i + d]);
      }
    }
    free(tabs);
    return;
  }
  int c = n < 500 ? 6 : (n < 800 ? 7 : 8);
  int nb = 1 << c;
  int nwin = (256 + c - 1) / c;
  ge* buckets = (ge*)malloc(sizeof(ge) * nb);
  for (int w = nwin - 1; w >= 0; --w) {
    for (int k = 0; k < c; ++k) ge_dbl(r, r);
    for (int b = 0; b < nb; ++b) ge_identity(&buckets[b]);
    for (size_t i = 0; i < n; ++i) {
      const uint8_t* s = scalars + 32 * i;
      int d = 0;
      for (int k = 0; k < c; ++k) {
        int bit = w * c + k;
        if (bit < 256) d |= ((s[bit >> 3] >> (bit & 7)) & 1) << k;
      }
      if (d) ge_add(&buckets[d], &buckets[d], &pts[i]);
    }
    ge run, tot;
    ge_identity(&run); ge_identity(&tot);
    for (int b = nb - 1; b >= 1; --b) {
      ge_add(&run, &run, &buckets[b]);
      ge_add(&tot, &tot, &run);
    }
    ge_add(r, r, &tot);
  }
  free(buckets);
}

/* ------------------------------------------------------------------------------------ */
/* Initialisation                                                                        */
/* ------------------------------------------------------------------------------------ */

static void init_constants(void) {
  fe a, b, t;
  /* d = -121665 / 121666 */
  fe_from_u64(&a, 121665); fe_neg(&a, &a);
  fe_from_u64(&b, 121666); fe_invert(&t, &b);
  fe_mul(&FE_D, &a, &t);
  fe_add(&FE_D2, &FE_D, &FE_D);
  /* sqrt(-1) = 2^((p-1)/4) = 2^(2^253 - 5): 2^(2^252-3) squared times 2 */
  fe two; fe_from_u64(&two, 2);
  fe_pow22523(&t, &two);         /* 2^((p-5)/8) */
  fe_sq(&a, &t); fe_mul(&FE_SQRTM1, &a, &two);   /* 2^((p-5)/4 + 1) = 2^((p-1)/4) */
  /* B: y = 4/5, x non-negative */
  uint8_t by[32];
  fe_from_u64(&a, 4); fe_from_u64(&b, 5); fe_invert(&t, &b); fe_mul(&a, &a, &t);
  fe_tobytes(by, &a);
  ge_frombytes(&GE_B, by);
  ge_table16(GE_B_TABLE, &GE_B);
  sc_init_constants();
}
static inline void ensure_init(void) { pthread_once(&g_once, init_constants); }

/* ------------------------------------------------------------------------------------ */
/* Keys and signing (fixtures)                                                           */
/* ------------------------------------------------------------------------------------ */
static void hram(uint8_t k[32], const uint8_t R[32], const uint8_t A[32], const uint8_t* m,
                 size_t len) {
  sha512_ctx c;
  uint8_t h[64];
  sha512_init(&c);
  sha512_update(&c, R, 32);
  sha512_update(&c, A, 32);
  sha512_update(&c, m, len);
  sha512_final(&c, h);
  nwo_scalar_reduce64(h, k);
}

void nwo_hram(const uint8_t R[32], const uint8_t A[32], const uint8_t* msg, size_t len,
              uint8_t k[32]) {
  ensure_init();
  hram(k, R, A, msg, len);
}

void nwo_keypair_from_seed(const uint8_t seed[32], uint8_t pk[32], uint8_t sk[64]) {
  ensure_init();
  uint8_t h[64];
  nwo_sha512(seed, 32, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  ge A;
  ge_scalarmult(&A, h, &GE_B);
  ge_tobytes(pk, &A);
  memcpy(sk, seed, 32);
  memcpy(sk + 32, pk, 32);
}

void nwo_sign_raw(const uint8_t a[32], const uint8_t prefix[32], const uint8_t A[32],
                  const uint8_t* msg, size_t len, uint8_t sig[64]) {
  ensure_init();
  sha512_ctx c;
  uint8_t h[64], r[32], k[32], ka[32];
  sha512_init(&c);
  sha512_update(&c, prefix, 32);
  sha512_update(&c, msg, len);
  sha512_final(&c, h);
  nwo_scalar_reduce64(h, r);
  ge R;
  ge_scalarmult(&R, r, &GE_B);
  ge_tobytes(sig, &R);
  hram(k, sig, A, msg, len);
  nwo_scalar_mul(k, a, ka);
  nwo_scalar_add(ka, r, sig + 32);
}

void nwo_sign(const uint8_t sk[64], const uint8_t* msg, size_t len, uint8_t sig[64]) {
  uint8_t h[64];
  nwo_sha512(sk, 32, h);
  h[0] &= 248; h[31] &= 127; h[31] |= 64;
  nwo_sign_raw(h, h + 32, sk + 32, msg, len, sig);
}

/* ------------------------------------------------------------------------------------ */
/* Verification                                                                          */
/* ------------------------------------------------------------------------------------ */
int nwo_verify_strict(const uint8_t* msg, size_t len, const uint8_t pk[32],
                      const uint8_t sig[64]) {
  ensure_init();
  /* crypto/src/lib.rs:201 ed25519::Signature::from_bytes: top 3 bits of s must be 0. */
  if (sig[63] & 0xE0) return NWO_ERR_S_HIGH_BITS;
  /* crypto/src/lib.rs:202 dalek::PublicKey::from_bytes -> decompress A. */
  ge A;
  if (!ge_frombytes(&A, pk)) return NWO_ERR_A_DECODE;
  /* crypto/src/lib.rs:203 verify_strict: InternalSignature::try_from -> check_scalar. */
  if (!sc_is_canonical(sig + 32)) return NWO_ERR_S_NONCANONICAL;
  ge R;
  if (!ge_frombytes(&R, sig)) return NWO_ERR_R_DECODE;
  if (ge_is_small_order(&R)) return NWO_ERR_R_SMALL_ORDER;
  if (ge_is_small_order(&A)) return NWO_ERR_A_SMALL_ORDER;
  uint8_t k[32];
  hram(k, sig, pk, msg, len);
  ge minusA, Rp;
  ge_neg(&minusA, &A);
  ge_double_scalarmult_vartime(&Rp, sig + 32, k, &minusA);   /* [s]B + [k](-A) */
  return ge_eq(&Rp, &R) ? NWO_OK : NWO_ERR_EQUATION;
}

void nwo_verify_strict_many(const uint8_t* msgs, size_t msg_stride, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, int32_t* status, int nthreads) {
  ensure_init();
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
#endif
  for (long i = 0; i < (long)n; ++i)
    status[i] = nwo_verify_strict(msgs + msg_stride * i, 32, pks + 32 * i, sigs + 64 * i);
  (void)nthreads;
}

static void random_z(uint8_t* z16, size_t n) {
  uint8_t key[32], nonce[8] = {0};
  size_t got = 0;
  while (got < sizeof(key)) {
    ssize_t r = getrandom(key + got, sizeof(key) - got, 0);
    if (r > 0) got += (size_t)r;
  }
  nwo_chacha20_keystream(key, nonce, 0, z16, 16 * n);
}

int nwo_verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs,
                     size_t n, const uint8_t* z16, size_t* fail_index) {
  ensure_init();
  if (fail_index) *fail_index = n;
  if (n == 0) return NWO_OK;   /* dalek: MSM over [0]B = identity */
  size_t npts = 2 * n + 1;
  ge* pts = (ge*)malloc(sizeof(ge) * npts);
  uint8_t* sc = (uint8_t*)malloc(32 * npts);
  uint8_t* zbuf = NULL;
  int status = NWO_OK;
  size_t idx = n;
  /* crypto/src/lib.rs:214-217: per vote, signature parse then key decompress; first `?`
   * failure returns. */
  for (size_t i = 0; i < n && status == NWO_OK; ++i) {
    if (sigs[64 * i + 63] & 0xE0) { status = NWO_ERR_S_HIGH_BITS; idx = i; break; }
    if (!ge_frombytes(&pts[1 + n + i], pks + 32 * i)) { status = NWO_ERR_A_DECODE; idx = i; break; }
  }
  /* dalek verify_batch: InternalSignature::try_from over all signatures (check_scalar). */
  if (status == NWO_OK) {
    for (size_t i = 0; i < n; ++i)
      if (!sc_is_canonical(sigs + 64 * i + 32)) { status = NWO_ERR_S_NONCANONICAL; idx = i; break; }
  }
  /* Rs decompressed inside optional_multiscalar_mul: any None -> VerifyError. */
  if (status == NWO_OK) {
    for (size_t i = 0; i < n; ++i)
      if (!ge_frombytes(&pts[1 + i], sigs + 64 * i)) { status = NWO_ERR_R_DECODE; idx = i; break; }
  }
  if (status == NWO_OK) {
    if (!z16) { zbuf = (uint8_t*)malloc(16 * n); random_z(zbuf, n); z16 = zbuf; }
    uint8_t bcoef[32] = {0};
    for (size_t i = 0; i < n; ++i) {
      uint8_t z[32] = {0}, k[32], t[32];
      memcpy(z, z16 + 16 * i, 16);
      hram(k, sigs + 64 * i, pks + 32 * i, digest, 32);
      memcpy(sc + 32 * (1 + i), z, 32);                    /* z_i  * R_i              */
      nwo_scalar_mul(z, k, sc + 32 * (1 + n + i));         /* (z_i k_i mod l) * A_i   */
      nwo_scalar_mul(z, sigs + 64 * i + 32, t);            /* z_i s_i                 */
      nwo_scalar_add(bcoef, t, bcoef);
    }
    sc_neg(sc, bcoef);                                     /* -(sum z_i s_i) * B      */
    pts[0] = GE_B;
    ge sum;
    ge_msm(&sum, sc, pts, npts);
    if (!ge_is_identity(&sum)) status = NWO_ERR_EQUATION;
  }
  free(pts); free(sc); free(zbuf);
  if (fail_index) *fail_index = idx;
  return status;
}

void nwo_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                           const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                           int32_t* status, int nthreads) {
  ensure_init();
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
  for (long b = 0; b < (long)nbatches; ++b) {
    size_t off = offsets[b], cnt = offsets[b + 1] - offsets[b];
    status[b] = nwo_verify_batch(digests + 32 * b, pks + 32 * off, sigs + 64 * off, cnt,
                                 z16 ? z16 + 16 * off : NULL, NULL);
  }
  (void)nthreads;
}

/* ------------------------------------------------------------------------------------ */
/* Helpers                                                                               */
/* ------------------------------------------------------------------------------------ */
int nwo_decompress(const uint8_t in[32], uint8_t out[32]) {
  ensure_init();
  ge p;
  if (!ge_frombytes(&p, in)) return 0;
  ge_tobytes(out, &p);
  return 1;
}
int nwo_is_small_order(const uint8_t in[32]) {
  ensure_init();
  ge p;
  if (!ge_frombytes(&p, in)) return -1;
  return ge_is_small_order(&p);
}
void nwo_scalarmult_base(const uint8_t s[32], uint8_t out[32]) {
  ensure_init();
  ge r;
  ge_scalarmult(&r, s, &GE_B);
  ge_tobytes(out, &r);
}
int nwo_scalarmult(const uint8_t s[32], const uint8_t P[32], uint8_t out[32]) {
  ensure_init();
  ge p, r;
  if (!ge_frombytes(&p, P)) return 0;
  ge_scalarmult(&r, s, &p);
  ge_tobytes(out, &r);
  return 1;
}
int nwo_point_add(const uint8_t P[32], const uint8_t Q[32], uint8_t out[32]) {
  ensure_init();
  ge p, q, r;
  if (!ge_frombytes(&p, P) || !ge_frombytes(&q, Q)) return 0;
  ge_add(&r, &p, &q);
  ge_tobytes(out, &r);
  return 1;
}
int nwo_msm(const uint8_t* scalars, const uint8_t* points, size_t n, uint8_t out[32],
            int* is_identity) {
  ensure_init();
  ge* pts = (ge*)malloc(sizeof(ge) * (n ? n : 1));
  for (size_t i = 0; i < n; ++i)
    if (!ge_frombytes(&pts[i], points + 32 * i)) { free(pts); return 0; }
  ge r;
  ge_msm(&r, scalars, pts, n);
  ge_tobytes(out, &r);
  if (is_identity) *is_identity = ge_is_identity(&r);
  free(pts);
  return 1;
}

/* ==================================================================================== */
/* Primary messages (TEST INFRASTRUCTURE): Header::verify, Vote::verify,                */
/* Certificate::verify — /root/reference/primary/src/messages.rs:48-67, 131-153,        */
/* 189-234; Committee — /root/reference/config/src/lib.rs:139-173.                       */
/* ==================================================================================== */

/* BTreeMap<PublicKey, Authority>::get over the sorted keys: index or -1. */
static long committee_find(const nwo_committee* c, const uint8_t pk[32]) {
  long lo = 0, hi = (long)c->nauth - 1;
  while (lo <= hi) {
    long mid = (lo + hi) / 2;
    int cmp = memcmp(c->pks + 32 * mid, pk, 32);
    if (cmp == 0) return mid;
    if (cmp < 0) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

/* Committee::stake (lib.rs:148-151): 0 for unknown keys. */
static uint32_t committee_stake(const nwo_committee* c, const uint8_t pk[32]) {
  long a = committee_find(c, pk);
  return a < 0 ? 0u : c->stakes[a];
}

/* Committee::quorum_threshold (lib.rs:167-173), config::Stake = u32 arithmetic. */
static uint32_t committee_quorum(const nwo_committee* c) {
  uint32_t total = 0;
  for (size_t a = 0; a < c->nauth; ++a) total += c->stakes[a];
  return 2u * total / 3u + 1u;
}

/* Sha512(x || round LE || y)[..32]: Vote::digest (messages.rs:145-153) and
 * Certificate::digest (226-234). */
void nwo_digest_72(const uint8_t x[32], uint64_t round, const uint8_t y[32], uint8_t out[32]) {
  uint8_t buf[72], h[64];
  memcpy(buf, x, 32);
  for (int i = 0; i < 8; ++i) buf[32 + i] = (uint8_t)(round >> (8 * i));
  memcpy(buf + 40, y, 32);
  nwo_sha512(buf, 72, h);
  memcpy(out, h, 32);
}

/* The signature checks the message layer calls: the checker's (nwo_*) or the timed
 * dalek-equivalent restatement's (nwd_*, nw_dalek.c). */
typedef struct {
  int (*strict)(const uint8_t*, size_t, const uint8_t*, const uint8_t*);
  int (*batch)(const uint8_t*, const uint8_t*, const uint8_t*, size_t, const uint8_t*, size_t*);
} sig_engine;
static const sig_engine ENGINE_CHECK = {nwo_verify_strict, nwo_verify_batch};
static const sig_engine ENGINE_DALEK = {nwd_verify_strict, nwd_verify_batch};

/* Header::verify (messages.rs:48-67). hb = author || round || P x (digest || wid) || parents. */
static int header_verify(const sig_engine* E, const nwo_committee* c, const uint8_t* hb,
                         size_t hlen, uint32_t np, const uint8_t id[32], const uint8_t sig[64],
                         uint64_t* index) {
  uint8_t h[64];
  nwo_sha512(hb, hlen, h);
  if (memcmp(h, id, 32) != 0) return NWO_DAG_INVALID_HEADER_ID;
  long a = committee_find(c, hb);
  if (a < 0 || c->stakes[a] == 0) { *index = UINT64_MAX; return NWO_DAG_UNKNOWN_AUTHORITY; }
  for (uint32_t e = 0; e < np; ++e) {
    uint32_t wid = load32_le(hb + 40 + 36 * (size_t)e + 32);
    int found = 0;
    for (uint64_t w = c->worker_offsets[a]; w < c->worker_offsets[a + 1]; ++w)
      found |= c->worker_ids[w] == wid;
    if (!found) { *index = e; return NWO_DAG_MALFORMED_HEADER; }
  }
  int st = E->strict(id, 32, hb, sig);
  return st ? NWO_DAG_INVALID_SIGNATURE + st : 0;
}

int nwo_header_verify(const nwo_committee* c, const uint8_t* hb, size_t hlen, uint32_t np,
                      const uint8_t id[32], const uint8_t sig[64], uint64_t* index) {
  uint64_t ix = 0;
  ensure_init();
  int st = header_verify(&ENGINE_CHECK, c, hb, hlen, np, id, sig, &ix);
  if (index) *index = ix;
  return st;
}

static int certificate_verify(const sig_engine* E, const nwo_committee* c, const uint8_t* hb,
                              size_t hlen, uint32_t np, const uint8_t id[32],
                              const uint8_t hsig[64], const uint8_t* vote_pks,
                              const uint8_t* vote_sigs, size_t nvotes, const uint8_t* z16,
                              uint64_t* index) {
  uint64_t ix = 0;
  int st = 0;
  ensure_init();
  uint64_t round = 0;
  for (int i = 0; i < 8; ++i) round |= (uint64_t)hb[32 + i] << (8 * i);
  /* Genesis certificates are always valid: (id, round, origin) == (0, 0, authority). */
  int idzero = 1;
  for (int i = 0; i < 32; ++i) idzero &= id[i] == 0;
  if (idzero && round == 0 && committee_find(c, hb) >= 0) goto done;
  st = header_verify(E, c, hb, hlen, np, id, hsig, &ix);
  if (st) goto done;
  {
    uint32_t weight = 0;
    for (size_t v = 0; v < nvotes; ++v) {
      for (size_t u = 0; u < v; ++u)
        if (memcmp(vote_pks + 32 * u, vote_pks + 32 * v, 32) == 0) {
          st = NWO_DAG_AUTHORITY_REUSE; ix = v; goto done;
        }
      uint32_t s = committee_stake(c, vote_pks + 32 * v);
      if (s == 0) { st = NWO_DAG_UNKNOWN_AUTHORITY; ix = v; goto done; }
      weight += s;
    }
    if (weight < committee_quorum(c)) { st = NWO_DAG_REQUIRES_QUORUM; goto done; }
    uint8_t cd[32];
    nwo_digest_72(id, round, hb, cd);
    size_t fi = 0;
    int b = E->batch(cd, vote_pks, vote_sigs, nvotes, z16, &fi);
    if (b) { st = NWO_DAG_INVALID_VOTES + b; ix = fi; }
  }
done:
  if (index) *index = ix;
  return st;
}

int nwo_certificate_verify(const nwo_committee* c, const uint8_t* hb, size_t hlen,
                           uint32_t np, const uint8_t id[32], const uint8_t hsig[64],
                           const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t nvotes,
                           const uint8_t* z16, uint64_t* index) {
  return certificate_verify(&ENGINE_CHECK, c, hb, hlen, np, id, hsig, vote_pks, vote_sigs,
                            nvotes, z16, index);
}

static void certificates_verify_many(const sig_engine* E, const nwo_committee* c,
                                     const uint8_t* header_bytes, const uint64_t* header_offsets,
                                     const uint32_t* payload_counts, const uint8_t* ids,
                                     const uint8_t* header_sigs, const uint64_t* vote_offsets,
                                     const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n,
                                     const uint8_t* z16, int headers_only, int32_t* status,
                                     uint64_t* index, int nthreads) {
  ensure_init();
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
  for (long i = 0; i < (long)n; ++i) {
    const uint8_t* hb = header_bytes + header_offsets[i];
    const size_t hl = header_offsets[i + 1] - header_offsets[i];
    uint64_t ix = 0;
    if (headers_only) {
      status[i] = header_verify(E, c, hb, hl, payload_counts[i], ids + 32 * i,
                                header_sigs + 64 * i, &ix);
    } else {
      const uint64_t vb = vote_offsets[i], nv = vote_offsets[i + 1] - vb;
      status[i] = certificate_verify(E, c, hb, hl, payload_counts[i], ids + 32 * i,
                                     header_sigs + 64 * i, vote_pks + 32 * vb,
                                     vote_sigs + 64 * vb, nv, z16 ? z16 + 16 * vb : NULL, &ix);
    }
    if (index) index[i] = ix;
  }
  (void)nthreads;
}

void nwo_certificates_verify_many(const nwo_committee* c, const uint8_t* header_bytes,
                                  const uint64_t* header_offsets, const uint32_t* payload_counts,
                                  const uint8_t* ids, const uint8_t* header_sigs,
                                  const uint64_t* vote_offsets, const uint8_t* vote_pks,
                                  const uint8_t* vote_sigs, size_t n, const uint8_t* z16,
                                  int headers_only, int32_t* status, uint64_t* index,
                                  int nthreads) {
  certificates_verify_many(&ENGINE_CHECK, c, header_bytes, header_offsets, payload_counts, ids,
                           header_sigs, vote_offsets, vote_pks, vote_sigs, n, z16, headers_only,
                           status, index, nthreads);
}

void nwd_certificates_verify_many(const nwo_committee* c, const uint8_t* header_bytes,
                                  const uint64_t* header_offsets, const uint32_t* payload_counts,
                                  const uint8_t* ids, const uint8_t* header_sigs,
                                  const uint64_t* vote_offsets, const uint8_t* vote_pks,
                                  const uint8_t* vote_sigs, size_t n, const uint8_t* z16,
                                  int headers_only, int32_t* status, uint64_t* index,
                                  int nthreads) {
  certificates_verify_many(&ENGINE_DALEK, c, header_bytes, header_offsets, payload_counts, ids,
                           header_sigs, vote_offsets, vote_pks, vote_sigs, n, z16, headers_only,
                           status, index, nthreads);
}

/* Vote::verify (messages.rs:131-142). */
void nwo_votes_verify_many(const nwo_committee* c, const uint8_t* ids, const uint64_t* rounds,
                           const uint8_t* origins, const uint8_t* authors, const uint8_t* sigs,
                           size_t n, int32_t* status) {
  ensure_init();
  for (size_t i = 0; i < n; ++i) {
    if (committee_stake(c, authors + 32 * i) == 0) { status[i] = NWO_DAG_UNKNOWN_AUTHORITY; continue; }
    uint8_t d[32];
    nwo_digest_72(ids + 32 * i, rounds[i], origins + 32 * i, d);
    int st = nwo_verify_strict(d, 32, authors + 32 * i, sigs + 64 * i);
    status[i] = st ? NWO_DAG_INVALID_SIGNATURE + st : 0;
  }
}
