// nw_scalar.hpp — scalars mod l = 2^252 + 27742317777372353535851937790883648493.
//
// 8 little-endian 32-bit words. Barrett reduction (HAC 14.42, b = 2^32, k = 8) of
// products up to 512 bits: curve25519-dalek Scalar::from_hash (k = H(R||A||M) mod l),
// Scalar * Scalar and Scalar + Scalar as used by verify_strict / verify_batch [ext].
#pragma once
#include "nw_field.hpp"

namespace nw {

struct sc { uint32_t w[8]; };

static constexpr uint32_t L_W[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                     0u, 0u, 0u, 0x10000000u};
// mu = floor(2^512 / l), 9 words.
static constexpr uint32_t MU_W[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du,
                                      0xffffffebu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                                      0x0000000fu};

// r (9 words) -= l if r >= l; returns whether it subtracted.
NW_HD bool sc_sub_l_if_geq9(uint32_t r[9]) {
  // r >= l ? (l has 8 words; r[8] != 0 means r > l)
  bool geq = r[8] != 0;
  if (!geq) {
    bool decided = false;
#pragma unroll
    for (int i = 7; i >= 0; --i) {
      if (!decided && r[i] != L_W[i]) { geq = r[i] > L_W[i]; decided = true; }
    }
    if (!decided) geq = true;
  }
  uint64_t borrow = 0;
  uint32_t t[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t d = (uint64_t)r[i] - (i < 8 ? L_W[i] : 0u) - borrow;
    t[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) r[i] = geq ? t[i] : r[i];
  return geq;
}

// x: 16 words (< 2^512) -> x mod l.
NW_HD void sc_reduce512(sc& out, const uint32_t x[16]) {
  // q2 = floor(x / b^7) * mu ; only words 9.. of q2 are needed, but the carries from the
  // low words matter, so compute the full product (81 MACs).
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      uint64_t t = (uint64_t)x[7 + i] * MU_W[j] + q2[i + j] + c;
      q2[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    q2[i + 9] = (uint32_t)c;
  }
  // r2 = (q3 * l) mod b^9, q3 = q2[9..17]
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i + j < 9) {
        uint64_t t = (uint64_t)q2[9 + i] * L_W[j] + r2[i + j] + c;
        r2[i + j] = (uint32_t)t;
        c = t >> 32;
      }
    }
    if (i == 0) r2[8] = (uint32_t)c;   // row 0's carry lands in word 8 (still < b^9)
  }
  uint32_t r[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  sc_sub_l_if_geq9(r);
  sc_sub_l_if_geq9(r);
#pragma unroll
  for (int i = 0; i < 8; ++i) out.w[i] = r[i];
}

// s < l (dalek check_scalar / Scalar::from_canonical_bytes).
NW_HD bool sc_is_canonical(const sc& s) {
  bool lt = false, decided = false;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    if (!decided && s.w[i] != L_W[i]) { lt = s.w[i] < L_W[i]; decided = true; }
  }
  return decided && lt;
}

// (a * b) mod l for a, b < 2^256.
NW_HD void sc_mul(sc& out, const sc& a, const sc& b) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t t = (uint64_t)a.w[i] * b.w[j] + x[i + j] + c;
      x[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    x[i + 8] = (uint32_t)c;
  }
  sc_reduce512(out, x);
}

// (a + b) mod l for a, b < l.
NW_HD void sc_add(sc& out, const sc& a, const sc& b) {
  uint32_t r[9];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.w[i] + b.w[i];
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  r[8] = (uint32_t)c;
  sc_sub_l_if_geq9(r);
#pragma unroll
  for (int i = 0; i < 8; ++i) out.w[i] = r[i];
}

// (l - a) mod l for a < l.
NW_HD void sc_neg(sc& out, const sc& a) {
  uint32_t nz = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) nz |= a.w[i];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)L_W[i] - a.w[i] - borrow;
    out.w[i] = nz ? (uint32_t)d : 0u;
    borrow = (d >> 63) & 1;
  }
}

// Signed-digit recoding without a sequential pass: for digits of width w bits in
// [-2^(w-1), 2^(w-1)), add M = sum_i 2^(w-1) * 2^(w i); digit i is then
// ((s + M) >> (w i) & (2^w - 1)) - 2^(w-1). Valid for s < 2^253 (no overflow past 256 bits).
NW_HD void sc_recode(uint32_t out[8], const sc& s, uint32_t m_word) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)s.w[i] + m_word;
    out[i] = (uint32_t)c;
    c >>= 32;
  }
}

}  // namespace nw

namespace nw {

// ---------------------------------------------------------------------------------------
// Half-size scalars for strict verification (Antipa et al., "Accelerated verification of
// ECDSA signatures", SAC 2005; Pornin, "Optimized lattice basis reduction in dimension 2,
// and fast Schnorr and EdDSA signature verification", 2020).
//
// Find (u, v) with u = v k (mod 8l), v odd, |u|, |v| ~ 2^128, by the extended Euclidean
// algorithm on (8l, k) stopped at the first remainder below 2^128. Then for ANY point D on
// the curve (group order 8l): [v] D = 0 <=> D = 0, because gcd(v, 8l) = 1 — so
//   R + [k]A - [s]B == 0   <=>   [v]R + [u]A - [v s mod l]B == 0
// exactly, torsion components included (mixed-order A keeps dalek's verify_strict
// verdict), while the shared ladder is ~128 doublings instead of 252.
//
// State: X = (xr, -xt), Y = (yr, +-yt) lattice vectors r = t k (mod 8l) with opposite-sign
// t; quotients are estimated in f64 and never overshoot. If the remainder does not drop
// below 2^128 within the iteration cap (a quotient >= 2^32 somewhere, i.e. a ground k), the
// result is the trivial vector (k, 1): correct, only slower.
// ---------------------------------------------------------------------------------------
static constexpr uint32_t L8_W[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u,
                                      0u, 0u, 0u, 0x80000000u};   // 8 l

struct sc_half {
  uint32_t u[8];    // u >= 0, u < 2^253
  uint32_t v[5];    // |v|, odd
  bool vneg;        // v < 0
};

NW_HD double bn8_to_f64(const uint32_t w[8]) {
  double d = 0.0;
#pragma unroll
  for (int i = 7; i >= 0; --i) d = d * 4294967296.0 + (double)w[i];
  return d;
}

NW_HD bool bn8_lt(const uint32_t a[8], const uint32_t b[8]) {
  // a < b  <=>  a - b borrows
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) borrow = ((uint64_t)a[i] - b[i] - borrow) >> 63;
  return borrow != 0;
}

NW_HD int bn_bits(const uint32_t* w, int n) {
  int b = 0;
  for (int i = 0; i < n; ++i)
    if (w[i]) b = 32 * i + 32 - __builtin_clz(w[i]);
  return b;
}
NW_HD bool bn_lt(const uint32_t* a, const uint32_t* b, int n) {
  uint64_t borrow = 0;
  for (int i = 0; i < n; ++i) borrow = ((uint64_t)a[i] - b[i] - borrow) >> 63;
  return borrow != 0;
}
NW_HD void bn_add(uint32_t* r, const uint32_t* a, const uint32_t* b, int n) {
  uint64_t c = 0;
  for (int i = 0; i < n; ++i) { c += (uint64_t)a[i] + b[i]; r[i] = (uint32_t)c; c >>= 32; }
}
NW_HD void bn_sub(uint32_t* r, const uint32_t* a, const uint32_t* b, int n) {
  uint64_t borrow = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t d = (uint64_t)a[i] - b[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
}
// r = a - q b (no underflow), r = a + q b
NW_HD void bn_submul(uint32_t* r, const uint32_t* a, const uint32_t* b, uint32_t q, int n) {
  uint64_t c = 0, borrow = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t p = (uint64_t)q * b[i] + c;
    c = p >> 32;
    const uint64_t d = (uint64_t)a[i] - (uint32_t)p - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
}
NW_HD void bn_addmul(uint32_t* r, const uint32_t* a, const uint32_t* b, uint32_t q, int n) {
  uint64_t c = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t p = (uint64_t)q * b[i] + a[i] + c;
    r[i] = (uint32_t)p;
    c = p >> 32;
  }
}

// floor(x / 2^s) mod 2^52 for a 256-bit x (8 LE words), 0 <= s <= 204, as an exact double.
NW_HD double bn8_bits52(const uint32_t x[8], int s) {
  const int wi = s >> 5, b = s & 31;
  uint32_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    w0 = t == wi ? x[t] : w0;
    w1 = t == wi + 1 ? x[t] : w1;
    w2 = t == wi + 2 ? x[t] : w2;
  }
  const uint64_t lo = (((uint64_t)w1 << 32) | w0) >> b;
  const uint64_t hi = b ? ((uint64_t)w2 << (64 - b)) : 0ull;
  return (double)((lo | hi) & ((1ull << 52) - 1));
}

// floor(a / b) for integers 0 <= a < 2^53, 0 < b < 2^53 held exactly in doubles.
NW_HD double f64_floor_div(double a, double b) {
  double q = floor(a / b);
  if (fma(-q, b, a) < 0.0) q -= 1.0;   // a / b rounded up to an integer
  return q;
}

// r = |pa x - pb y| for 8-word x, y and 32-bit pa, pb (the true difference fits 256 bits).
NW_HD void bn8_absdiff_mul(uint32_t r[8], const uint32_t x[8], uint32_t pa, const uint32_t y[8],
                           uint32_t pb) {
  uint64_t c1 = 0, c2 = 0, borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t p1 = (uint64_t)pa * x[i] + c1;
    const uint64_t p2 = (uint64_t)pb * y[i] + c2;
    c1 = p1 >> 32;
    c2 = p2 >> 32;
    const uint64_t d = (uint64_t)(uint32_t)p1 - (uint32_t)p2 - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  // sign of the 9-word difference: (c1 - c2 - borrow) < 0
  if ((int64_t)(c1 - c2 - borrow) < 0) {   // negative: two's-complement negation
    uint64_t c = 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (uint64_t)(uint32_t)~r[i];
      r[i] = (uint32_t)c;
      c >>= 32;
    }
  }
}

// r = pa x + pb y for 5-word x, y (the sum fits 160 bits).
NW_HD void bn5_addmul2(uint32_t r[5], const uint32_t x[5], uint32_t pa, const uint32_t y[5],
                       uint32_t pb) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint64_t p1 = (uint64_t)pa * x[i];
    const uint64_t p2 = (uint64_t)pb * y[i];
    const uint64_t s = (p1 & 0xffffffffull) + (p2 & 0xffffffffull) + (c & 0xffffffffull);
    r[i] = (uint32_t)s;
    c = (p1 >> 32) + (p2 >> 32) + (c >> 32) + (s >> 32);
  }
}

#ifndef NW_SPLIT_LEHMER
#define NW_SPLIT_LEHMER 1
#endif

// Any lane of the wave (device) / this thread (host).
NW_HD bool nw_any(bool p) {
#ifdef __HIP_DEVICE_COMPILE__
  return __ballot(p) != 0;
#else
  return p;
#endif
}

template <bool LEHMER = NW_SPLIT_LEHMER != 0>
NW_HD void sc_half_split(sc_half& out, const sc& k) {
  uint32_t xr[8], yr[8], xt[5], yt[5];
#pragma unroll
  for (int i = 0; i < 8; ++i) { xr[i] = L8_W[i]; yr[i] = k.w[i]; }
#pragma unroll
  for (int i = 0; i < 5; ++i) { xt[i] = 0; yt[i] = i == 0 ? 1u : 0u; }
  bool yneg = false, done = false;
#pragma unroll 1
  for (int it = 0; it < 400; ++it) {
    done = (yr[4] | yr[5] | yr[6] | yr[7]) == 0;
    if (done) break;
    if (LEHMER) {
    // Lehmer round (Knuth, TAOCP 4.5.2 Algorithm L): Euclid on the leading 52 bits of
    // (xr, yr) in exact double arithmetic with cofactors A B / C D, each quotient accepted
    // only when both bracketing quotients agree (so it equals the full numbers' quotient),
    // and only while the remainder stays above 2^129 (the loop must stop at the FIRST
    // remainder below 2^128, as the one-step loop does); then one multi-word update
    // (xr, yr) <- (|A xr - B yr|, |C xr - D yr|), (xt, yt) <- (|A| xt + |B| yt, ...).
    {
      const int bx = bn_bits(xr, 8);   // > 128 here
      const int sh = bx - 52;
      double x = bn8_bits52(xr, sh), y = bn8_bits52(yr, sh);
      const int le = 130 - sh > 28 ? 130 - sh : 28;
      const double lim = ldexp(1.0, le);
      double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
      int j = 0;
#pragma unroll 1
      for (int st = 0; st < 64; ++st) {
        const double yc = y + C, yd = y + D;
        if (!(yc > 0.0) || !(yd > 0.0)) break;
        const double q = f64_floor_div(x + A, yc);
        if (q != f64_floor_div(x + B, yd)) break;
        const double r = fma(-q, y, x);
        const double nC = fma(-q, C, A), nD = fma(-q, D, B);
        if (r < lim || fabs(nC) >= 2147483648.0 || fabs(nD) >= 2147483648.0) break;
        A = C; B = D; C = nC; D = nD; x = y; y = r;
        ++j;
      }
      // Lanes that made Lehmer progress update; the one-step code below runs only in an
      // iteration where no lane of the wave could (SIMT: the wave would execute both).
      const bool any_progress = nw_any(j > 0);
      if (any_progress) {
        if (j == 0) continue;
        const uint32_t a = (uint32_t)fabs(A), b = (uint32_t)fabs(B);
        const uint32_t c = (uint32_t)fabs(C), d = (uint32_t)fabs(D);
        uint32_t nx[8], ny[8], nxt[5], nyt[5];
        bn8_absdiff_mul(nx, xr, a, yr, b);
        bn8_absdiff_mul(ny, xr, c, yr, d);
        bn5_addmul2(nxt, xt, a, yt, b);
        bn5_addmul2(nyt, xt, c, yt, d);
#pragma unroll
        for (int i = 0; i < 8; ++i) { xr[i] = nx[i]; yr[i] = ny[i]; }
#pragma unroll
        for (int i = 0; i < 5; ++i) { xt[i] = nxt[i]; yt[i] = nyt[i]; }
        yneg = (j & 1) ? !yneg : yneg;
        continue;
      }
    }
    }
    // q <= floor(xr / yr): relative error of the f64 quotient < 2^-49.
    const double qd = floor(bn8_to_f64(xr) / bn8_to_f64(yr) * (1.0 - 0x1p-46));
    const uint32_t q = qd >= 4294967295.0 ? 0xffffffffu : (qd < 1.0 ? 1u : (uint32_t)qd);
    // xr -= q yr (never negative), xt += q yt
    uint64_t c = 0, borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t p = (uint64_t)q * yr[i] + c;
      c = p >> 32;
      const uint64_t d = (uint64_t)xr[i] - (uint32_t)p - borrow;
      xr[i] = (uint32_t)d;
      borrow = (d >> 63) & 1;
    }
    c = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const uint64_t p = (uint64_t)q * yt[i] + xt[i] + c;
      xt[i] = (uint32_t)p;
      c = p >> 32;
    }
    if (bn8_lt(xr, yr)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { const uint32_t t = xr[i]; xr[i] = yr[i]; yr[i] = t; }
#pragma unroll
      for (int i = 0; i < 5; ++i) { const uint32_t t = xt[i]; xt[i] = yt[i]; yt[i] = t; }
      yneg = !yneg;
    }
  }
  if (done && (yt[0] & 1u)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) out.u[i] = yr[i];
#pragma unroll
    for (int i = 0; i < 5; ++i) out.v[i] = yt[i];
    out.vneg = yneg;
  } else if (done) {
    // Y's t is even, so X's is odd (consecutive cofactors are coprime) and every vector
    // X + a Y has an odd t. Take the shortest (max bit length of u, |v|) of X - Y, X + Y,
    // Z = X - q Y, Z + Y, Y - Z (q <= floor(xr / yr) as in the loop).
    int best = 1 << 30;
    uint32_t r[8], t[5];
    auto consider = [&](bool neg) {
      const int m = bn_bits(r, 8) > bn_bits(t, 5) ? bn_bits(r, 8) : bn_bits(t, 5);
      if (m < best) {
        best = m;
#pragma unroll
        for (int i = 0; i < 8; ++i) out.u[i] = r[i];
#pragma unroll
        for (int i = 0; i < 5; ++i) out.v[i] = t[i];
        out.vneg = neg;
      }
    };
    bn_sub(r, xr, yr, 8);  bn_add(t, xt, yt, 5);  consider(!yneg);              // X - Y
    bn_add(r, xr, yr, 8);                                                       // X + Y
    const bool y_ge_x = !bn_lt(yt, xt, 5);
    if (y_ge_x) bn_sub(t, yt, xt, 5); else bn_sub(t, xt, yt, 5);
    consider(y_ge_x ? yneg : !yneg);
    if (yr[0] | yr[1] | yr[2] | yr[3]) {
      const double qd = floor(bn8_to_f64(xr) / bn8_to_f64(yr) * (1.0 - 0x1p-46));
      const uint32_t q = qd >= 4294967295.0 ? 0xffffffffu : (qd < 1.0 ? 1u : (uint32_t)qd);
      uint32_t zr[8], zt[5];
      bn_submul(zr, xr, yr, q, 8);                                              // Z
      bn_addmul(zt, xt, yt, q, 5);
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = zr[i];
#pragma unroll
      for (int i = 0; i < 5; ++i) t[i] = zt[i];
      consider(!yneg);
      bn_add(r, zr, yr, 8);  bn_sub(t, zt, yt, 5);  consider(!yneg);            // Z + Y
      if (bn_lt(zr, yr, 8)) {                                                   // Y - Z
        bn_sub(r, yr, zr, 8);  bn_add(t, zt, yt, 5);  consider(yneg);
      }
    }
  }
  // Fallback (iteration cap, or u >= 2^252 / |v| >= 2^160): the trivial vector (k, 1).
  if (!done || (out.u[7] >> 28) != 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) out.u[i] = k.w[i];
#pragma unroll
    for (int i = 0; i < 5; ++i) out.v[i] = i == 0 ? 1u : 0u;
    out.vneg = false;
  }
}

}  // namespace nw
