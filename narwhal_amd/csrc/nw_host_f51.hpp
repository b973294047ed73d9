// nw_host_f51.hpp — GF(2^255 - 19) in five 51-bit limbs for the host path's comb checks
// (nw_host.cpp comb_sum / vote_check / verify_strict_keyed). The device kernels' radix-2^25.5
// form (nw_field.hpp) costs the CPU 100 32x32 products per field product; here a product is
// 25 64x64->128 ones (x86-64 MUL / MULX), about 3x fewer cycles. Host only: the kernels never
// include this file. Tables are converted from the radix-2^25.5 entries through their
// canonical bytes, so both forms hold the same field elements.
//
// Limb bounds: a "loose" element has limbs < 2^52 (every product, square and carried sum);
// inputs of mul / sq may have limbs up to 2^54 (sums and biased differences of loose ones):
// each 128-bit column then stays below 5 * 19 * 2^108 < 2^115, and the carries run in 128
// bits, so nothing overflows.
#pragma once
#include <stdint.h>
#include <string.h>

namespace nw {
namespace host {
namespace f51 {

typedef unsigned __int128 u128;
constexpr uint64_t kM = (1ull << 51) - 1;

struct fe { uint64_t v[5]; };
struct niels { fe ypx, ymx, xy2d; };   // affine (y + x, y - x, 2 d x y)
struct pt { fe X, Y, Z, T; };          // extended (X : Y : Z : T)

inline void fe_0(fe& h) { h = fe{{0, 0, 0, 0, 0}}; }
inline void fe_1(fe& h) { h = fe{{1, 0, 0, 0, 0}}; }

inline void add(fe& h, const fe& f, const fe& g) {
  for (int i = 0; i < 5; ++i) h.v[i] = f.v[i] + g.v[i];
}
// h = f - g + 4p (g loose: limbs < 2^52 < 4p's), limbs < 2^54
inline void sub(fe& h, const fe& f, const fe& g) {
  h.v[0] = f.v[0] + ((kM - 18) << 2) - g.v[0];
  for (int i = 1; i < 5; ++i) h.v[i] = f.v[i] + (kM << 2) - g.v[i];
}

inline void carry128(fe& h, u128 r0, u128 r1, u128 r2, u128 r3, u128 r4) {
  r1 += (uint64_t)(r0 >> 51);
  r2 += (uint64_t)(r1 >> 51);
  r3 += (uint64_t)(r2 >> 51);
  r4 += (uint64_t)(r3 >> 51);
  const u128 c = r4 >> 51;
  u128 t0 = (u128)((uint64_t)r0 & kM) + c * 19;
  h.v[0] = (uint64_t)t0 & kM;
  h.v[1] = ((uint64_t)r1 & kM) + (uint64_t)(t0 >> 51);
  h.v[2] = (uint64_t)r2 & kM;
  h.v[3] = (uint64_t)r3 & kM;
  h.v[4] = (uint64_t)r4 & kM;
}

inline void mul(fe& h, const fe& f, const fe& g) {
  const uint64_t a0 = f.v[0], a1 = f.v[1], a2 = f.v[2], a3 = f.v[3], a4 = f.v[4];
  const uint64_t b0 = g.v[0], b1 = g.v[1], b2 = g.v[2], b3 = g.v[3], b4 = g.v[4];
  const uint64_t b1n = 19 * b1, b2n = 19 * b2, b3n = 19 * b3, b4n = 19 * b4;   // < 2^59
  const u128 r0 = (u128)a0 * b0 + (u128)a1 * b4n + (u128)a2 * b3n + (u128)a3 * b2n + (u128)a4 * b1n;
  const u128 r1 = (u128)a0 * b1 + (u128)a1 * b0 + (u128)a2 * b4n + (u128)a3 * b3n + (u128)a4 * b2n;
  const u128 r2 = (u128)a0 * b2 + (u128)a1 * b1 + (u128)a2 * b0 + (u128)a3 * b4n + (u128)a4 * b3n;
  const u128 r3 = (u128)a0 * b3 + (u128)a1 * b2 + (u128)a2 * b1 + (u128)a3 * b0 + (u128)a4 * b4n;
  const u128 r4 = (u128)a0 * b4 + (u128)a1 * b3 + (u128)a2 * b2 + (u128)a3 * b1 + (u128)a4 * b0;
  carry128(h, r0, r1, r2, r3, r4);
}

inline void sq(fe& h, const fe& f) {
  const uint64_t a0 = f.v[0], a1 = f.v[1], a2 = f.v[2], a3 = f.v[3], a4 = f.v[4];
  const uint64_t d0 = 2 * a0, d1 = 2 * a1, d2 = 2 * a2;
  const uint64_t a3n = 19 * a3, a4n = 19 * a4;
  const u128 r0 = (u128)a0 * a0 + (u128)d1 * a4n + (u128)d2 * a3n;
  const u128 r1 = (u128)d0 * a1 + (u128)d2 * a4n + (u128)a3 * a3n;
  const u128 r2 = (u128)d0 * a2 + (u128)a1 * a1 + (u128)(2 * a3) * a4n;
  const u128 r3 = (u128)d0 * a3 + (u128)d1 * a2 + (u128)a4 * a4n;
  const u128 r4 = (u128)d0 * a4 + (u128)d1 * a3 + (u128)a2 * a2;
  carry128(h, r0, r1, r2, r3, r4);
}

inline void frombytes(fe& h, const uint8_t s[32]) {   // bit 255 ignored
  uint64_t w[4];
  memcpy(w, s, 32);
  h.v[0] = w[0] & kM;
  h.v[1] = (w[0] >> 51 | w[1] << 13) & kM;
  h.v[2] = (w[1] >> 38 | w[2] << 26) & kM;
  h.v[3] = (w[2] >> 25 | w[3] << 39) & kM;
  h.v[4] = (w[3] >> 12) & kM;
}

// canonical little-endian bytes (limbs < 2^54 accepted)
inline void tobytes(uint8_t s[32], const fe& f) {
  uint64_t t[5];
  memcpy(t, f.v, sizeof t);
  for (int pass = 0; pass < 2; ++pass) {   // carry to limbs < 2^51, value < 2^255 + small
    for (int i = 0; i < 4; ++i) {
      t[i + 1] += t[i] >> 51;
      t[i] &= kM;
    }
    t[0] += 19 * (t[4] >> 51);
    t[4] &= kM;
  }
  // now t < 2^255 + 19 * small; subtract p if t >= p: q = (t + 19) >> 255
  uint64_t q = (t[0] + 19) >> 51;
  q = (t[1] + q) >> 51;
  q = (t[2] + q) >> 51;
  q = (t[3] + q) >> 51;
  q = (t[4] + q) >> 51;
  t[0] += 19 * q;
  for (int i = 0; i < 4; ++i) {
    t[i + 1] += t[i] >> 51;
    t[i] &= kM;
  }
  t[4] &= kM;
  const uint64_t w0 = t[0] | t[1] << 51, w1 = t[1] >> 13 | t[2] << 38, w2 = t[2] >> 26 | t[3] << 25,
                 w3 = t[3] >> 39 | t[4] << 12;
  memcpy(s, &w0, 8);
  memcpy(s + 8, &w1, 8);
  memcpy(s + 16, &w2, 8);
  memcpy(s + 24, &w3, 8);
}

inline bool eq(const fe& f, const fe& g) {
  uint8_t a[32], b[32];
  tobytes(a, f);
  tobytes(b, g);
  return memcmp(a, b, 32) == 0;
}
inline bool iszero(const fe& f) {
  uint8_t a[32];
  tobytes(a, f);
  uint8_t o = 0;
  for (int i = 0; i < 32; ++i) o |= a[i];
  return o == 0;
}
inline uint32_t isnegative(const fe& f) {
  uint8_t a[32];
  tobytes(a, f);
  return a[0] & 1u;
}

// f^(p - 2): 254 squarings, 11 products (the usual addition chain of 2^255 - 21)
inline void sqn(fe& h, const fe& f, int n) {
  sq(h, f);
  for (int i = 1; i < n; ++i) sq(h, h);
}
inline void invert(fe& out, const fe& z) {
  fe z2, z9, z11, z2_5_0, z2_10_0, z2_20_0, z2_50_0, z2_100_0, t;
  sq(z2, z);                    // 2
  sqn(t, z2, 2);                // 8
  mul(z9, t, z);                // 9
  mul(z11, z9, z2);             // 11
  sq(t, z11);                   // 22
  mul(z2_5_0, t, z9);           // 2^5 - 1
  sqn(t, z2_5_0, 5);
  mul(z2_10_0, t, z2_5_0);      // 2^10 - 1
  sqn(t, z2_10_0, 10);
  mul(z2_20_0, t, z2_10_0);     // 2^20 - 1
  sqn(t, z2_20_0, 20);
  mul(t, t, z2_20_0);           // 2^40 - 1
  sqn(t, t, 10);
  mul(z2_50_0, t, z2_10_0);     // 2^50 - 1
  sqn(t, z2_50_0, 50);
  mul(z2_100_0, t, z2_50_0);    // 2^100 - 1
  sqn(t, z2_100_0, 100);
  mul(t, t, z2_100_0);          // 2^200 - 1
  sqn(t, t, 50);
  mul(t, t, z2_50_0);           // 2^250 - 1
  sqn(t, t, 5);                 // 2^255 - 2^5
  mul(out, t, z11);             // 2^255 - 21
}

inline void pt_identity(pt& p) { fe_0(p.X); fe_1(p.Y); fe_1(p.Z); fe_0(p.T); }

inline void niels_cneg(niels& n, bool neg) {
  if (!neg) return;
  const fe t = n.ypx;
  n.ypx = n.ymx;
  n.ymx = t;
  fe z;
  fe_0(z);
  sub(n.xy2d, z, n.xy2d);
}

// r = p + q, q affine niels (add-2008-hwcd-3 with Z2 = 1; the same formula as nw_point.hpp
// ge_add_niels)
inline void add_niels(pt& r, const pt& p, const niels& q) {
  fe a, b, c, d, e, f, g, h;
  sub(a, p.Y, p.X);
  mul(a, a, q.ymx);
  add(b, p.Y, p.X);
  mul(b, b, q.ypx);
  mul(c, q.xy2d, p.T);
  add(d, p.Z, p.Z);
  sub(e, b, a);
  sub(f, d, c);
  add(g, d, c);
  add(h, b, a);
  mul(r.X, e, f);
  mul(r.Z, g, f);
  mul(r.Y, g, h);
  mul(r.T, e, h);
}

}  // namespace f51
}  // namespace host
}  // namespace nw
