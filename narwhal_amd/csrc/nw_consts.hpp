// nw_consts.hpp — curve constants and the fixed-base table, derived from their
// definitions (d = -121665/121666, sqrt(-1) = 2^((p-1)/4), B = (x >= 0, 4/5)) with the same
// arithmetic the kernels use. Computed once on the host and uploaded to constant memory.
#pragma once
#include "nw_strict.hpp"

namespace nw {

NW_HD void fe_from_u32(fe& h, uint32_t x) {
  fe_0(h);
  h.v[0] = x & M26;
  h.v[1] = x >> 26;
}

// tab[j] = j * P for j = 0..128 (affine niels).
inline void niels_multiples(ge_niels tab[129], const ge& P, const fe& d2) {
  ge_niels_identity(tab[0]);
  ge_cached cP;
  ge_to_cached(cP, P, d2);
  ge acc = P;
  for (int j = 1; j <= 128; ++j) {
    ge_to_niels(tab[j], acc, d2);
    ge nxt;
    ge_add_cached(nxt, acc, cP, true);
    acc = nxt;
  }
}

// btab[j] = j * B for j = 0..128 (affine niels).
inline void compute_consts(curve_consts& k, ge_niels btab[129]) {
  fe a, b, t, two;
  fe_from_u32(a, 121665);
  fe_neg(a, a);
  fe_from_u32(b, 121666);
  fe_invert(t, b);
  fe_mul(k.d, a, t);
  fe_add(k.d2, k.d, k.d);
  fe_carry(k.d2);
  fe_from_u32(two, 2);
  fe_pow22523(t, two);   // 2^((p-5)/8)
  fe_sq(a, t);
  fe_mul(k.sqrtm1, a, two);   // 2^((p-1)/4)
  fe_from_u32(a, 4);
  fe_from_u32(b, 5);
  fe_invert(t, b);
  fe_mul(a, a, t);
  uint32_t yw[8];
  fe_tobytes(yw, a);
  ge B;
  ge_frombytes(B, yw, k);
  ge_niels_identity(btab[0]);
  ge_cached cB;
  ge_to_cached(cB, B, k.d2);
  ge acc = B;
  for (int j = 1; j <= 128; ++j) {
    ge_to_niels(btab[j], acc, k.d2);
    ge nxt;
    ge_add_cached(nxt, acc, cB, true);
    acc = nxt;
  }
}

// The 128-bit half-size verification constants (nw_strict.hpp): canonical y of the small-
// order points, and b128[j] = j * 2^128 B.
inline void compute_strict_consts(strict_consts& sk, ge_niels b128[129]) {
  ge_niels btab[129];
  compute_consts(sk.k, btab);
  static const uint8_t y8_enc[32] = {0x26, 0xe8, 0x95, 0x8f, 0xc2, 0xb2, 0x27, 0xb0,
                                     0x45, 0xc3, 0xf4, 0x89, 0xf2, 0xef, 0x98, 0xf0,
                                     0xd5, 0xdf, 0xac, 0x05, 0xd3, 0xc6, 0x33, 0x39,
                                     0xb1, 0x38, 0x02, 0x88, 0x6d, 0x53, 0xfc, 0x05};
  uint32_t w[8];
  for (int i = 0; i < 8; ++i)
    w[i] = (uint32_t)y8_enc[4 * i] | ((uint32_t)y8_enc[4 * i + 1] << 8) |
           ((uint32_t)y8_enc[4 * i + 2] << 16) | ((uint32_t)y8_enc[4 * i + 3] << 24);
  fe y8, t, one;
  fe_frombytes(y8, w);
  fe_0(t);
  fe_canonical(sk.small_y[0], t);                 // y = 0 (order 4)
  fe_1(one);
  fe_canonical(sk.small_y[1], one);               // identity
  fe_neg(t, one);
  fe_canonical(sk.small_y[2], t);                 // order 2
  fe_canonical(sk.small_y[3], y8);                // order 8
  fe_neg(t, y8);
  fe_canonical(sk.small_y[4], t);                 // order 8
  // B = (x >= 0, 4/5); B128 = 2^128 B
  fe a, b;
  fe_from_u32(a, 4);
  fe_from_u32(b, 5);
  fe_invert(t, b);
  fe_mul(a, a, t);
  uint32_t yw[8];
  fe_tobytes(yw, a);
  ge B;
  ge_frombytes(B, yw, sk.k);
  for (int i = 0; i < 128; ++i) {
    ge d;
    ge_dbl(d, B, true);
    B = d;
  }
  niels_multiples(b128, B, sk.k.d2);
}

// torsion_consts (nw_strict.hpp): affine [j] T8, j = 0..7, T8 = decompress(y8, sign 0).
inline void compute_torsion(torsion_consts& tc) {
  curve_consts k;
  ge_niels btab[129];
  compute_consts(k, btab);
  static const uint8_t y8_enc[32] = {0x26, 0xe8, 0x95, 0x8f, 0xc2, 0xb2, 0x27, 0xb0,
                                     0x45, 0xc3, 0xf4, 0x89, 0xf2, 0xef, 0x98, 0xf0,
                                     0xd5, 0xdf, 0xac, 0x05, 0xd3, 0xc6, 0x33, 0x39,
                                     0xb1, 0x38, 0x02, 0x88, 0x6d, 0x53, 0xfc, 0x05};
  uint32_t w[8];
  for (int i = 0; i < 8; ++i)
    w[i] = (uint32_t)y8_enc[4 * i] | ((uint32_t)y8_enc[4 * i + 1] << 8) |
           ((uint32_t)y8_enc[4 * i + 2] << 16) | ((uint32_t)y8_enc[4 * i + 3] << 24);
  ge T8, acc;
  ge_frombytes(T8, w, k);
  ge_cached c8;
  ge_to_cached(c8, T8, k.d2);
  ge_identity(acc);
  for (int j = 0; j < 8; ++j) {
    fe zi, t;
    fe_invert(zi, acc.Z);
    fe_mul(t, acc.X, zi);
    fe_canonical(tc.x[j], t);
    fe_mul(t, acc.Y, zi);
    fe_canonical(tc.y[j], t);
    ge nxt;
    ge_add_cached(nxt, acc, c8, true);
    acc = nxt;
  }
}

}  // namespace nw

namespace nw {
// Affine niels form of p given zi = 1/Z.
inline void ge_to_niels_zi(ge_niels& n, const ge& p, const fe& zi, const fe& d2) {
  fe x, y;
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_add(n.ypx, y, x); fe_carry(n.ypx);
  fe_sub(n.ymx, y, x);
  fe_mul(n.xy2d, x, y);
  fe_mul(n.xy2d, n.xy2d, d2);
}

// The strict kernel's wide B tables (nw_strict.hpp, signed bw-bit windows of w = w0 +
// 2^128 w1): out[h * n + j] = j * 2^(128 h) * B, j = 0..n-1, n = 2^(bw-1) + 1, h = 0, 1,
// in padded affine niels form (128 B entries). j * P by repeated addition, the 2n
// inversions batched into one (Montgomery's trick). bw = 16: 2 x 32,769 entries, 8.4 MB.
inline void compute_wide_btab(ge_niels_pad* out, int bw) {
  const uint32_t n = (1u << (bw - 1)) + 1;
  strict_consts sk;
  ge_niels b128[129];
  compute_strict_consts(sk, b128);
  fe a, b, t;
  fe_from_u32(a, 4);
  fe_from_u32(b, 5);
  fe_invert(t, b);
  fe_mul(a, a, t);
  uint32_t yw[8];
  fe_tobytes(yw, a);
  ge P;
  ge_frombytes(P, yw, sk.k);   // B
  ge* pts = new ge[n];
  fe* pre = new fe[n];
  for (int h = 0; h < 2; ++h) {
    if (h == 1)
      for (int i = 0; i < 128; ++i) { ge d; ge_dbl(d, P, true); P = d; }   // 2^128 B
    ge_cached cP;
    ge_to_cached(cP, P, sk.k.d2);
    pts[1] = P;
    for (uint32_t j = 2; j < n; ++j) ge_add_cached(pts[j], pts[j - 1], cP, true);
    fe_1(pre[0]);
    for (uint32_t j = 1; j < n; ++j) fe_mul(pre[j], pre[j - 1], pts[j].Z);
    fe inv;
    fe_invert(inv, pre[n - 1]);
    ge_niels_pad* o = out + (size_t)h * n;
    for (uint32_t j = n - 1; j >= 1; --j) {
      fe zi;
      fe_mul(zi, inv, pre[j - 1]);   // 1 / Z_j
      fe_mul(inv, inv, pts[j].Z);    // 1 / (Z_1 ... Z_{j-1})
      ge_to_niels_zi(o[j].n, pts[j], zi, sk.k.d2);
      o[j].pad[0] = o[j].pad[1] = 0;
    }
    ge_niels_identity(o[0].n);
    o[0].pad[0] = o[0].pad[1] = 0;
  }
  delete[] pts;
  delete[] pre;
}

// Fixed-base comb for [b]B with signed 8-bit digits and no doublings:
// comb[w * 129 + j] = j * 2^(8 w) * B, w = 0..31, j = 0..128 (affine niels), 495 KB.
inline void compute_comb(ge_niels* comb) {
  curve_consts k;
  ge_niels btab[129];
  compute_consts(k, btab);
  fe a, b, t;
  fe_from_u32(a, 4);
  fe_from_u32(b, 5);
  fe_invert(t, b);
  fe_mul(a, a, t);
  uint32_t yw[8];
  fe_tobytes(yw, a);
  ge base;
  ge_frombytes(base, yw, k);   // B
  for (int w = 0; w < 32; ++w) {
    ge_niels_identity(comb[w * 129]);
    ge_cached cb;
    ge_to_cached(cb, base, k.d2);
    ge acc = base;
    for (int j = 1; j <= 128; ++j) {
      ge_to_niels(comb[w * 129 + j], acc, k.d2);
      ge nxt;
      ge_add_cached(nxt, acc, cb, true);
      acc = nxt;
    }
    for (int d = 0; d < 8; ++d) ge_dbl(base, base, d == 7);   // 2^(8(w+1)) B
  }
}
}  // namespace nw
