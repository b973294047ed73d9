// nw_point.hpp — edwards25519 (-x^2 + y^2 = 1 + d x^2 y^2) group law on gfx950.
//
// Extended coordinates (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z. Unified add-2008-hwcd-3
// (complete for this curve: also valid for doubling and the identity) and dbl-2008-hwcd,
// the same formulas curve25519-dalek uses [ext]. Table entries are kept in "cached"
// (Y+X, Y-X, 2Z, 2dT) or affine "niels" (y+x, y-x, 2dxy) form so one addition is 8 / 7
// field multiplications.
#pragma once
#include "nw_field.hpp"

namespace nw {

struct ge { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z2, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };
// 128-byte entry of a large table in global memory (eight aligned 16-byte loads).
struct alignas(16) ge_niels_pad { ge_niels n; uint32_t pad[2]; };

// Field constants (derived on the host at init from their definitions; see nw_api.cpp).
struct curve_consts {
  fe d;        // -121665/121666
  fe d2;       // 2d
  fe sqrtm1;   // 2^((p-1)/4)
};

NW_HD void ge_identity(ge& p) { fe_0(p.X); fe_1(p.Y); fe_1(p.Z); fe_0(p.T); }
NW_HD void ge_cached_identity(ge_cached& c) {
  fe_1(c.YpX); fe_1(c.YmX); fe_0(c.Z2); c.Z2.v[0] = 2; fe_0(c.T2d);
}
NW_HD void ge_niels_identity(ge_niels& n) { fe_1(n.ypx); fe_1(n.ymx); fe_0(n.xy2d); }

NW_HD void ge_to_cached(ge_cached& c, const ge& p, const fe& d2) {
  fe_add(c.YpX, p.Y, p.X); fe_carry(c.YpX);
  fe_sub(c.YmX, p.Y, p.X);
  fe_add(c.Z2, p.Z, p.Z); fe_carry(c.Z2);
  fe_mul(c.T2d, p.T, d2);
}

// Uncarried differences (fe_sub_nc) are used only as the FIRST fe_mul operand (the second
// is multiplied by 19 in 32 bits and must stay carried); tests/test_field_bounds.py checks
// every (first, second) operand pair below. The output products are ordered so that two
// share each second operand (f, h) and two each first one (e, g): the inlined multiplies
// then compute each operand's x19 / x2 limb scalings once (CSE), not twice.

// r = p + q (q cached). Computes T3 only when want_t.
NW_HD void ge_add_cached(ge& r, const ge& p, const ge_cached& q, bool want_t) {
  fe a, b, c, d, e, f, g, h;
  fe_sub_nc(a, p.Y, p.X);
  fe_mul(a, a, q.YmX);
  fe_add(b, p.Y, p.X);
  fe_mul(b, b, q.YpX);
  fe_mul(c, q.T2d, p.T);
  fe_mul(d, p.Z, q.Z2);
  fe_sub_nc(e, b, a);
  fe_sub(f, d, c);
  fe_add(g, d, c);
  fe_add(h, b, a);
  fe_mul(r.X, e, f);
  fe_mul(r.Z, g, f);
  fe_mul(r.Y, g, h);
  if (want_t) fe_mul(r.T, e, h);
}

// r = p - q (q cached): swap YpX/YmX and negate 2dT.
NW_HD void ge_sub_cached(ge& r, const ge& p, const ge_cached& q, bool want_t) {
  fe a, b, c, d, e, f, g, h;
  fe_sub_nc(a, p.Y, p.X);
  fe_mul(a, a, q.YpX);
  fe_add(b, p.Y, p.X);
  fe_mul(b, b, q.YmX);
  fe_mul(c, q.T2d, p.T);
  fe_mul(d, p.Z, q.Z2);
  fe_sub_nc(e, b, a);
  fe_add(f, d, c);
  fe_sub_nc(g, d, c);
  fe_add(h, b, a);
  fe_mul(r.X, e, f);
  fe_mul(r.Z, g, f);
  fe_mul(r.Y, g, h);
  if (want_t) fe_mul(r.T, e, h);
}

// r = p + q (q affine niels, Z = 1).
NW_HD void ge_add_niels(ge& r, const ge& p, const ge_niels& q, bool want_t) {
  fe a, b, c, d, e, f, g, h;
  fe_sub_nc(a, p.Y, p.X);
  fe_mul(a, a, q.ymx);
  fe_add(b, p.Y, p.X);
  fe_mul(b, b, q.ypx);
  fe_mul(c, q.xy2d, p.T);
  fe_add(d, p.Z, p.Z);
  fe_sub_nc(e, b, a);
  fe_sub(f, d, c);
  fe_add(g, d, c);
  fe_add(h, b, a);
  fe_mul(r.X, e, f);
  fe_mul(r.Z, g, f);
  fe_mul(r.Y, g, h);
  if (want_t) fe_mul(r.T, e, h);
}

// r = p + q, q either cached or (affine, wave-uniform) an affine niels point held in cached
// form (q.Z2 unused: 2 Z1 Z2 = 2 Z1). One routine for every ladder term. T3 only when
// want_t (wave-uniform): the doublings that follow a window's last addition never read T.
NW_HD void ge_add_any(ge& r, const ge& p, const ge_cached& q, bool affine, bool want_t = true) {
  fe a, b, c, d, e, f, g, h;
  fe_sub_nc(a, p.Y, p.X);
  fe_mul(a, a, q.YmX);
  fe_add(b, p.Y, p.X);
  fe_mul(b, b, q.YpX);
  fe_mul(c, q.T2d, p.T);
  if (affine) fe_add(d, p.Z, p.Z);
  else fe_mul(d, p.Z, q.Z2);
  fe_sub_nc(e, b, a);
  fe_sub(f, d, c);
  fe_add(g, d, c);
  fe_add(h, b, a);
  fe_mul(r.X, e, f);
  fe_mul(r.Z, g, f);
  fe_mul(r.Y, g, h);
  if (want_t) fe_mul(r.T, e, h);
}

// ge_add_any with q's 2dT NEGATED by the caller (q = (Y+X, Y-X, 2Z, -2dT)): c' = -2dT T1,
// so f = d + c' and g = d - c' need no carry pass (f <= L / P15 is the second operand of its
// products, g = S(d) the first; every pair is one tests/test_field_bounds.py checks). The
// ladder's sign selection already negates 2dT conditionally, so flipping its condition makes
// this free (NW_ADD_NEGC).
NW_HD void ge_add_any_negc(ge& r, const ge& p, const ge_cached& q, bool affine,
                           bool want_t = true) {
  fe a, b, c, d, e, f, g, h;
  fe_sub_nc(a, p.Y, p.X);
  fe_mul(a, a, q.YmX);
  fe_add(b, p.Y, p.X);
  fe_mul(b, b, q.YpX);
  fe_mul(c, q.T2d, p.T);
  if (affine) fe_add(d, p.Z, p.Z);
  else fe_mul(d, p.Z, q.Z2);
  fe_sub_nc(e, b, a);
  fe_add(f, d, c);
  fe_sub_nc(g, d, c);
  fe_add(h, b, a);
  fe_mul(r.X, e, f);
  fe_mul(r.Z, g, f);
  fe_mul(r.Y, g, h);
  if (want_t) fe_mul(r.T, e, h);
}

// Conditionally negate a niels point: -(x, y) = (-x, y) -> swap y+x / y-x, negate 2dxy.
NW_HD void ge_niels_cneg(ge_niels& n, bool neg) {
  fe t;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t a = n.ypx.v[i], b = n.ymx.v[i];
    n.ypx.v[i] = neg ? b : a;
    n.ymx.v[i] = neg ? a : b;
  }
  fe_neg_nc(t, n.xy2d);
  fe_cmov(n.xy2d, t, neg);
}
NW_HD void ge_cached_cneg(ge_cached& c, bool neg) {
  fe t;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t a = c.YpX.v[i], b = c.YmX.v[i];
    c.YpX.v[i] = neg ? b : a;
    c.YmX.v[i] = neg ? a : b;
  }
  fe_neg_nc(t, c.T2d);
  fe_cmov(c.T2d, t, neg);
}
// ge_cached_cneg for ge_add_any_negc: +-q with its 2dT negated (Y+X / Y-X swapped when neg,
// 2dT negated when NOT neg)
NW_HD void ge_cached_cneg_negc(ge_cached& c, bool neg) {
  fe t;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t a = c.YpX.v[i], b = c.YmX.v[i];
    c.YpX.v[i] = neg ? b : a;
    c.YmX.v[i] = neg ? a : b;
  }
  fe_neg_nc(t, c.T2d);
  fe_cmov(c.T2d, t, !neg);
}

// r = 2p (dbl-2008-hwcd, a = -1, with E, G, H negated so every operand stays non-negative:
// E' = (A+B) - (X+Y)^2, G' = A - B, F' = G' + 2Z^2, H' = A + B; X3 = E'F', Y3 = G'H',
// Z3 = G'F', T3 = E'H').
NW_HD void ge_dbl(ge& r, const ge& p, bool want_t) {
  fe A, B, C, E, F, G, H, t;
  fe_sq(A, p.X);
  fe_sq(B, p.Y);
  fe_sq(C, p.Z);
  fe_add(C, C, C);
  fe_add(H, A, B);
  fe_add(t, p.X, p.Y);
  fe_sq(t, t);
  fe_sub_nc(E, H, t);
  fe_sub(G, A, B);
  fe_add(F, G, C);
  fe_mul(r.X, E, F);
  fe_mul(r.Z, G, F);
  fe_mul(r.Y, G, H);
  if (want_t) fe_mul(r.T, E, H);
}

NW_HD void ge_neg(ge& r, const ge& p) {
  fe_neg(r.X, p.X); fe_copy(r.Y, p.Y); fe_copy(r.Z, p.Z); fe_neg(r.T, p.T);
}

// curve25519-dalek EdwardsPoint::is_identity: X == 0 and Y == Z (projective).
NW_HD bool ge_is_identity(const ge& p) { return fe_iszero(p.X) && fe_eq(p.Y, p.Z); }

// 8P == identity (mul_by_cofactor then is_identity).
NW_HD bool ge_is_small_order(const ge& p) {
  ge t;
  ge_dbl(t, p, false);
  ge_dbl(t, t, false);
  ge_dbl(t, t, false);
  return ge_is_identity(t);
}

// Projective equality against an affine point q (q.Z == 1): X_p == x_q Z_p, Y_p == y_q Z_p.
NW_HD bool ge_eq_affine(const ge& p, const ge& q) {
  fe a;
  fe_mul(a, q.X, p.Z);
  if (!fe_eq(a, p.X)) return false;
  fe_mul(a, q.Y, p.Z);
  return fe_eq(a, p.Y);
}

// Register barrier: the optimiser may not move computation on f across this point (device
// only). Used to keep work that follows a long exponentiation from being hoisted above it
// and held (spilled) across its loop.
NW_HD void fe_barrier(fe& f) {
#ifdef __HIP_DEVICE_COMPILE__
#pragma unroll
  for (int i = 0; i < 10; ++i) asm volatile("" : "+v"(f.v[i]));
#else
  (void)f;
#endif
}

// The last step of curve25519-dalek FieldElement::sqrt_ratio_i -> (was_nonzero_square,
// non-negative r), given t = (u v^7)^((p-5)/8).
NW_HD bool fe_sqrt_ratio_finish(fe& r, const fe& u, const fe& v, const fe& t,
                                const curve_consts& k) {
  fe v3, uv3, check, neg_u, neg_u_i, r_prime, x;
  fe_sq(x, v);  fe_mul(v3, x, v);
  fe_mul(uv3, u, v3);
  fe_mul(r, uv3, t);
  fe_sq(x, r);
  fe_mul(check, v, x);
  fe_neg(neg_u, u);
  fe_mul(neg_u_i, neg_u, k.sqrtm1);
  bool correct = fe_eq(check, u);
  bool flipped = fe_eq(check, neg_u);
  bool flipped_i = fe_eq(check, neg_u_i);
  fe_mul(r_prime, k.sqrtm1, r);
  fe_cmov(r, r_prime, flipped || flipped_i);
  fe_neg(x, r);
  fe_cmov(r, x, fe_isnegative(r) != 0);
  return correct || flipped;
}

// curve25519-dalek FieldElement::sqrt_ratio_i -> (was_nonzero_square, non-negative r).
NW_HD bool fe_sqrt_ratio_i(fe& r, const fe& u, const fe& v, const curve_consts& k) {
  fe v3, v7, t, uv7;
  fe_sq(t, v);  fe_mul(v3, t, v);
  fe_sq(t, v3); fe_mul(v7, t, v);
  fe_mul(uv7, u, v7);
  fe_pow22523(t, uv7);
  return fe_sqrt_ratio_finish(r, u, v, t, k);
}

// u = y^2 - 1, v = d y^2 + 1 (the decompression ratio).
NW_HD void ge_decomp_uv(fe& u, fe& v, const fe& y, const curve_consts& k) {
  fe yy, one;
  fe_1(one);
  fe_sq(yy, y);
  fe_sub(u, yy, one);
  fe_mul(v, yy, k.d);
  v.v[0] += 1;
}

// curve25519-dalek CompressedEdwardsY::decompress. w = 8 LE words of the encoding.
// Returns success; p gets (X, Y, 1, XY) with Y as loaded (possibly >= p).
// Only y (and the power's own chain) is live across the (p-5)/8 power: u, v and u v^3 are
// recomputed after it (2 squarings + 3 multiplications) instead of being held in registers.
NW_HD bool ge_frombytes(ge& p, const uint32_t w[8], const curve_consts& k) {
  fe u, v, t;
  fe_frombytes(p.Y, w);
  {
    fe v3, v7, uv7;
    ge_decomp_uv(u, v, p.Y, k);
    fe_sq(t, v);  fe_mul(v3, t, v);
    fe_sq(t, v3); fe_mul(v7, t, v);
    fe_mul(uv7, u, v7);
    fe_pow22523(t, uv7);
  }
  fe_barrier(t);
  fe_barrier(p.Y);
  ge_decomp_uv(u, v, p.Y, k);
  bool ok = fe_sqrt_ratio_finish(p.X, u, v, t, k);
  fe_neg(t, p.X);
  fe_cmov(p.X, t, (w[7] >> 31) != 0);
  fe_1(p.Z);
  fe_mul(p.T, p.X, p.Y);
  return ok;
}

// Affine encoding: y with the parity of x in bit 255.
NW_HD void ge_tobytes(uint32_t w[8], const ge& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_tobytes(w, y);
  w[7] ^= fe_isnegative(x) << 31;
}

// Affine niels form of p (needs 1/Z).
NW_HD void ge_to_niels(ge_niels& n, const ge& p, const fe& d2) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_add(n.ypx, y, x); fe_carry(n.ypx);
  fe_sub(n.ymx, y, x);
  fe_mul(n.xy2d, x, y);
  fe_mul(n.xy2d, n.xy2d, d2);
}

}  // namespace nw
