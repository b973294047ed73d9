// nw_lp.hpp — limb-parallel GF(2^255 - 19) and edwards25519 point arithmetic for ONE
// latency-bound chain per wave: the 248-doubling Horner over the Pippenger windows in
// k_pip_final (crypto::Signature::verify_batch, crypto/src/lib.rs:206-219; config 1).
//
// A lone wave is issue-bound: every VALU instruction costs its full issue whatever its
// active lanes, so the chain's time is its instruction count. Here one wave holds one point:
// row r (lanes 16r .. 16r+15) holds coordinate r of (X, Y, Z, T) and lane k < 10 of a row
// holds limb k (radix 2^25.5, the same limbs as nw_field.hpp; lanes 10..15 hold 0). Limb-
// wise additions are then ONE instruction, and a product is 10 multiply-accumulates per
// lane: lane k accumulates column k = sum_j f_j g_{(k - j) mod 10} (x19 when wrapped, x2
// for odd j with even k), with f_j broadcast by DPP row_newbcast. The four independent
// products of each formula stage run in the four rows.
//
// Cross-lane moves stay in the VALU: g_{k-j} (or the wrapped 19 g_{k+10-j}) is one DPP
// row_ror:j of g with the wrap parked in the dead lanes (lp_mul), the x2 of odd x odd limbs
// is folded into g's odd source lanes for odd j; a coordinate is broadcast to all four rows
// by gfx950's v_permlane16_swap + v_permlane32_swap (three instructions for all four rows).
// (The round-2 ds_bpermute form, an LDS-path round trip per move, took 0.52 us per doubling;
// the round-4 shift pair per term, row_shr:j + row_shl:(10-j) + an add, 0.43 us.)
//
// Operand discipline is nw_point.hpp's (same products, same first/second operand roles:
// the second operand is the one scaled by 19, the first by 2); lp_carry64 leaves limbs in
// the T_LP bound, for which tests/test_field_bounds.py checks every operand pair.
#pragma once
#include "nw_point.hpp"

namespace nw {

struct lp_ctx {
  uint32_t k;          // limb index (lane & 15)
  uint32_t row;        // coordinate (lane >> 4)
  uint32_t mask;       // M26 / M25 for limbs 0..9, 0 above
  uint32_t sh;         // 26 / 25
  uint32_t c0;         // incoming-carry factor: 19 in limb 0 (wrapped from limb 9), 1 in
                       // limbs 1..9, 0 above (lanes 10..15 stay 0)
  uint32_t p4;         // limb k of 4p (0 above limb 9)
  uint32_t odd;        // 1 in odd limbs (the source side of the x2 of odd x odd limbs)
  uint32_t m1, m2;     // ~0 in rows with bit 0 / bit 1 of the row index set (lp_sel masks)
};

__device__ __forceinline__ lp_ctx lp_init(uint32_t lane) {
  lp_ctx c;
  c.k = lane & 15;
  c.row = (lane >> 4) & 3;
  const bool live = c.k < 10;
  c.mask = !live ? 0u : (c.k & 1) ? M25 : M26;
  c.sh = (c.k & 1) ? 25u : 26u;
  c.c0 = c.k == 0 ? 19u : live ? 1u : 0u;
  c.p4 = !live ? 0u : c.k == 0 ? 0xfffffb4u : (c.k & 1) ? 0x7fffffcu : 0xffffffcu;
  c.odd = c.k & 1;
  c.m1 = (c.row & 1) ? ~0u : 0u;
  c.m2 = (c.row & 2) ? ~0u : 0u;
  return c;
}

// DPP move; lanes whose source is outside the row read 0 (bound_ctrl).
template <int CTRL>
__device__ __forceinline__ uint32_t lp_dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, true);
}

// Carry of value x (64-bit) of limb k into limb k+1 (limb 9's times 19 into limb 0):
// the incoming carry of this lane.
__device__ __forceinline__ uint64_t lp_carry_in64(const lp_ctx& c, uint64_t carry) {
  const uint32_t lo = (uint32_t)carry, hi = (uint32_t)(carry >> 32);
  // row_shr:1 (lane k <- lane k-1) for k >= 1; row_ror:7 (lane 0 <- lane 9) for k = 0
  const uint32_t lo1 = lp_dpp<0x111>(lo), hi1 = lp_dpp<0x111>(hi);
  const uint32_t lo9 = lp_dpp<0x127>(lo), hi9 = lp_dpp<0x127>(hi);
  const uint32_t l = c.k == 0 ? lo9 : lo1, h = c.k == 0 ? hi9 : hi1;
  return (uint64_t)l * c.c0 + ((uint64_t)(h * c.c0) << 32);
}
__device__ __forceinline__ uint32_t lp_carry_in32(const lp_ctx& c, uint32_t carry) {
  const uint32_t x1 = lp_dpp<0x111>(carry), x9 = lp_dpp<0x127>(carry);
  return (c.k == 0 ? x9 : x1) * c.c0;
}

// 64-bit columns (< 2^64) -> limbs in two parallel carry passes: after the first, limb k
// holds < 2^26 + 19 * 2^39 (limb 0) / < 2^26 + 2^39; after the second, limb 0 < 2^26 +
// 2^18.3, limb 1 < 2^25 + 2^17.3, the others < 2^26 / 2^25 + 2^14 -- the "T_LP" bound,
// checked with every operand pair of the point formulas in tests/test_field_bounds.py.
// (Lanes 10..15 hold 0 and receive no carry, so they stay 0.)
__device__ __forceinline__ uint32_t lp_carry64(const lp_ctx& c, uint64_t col) {
  const uint64_t t = (col & c.mask) + lp_carry_in64(c, col >> c.sh);
  return (uint32_t)(t & c.mask) + lp_carry_in32(c, (uint32_t)(t >> c.sh));
}
// 32-bit limbs below 2^29 (a difference a + 4p - b) -> one pass: carries < 2^4 (x19 into
// limb 0), inside T_LP.
__device__ __forceinline__ uint32_t lp_carry32(const lp_ctx& c, uint32_t x) {
  return (x & c.mask) + lp_carry_in32(c, x >> c.sh);
}

// Term j of column k from ONE rotate: the row's dead lanes 10..15 carry the wrapped operand
// (lane L holds 19 g_{L-6}), so row_ror:j hands lane k < j exactly 19 g_{k+10-j} and lane
// k >= j g_{k-j}. For j >= 7 the wrap also reaches lanes 7..9, so those terms rotate a second
// vector whose lanes 7..15 hold 19 g_{L-6} (lanes 0..2 keep g; 3..6 are never read by them).
// Three instructions per term instead of five (broadcast, rotate, multiply-accumulate); the
// dead lanes accumulate garbage that lp_carry64 drops (mask 0, incoming-carry factor 0, and
// no live lane reads a dead lane's carry: lane 0 takes lane 9's).
// (The compiler merges the two accumulator chains below into one; keeping them apart with
// an empty asm measured slower: config 1 0.3240 vs 0.3184 ms, profiles/r05j.)
template <int J>
__device__ __forceinline__ uint64_t lp_mac_ror(uint64_t acc, uint32_t f, uint32_t gsrc) {
  const uint32_t gj = J == 0 ? gsrc : lp_dpp<0x120 + J>(gsrc);   // row_ror:J
  return acc + (uint64_t)lp_dpp<0x150 + J>(f) * gj;
}

__device__ __forceinline__ uint32_t lp_mul(const lp_ctx& c, uint32_t f, uint32_t g) {
  const uint32_t go = g << c.odd;                                // odd source limbs x 2
  const uint32_t we = lp_dpp<0x126>(g * 19u), wo = lp_dpp<0x126>(go * 19u);   // row_ror:6
  const bool lo10 = c.k < 10, lo7 = c.k < 7;
  const uint32_t ge = lo10 ? g : we, gov = lo10 ? go : wo;       // terms 0..6
  const uint32_t he = lo7 ? g : we, ho = lo7 ? go : wo;          // terms 7..9
  uint64_t a = 0, b = 0;   // two chains
  a = lp_mac_ror<0>(a, f, g);    b = lp_mac_ror<1>(b, f, gov);
  a = lp_mac_ror<2>(a, f, ge);   b = lp_mac_ror<3>(b, f, gov);
  a = lp_mac_ror<4>(a, f, ge);   b = lp_mac_ror<5>(b, f, gov);
  a = lp_mac_ror<6>(a, f, ge);   b = lp_mac_ror<7>(b, f, ho);
  a = lp_mac_ror<8>(a, f, he);   b = lp_mac_ror<9>(b, f, ho);
  return lp_carry64(c, a + b);
}
// Limb k of rows 0..3, each in every row.
struct lp_rows {
  uint32_t r0, r1, r2, r3;
};
__device__ __forceinline__ lp_rows lp_rows_of(const lp_ctx& c, uint32_t x) {
  // permlane16_swap(x, x): odd rows of the first copy <-> even rows of the second, giving
  // rows (0, 0, 2, 2) and (1, 1, 3, 3); permlane32_swap of each with itself: upper half of
  // the first copy <-> lower half of the second, giving (0, 0, 0, 0) / (2, 2, 2, 2) etc.
  (void)c;
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const auto e = __builtin_amdgcn_permlane32_swap(p[0], p[0], false, false);
  const auto o = __builtin_amdgcn_permlane32_swap(p[1], p[1], false, false);
  return {e[0], o[0], e[1], o[1]};
}
// Row-wise select as three bitfield inserts (v_bfi_b32): a ternary chain on the row index
// is compiled into divergent branches with every operand sunk into its own arm.
__device__ __forceinline__ uint32_t lp_bfi(uint32_t m, uint32_t a, uint32_t b) {
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ uint32_t lp_sel(const lp_ctx& c, uint32_t a0, uint32_t a1,
                                           uint32_t a2, uint32_t a3) {
  return lp_bfi(c.m2, lp_bfi(c.m1, a3, a2), lp_bfi(c.m1, a1, a0));
}
// a + 4p - b uncarried (fe_sub_nc) and carried (fe_sub).
__device__ __forceinline__ uint32_t lp_sub_nc(const lp_ctx& c, uint32_t a, uint32_t b) {
  return a + c.p4 - b;
}
__device__ __forceinline__ uint32_t lp_sub(const lp_ctx& c, uint32_t a, uint32_t b) {
  return lp_carry32(c, a + c.p4 - b);
}

// Stage 2 shared by doubling and addition: X3 = E F, Y3 = G H, Z3 = F G, T3 = E H.
__device__ __forceinline__ uint32_t lp_stage2(const lp_ctx& c, uint32_t E, uint32_t F,
                                              uint32_t G, uint32_t H) {
  return lp_mul(c, lp_sel(c, E, G, F, E), lp_sel(c, F, H, G, H));
}

// 2P (ge_dbl with T): A = X^2, B = Y^2, C = Z^2, t = (X + Y)^2 in rows 0..3, then stage 2.
__device__ __forceinline__ uint32_t lp_dbl(const lp_ctx& c, uint32_t v) {
  const lp_rows P = lp_rows_of(c, v);
  const uint32_t in = lp_sel(c, v, v, v, P.r0 + P.r1);
  const uint32_t s = lp_mul(c, in, in);
  const lp_rows S = lp_rows_of(c, s);
  const uint32_t A = S.r0, B = S.r1, C = S.r2, t = S.r3;
  const uint32_t H = A + B;
  const uint32_t E = lp_sub_nc(c, H, t);
  const uint32_t G = lp_sub(c, A, B);
  const uint32_t F = G + C + C;
  return lp_stage2(c, E, F, G, H);
}

// P + Q, row q of tab holding component q of Q in the order (YmX, YpX, T2d, Z2)
// (ge_add_cached with T; an affine niels Q has Z2 = 2).
__device__ __forceinline__ uint32_t lp_add(const lp_ctx& c, uint32_t v, uint32_t tab) {
  const lp_rows P = lp_rows_of(c, v);
  const uint32_t X = P.r0, Y = P.r1;
  const uint32_t sw = lp_sel(c, X, Y, P.r3, P.r2);   // rows 2 and 3 swapped: T, Z
  const uint32_t ymx = lp_sub_nc(c, Y, X), ypx = Y + X;
  // a = (Y - X) YmX, b = (Y + X) YpX, c = T2d T, d = Z Z2 (operand order as ge_add_cached)
  const uint32_t m = lp_mul(c, lp_sel(c, ymx, ypx, tab, sw), lp_sel(c, tab, tab, sw, tab));
  const lp_rows M = lp_rows_of(c, m);
  const uint32_t A = M.r0, B = M.r1, C = M.r2, D = M.r3;
  return lp_stage2(c, lp_sub_nc(c, B, A), lp_sub(c, D, C), D + C, B + A);
}

// Cached form (YpX, YmX, Z2, T2d; carried) of the point, row r producing the component
// that lp_cached_component reads back for row r: YmX, YpX, T2d, Z2. d2l: limb k of 2d.
__device__ __forceinline__ uint32_t lp_to_cached(const lp_ctx& c, uint32_t v, uint32_t d2l) {
  const lp_rows P = lp_rows_of(c, v);
  const uint32_t X = P.r0, Y = P.r1, Z = P.r2, T = P.r3;
  const uint32_t prod = lp_mul(c, T, d2l);                       // T 2d (row 2 keeps it)
  const uint32_t sum = lp_carry32(c, lp_sel(c, Y + c.p4 - X, Y + X, Z + Z, Z + Z));
  return lp_sel(c, sum, sum, prod, sum);
}

__device__ __forceinline__ uint32_t lp_identity(const lp_ctx& c) {
  return (c.k == 0 && (c.row == 1 || c.row == 2)) ? 1u : 0u;
}

// Component (row) of a cached point in memory, in lp_add's order.
__device__ __forceinline__ uint32_t lp_cached_component(const lp_ctx& c, const ge_cached& p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&p);   // YpX, YmX, Z2, T2d
  const uint32_t x = w[10 * (c.row ^ 1u) + (c.k < 10 ? c.k : 9u)];   // rows 0..3: 1, 0, 3, 2
  return c.k < 10 ? x : 0u;
}

// Component of sign * n for an affine niels point n (Z2 = 2), in lp_add's order.
__device__ __forceinline__ uint32_t lp_niels_component(const lp_ctx& c, const ge_niels& n,
                                                       bool neg) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&n);   // ypx, ymx, xy2d
  const uint32_t kk = c.k < 10 ? c.k : 0u;
  // rows 0/1: ymx/ypx of sign * n (swapped when negative); row 2: +-xy2d; row 3: 2
  const uint32_t field = c.row == 2 ? 2u : (((c.row == 1) != neg) ? 0u : 1u);
  const uint32_t x = w[10 * field + kk];
  const uint32_t t = (c.row == 2 && neg) ? c.p4 - x : x;   // fe_neg_nc
  const uint32_t r = c.row == 3 ? (c.k == 0 ? 2u : 0u) : t;
  return c.k < 10 ? r : 0u;
}

// Every lane: is the point the identity (X == 0 and Y == Z, curve25519-dalek is_identity)?
// s_tmp: 40 words of LDS.
__device__ __forceinline__ bool lp_is_identity(const lp_ctx& c, uint32_t v, uint32_t* s_tmp) {
  if (c.k < 10) s_tmp[10 * c.row + c.k] = v;
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  fe X, Y, Z;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    X.v[i] = s_tmp[i];
    Y.v[i] = s_tmp[10 + i];
    Z.v[i] = s_tmp[20 + i];
  }
  return fe_iszero(X) && fe_eq(Y, Z);
}

}  // namespace nw
