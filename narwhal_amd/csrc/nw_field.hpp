// nw_field.hpp — GF(2^255 - 19) for gfx950 VALU.
//
// Representation: 10 unsigned 32-bit limbs, alternating 26/25 bits (radix 2^25.5), limb i
// at bit position ceil(25.5 i). Chosen from measurement (profiles/r01_ubench_valu_*.txt):
// on gfx950 v_mad_u64_u32 issues at the same half rate as v_add_co/v_addc/v_alignbit, so a
// radix-2^32 schoolbook product (64 MACs + ~60 carry ops) costs about as much as this
// radix's 100 MACs, and here every column accumulates in a 64-bit register with no carry
// instructions at all (column sums stay < 2^63 for the input bounds below).
//
// Bounds (per limb, even/odd):  T ("tight", every mul/sq/sub output) <= 2^26 / 2^25 (+2^18)
//                               L ("loose", sum of two T)            <= 2^27 / 2^26
// fe_mul / fe_sq accept inputs up to 1.5 * L: every column stays below 2^63.
// fe_sub(a, b) = a + 4p - b, carried to T; valid for b up to 2^28 per limb.
//
// Compiles for host and device (NW_HD) so tools/host_selftest can check the exact same
// code on the CPU; the product library only runs it on the GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NW_HD __host__ __device__ __forceinline__

namespace nw {

struct fe { uint32_t v[10]; };

static constexpr uint32_t M26 = (1u << 26) - 1;
static constexpr uint32_t M25 = (1u << 25) - 1;

NW_HD uint64_t mul32(uint32_t a, uint32_t b) { return (uint64_t)a * b; }

// acc + a * b as one v_mad_u64_u32. The empty asm makes the accumulator opaque so the
// compiler keeps the chain in the written order (a column's carry-in stays its first
// addend) instead of re-associating it into a product tree plus a separate 64-bit add.
NW_HD uint64_t mac(uint64_t acc, uint32_t a, uint32_t b) {
  uint64_t r = acc + (uint64_t)a * b;
#ifdef __HIP_DEVICE_COMPILE__
  asm("" : "+v"(r));
#endif
  return r;
}

NW_HD void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
NW_HD void fe_1(fe& h) { fe_0(h); h.v[0] = 1; }
NW_HD void fe_copy(fe& h, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i];
}

// Carry a 10 x 64-bit column vector down to T limbs (ref10 interleaved order).
NW_HD void fe_carry64(fe& out, uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3, uint64_t h4,
                      uint64_t h5, uint64_t h6, uint64_t h7, uint64_t h8, uint64_t h9) {
  uint64_t c;
  c = h0 >> 26; h1 += c; h0 &= M26;
  c = h4 >> 26; h5 += c; h4 &= M26;
  c = h1 >> 25; h2 += c; h1 &= M25;
  c = h5 >> 25; h6 += c; h5 &= M25;
  c = h2 >> 26; h3 += c; h2 &= M26;
  c = h6 >> 26; h7 += c; h6 &= M26;
  c = h3 >> 25; h4 += c; h3 &= M25;
  c = h7 >> 25; h8 += c; h7 &= M25;
  c = h4 >> 26; h5 += c; h4 &= M26;
  c = h8 >> 26; h9 += c; h8 &= M26;
  c = h9 >> 25; h0 += c * 19; h9 &= M25;
  c = h0 >> 26; h1 += c; h0 &= M26;
  out.v[0] = (uint32_t)h0; out.v[1] = (uint32_t)h1; out.v[2] = (uint32_t)h2;
  out.v[3] = (uint32_t)h3; out.v[4] = (uint32_t)h4; out.v[5] = (uint32_t)h5;
  out.v[6] = (uint32_t)h6; out.v[7] = (uint32_t)h7; out.v[8] = (uint32_t)h8;
  out.v[9] = (uint32_t)h9;
}

// 32-bit carry pass for limbs already < 2^32 (after add/sub).
NW_HD void fe_carry(fe& h) {
  uint32_t c;
  c = h.v[0] >> 26; h.v[1] += c; h.v[0] &= M26;
  c = h.v[1] >> 25; h.v[2] += c; h.v[1] &= M25;
  c = h.v[2] >> 26; h.v[3] += c; h.v[2] &= M26;
  c = h.v[3] >> 25; h.v[4] += c; h.v[3] &= M25;
  c = h.v[4] >> 26; h.v[5] += c; h.v[4] &= M26;
  c = h.v[5] >> 25; h.v[6] += c; h.v[5] &= M25;
  c = h.v[6] >> 26; h.v[7] += c; h.v[6] &= M26;
  c = h.v[7] >> 25; h.v[8] += c; h.v[7] &= M25;
  c = h.v[8] >> 26; h.v[9] += c; h.v[8] &= M26;
  c = h.v[9] >> 25; h.v[0] += c * 19; h.v[9] &= M25;
  c = h.v[0] >> 26; h.v[1] += c; h.v[0] &= M26;
}

// h = f + g (no carry: T + T -> L).
NW_HD void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}

// h = f - g + 4p, carried to T.
NW_HD void fe_sub(fe& h, const fe& f, const fe& g) {
  h.v[0] = (f.v[0] + 0xfffffb4u) - g.v[0];   // 4 * (2^26 - 19)
#pragma unroll
  for (int i = 1; i < 10; ++i)
    h.v[i] = (f.v[i] + ((i & 1) ? 0x7fffffcu : 0xffffffcu)) - g.v[i];
  fe_carry(h);
}
NW_HD void fe_neg(fe& h, const fe& f) { fe z; fe_0(z); fe_sub(h, z, f); }

// h = f - g + 4p WITHOUT the carry pass ("S" bound: limbs <= f + 4p, about 2^28.3 for
// f <= T, 2^28.6 for f <= L). Only for values whose every use is the FIRST operand of
// fe_mul (scaled by 2 in 32 bits; the second operand is scaled by 19 and must be <= 1.5L).
// Worst-case columns over the limb bounds (tests/test_field_bounds.py) stay below 2^64
// with their carry-in.
NW_HD void fe_sub_nc(fe& h, const fe& f, const fe& g) {
  h.v[0] = (f.v[0] + 0xfffffb4u) - g.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i)
    h.v[i] = (f.v[i] + ((i & 1) ? 0x7fffffcu : 0xffffffcu)) - g.v[i];
}
NW_HD void fe_neg_nc(fe& h, const fe& f) { fe z; fe_0(z); fe_sub_nc(h, z, f); }

// Carry-folded column reduction (fe_mul / fe_sq). Columns 0-4 and 5-9 are accumulated as
// two interleaved chains (independent v_mad_u64_u32 streams, so no dependent-issue wait
// states); inside a chain each column's carry is the initial accumulator of the next one,
// so no separate 64-bit add per step. fe_join finishes: a = column 4 (its carry goes into
// limb 5), b = column 9 (its carry wraps to limb 0 times 19). Every column stays < 2^63
// (input bounds above), so carries are < 2^39 and limbs land in T.
NW_HD void fe_join(fe& h, uint64_t a, uint64_t b) {
  h.v[4] = (uint32_t)a & M26;
  h.v[9] = (uint32_t)b & M25;
  const uint64_t t5 = (uint64_t)h.v[5] + (a >> 26);
  h.v[5] = (uint32_t)t5 & M25;
  h.v[6] += (uint32_t)(t5 >> 25);
  const uint64_t t0 = (uint64_t)h.v[0] + (b >> 25) * 19;
  h.v[0] = (uint32_t)t0 & M26;
  h.v[1] += (uint32_t)(t0 >> 26);
}

// (Five interleaved chains of two columns each measured 4 % slower in the strict kernel: fewer
// s_nop wait states, but at 3 waves per SIMD the other waves issue during them, and the
// extra joins and accumulators cost instructions and spills)
NW_HD void fe_mul(fe& h, const fe& f, const fe& g) {
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4];
  const uint32_t g5 = g.v[5], g6 = g.v[6], g7 = g.v[7], g8 = g.v[8], g9 = g.v[9];
  const uint32_t g1_19 = 19 * g1, g2_19 = 19 * g2, g3_19 = 19 * g3, g4_19 = 19 * g4,
                 g5_19 = 19 * g5, g6_19 = 19 * g6, g7_19 = 19 * g7, g8_19 = 19 * g8,
                 g9_19 = 19 * g9;
  const uint32_t f1_2 = 2 * f1, f3_2 = 2 * f3, f5_2 = 2 * f5, f7_2 = 2 * f7, f9_2 = 2 * f9;
  // Two interleaved carry-folded chains: columns 0-4 (a) and 5-9 (b).
  uint64_t a = 0, b = 0;
  a = mac(a, f0, g0); b = mac(b, f0, g5);
  a = mac(a, f1_2, g9_19); b = mac(b, f1, g4);
  a = mac(a, f2, g8_19); b = mac(b, f2, g3);
  a = mac(a, f3_2, g7_19); b = mac(b, f3, g2);
  a = mac(a, f4, g6_19); b = mac(b, f4, g1);
  a = mac(a, f5_2, g5_19); b = mac(b, f5, g0);
  a = mac(a, f6, g4_19); b = mac(b, f6, g9_19);
  a = mac(a, f7_2, g3_19); b = mac(b, f7, g8_19);
  a = mac(a, f8, g2_19); b = mac(b, f8, g7_19);
  a = mac(a, f9_2, g1_19); b = mac(b, f9, g6_19);
  h.v[0] = (uint32_t)a & M26; a >>= 26; h.v[5] = (uint32_t)b & M25; b >>= 25;
  a = mac(a, f0, g1); b = mac(b, f0, g6);
  a = mac(a, f1, g0); b = mac(b, f1_2, g5);
  a = mac(a, f2, g9_19); b = mac(b, f2, g4);
  a = mac(a, f3, g8_19); b = mac(b, f3_2, g3);
  a = mac(a, f4, g7_19); b = mac(b, f4, g2);
  a = mac(a, f5, g6_19); b = mac(b, f5_2, g1);
  a = mac(a, f6, g5_19); b = mac(b, f6, g0);
  a = mac(a, f7, g4_19); b = mac(b, f7_2, g9_19);
  a = mac(a, f8, g3_19); b = mac(b, f8, g8_19);
  a = mac(a, f9, g2_19); b = mac(b, f9_2, g7_19);
  h.v[1] = (uint32_t)a & M25; a >>= 25; h.v[6] = (uint32_t)b & M26; b >>= 26;
  a = mac(a, f0, g2); b = mac(b, f0, g7);
  a = mac(a, f1_2, g1); b = mac(b, f1, g6);
  a = mac(a, f2, g0); b = mac(b, f2, g5);
  a = mac(a, f3_2, g9_19); b = mac(b, f3, g4);
  a = mac(a, f4, g8_19); b = mac(b, f4, g3);
  a = mac(a, f5_2, g7_19); b = mac(b, f5, g2);
  a = mac(a, f6, g6_19); b = mac(b, f6, g1);
  a = mac(a, f7_2, g5_19); b = mac(b, f7, g0);
  a = mac(a, f8, g4_19); b = mac(b, f8, g9_19);
  a = mac(a, f9_2, g3_19); b = mac(b, f9, g8_19);
  h.v[2] = (uint32_t)a & M26; a >>= 26; h.v[7] = (uint32_t)b & M25; b >>= 25;
  a = mac(a, f0, g3); b = mac(b, f0, g8);
  a = mac(a, f1, g2); b = mac(b, f1_2, g7);
  a = mac(a, f2, g1); b = mac(b, f2, g6);
  a = mac(a, f3, g0); b = mac(b, f3_2, g5);
  a = mac(a, f4, g9_19); b = mac(b, f4, g4);
  a = mac(a, f5, g8_19); b = mac(b, f5_2, g3);
  a = mac(a, f6, g7_19); b = mac(b, f6, g2);
  a = mac(a, f7, g6_19); b = mac(b, f7_2, g1);
  a = mac(a, f8, g5_19); b = mac(b, f8, g0);
  a = mac(a, f9, g4_19); b = mac(b, f9_2, g9_19);
  h.v[3] = (uint32_t)a & M25; a >>= 25; h.v[8] = (uint32_t)b & M26; b >>= 26;
  a = mac(a, f0, g4); b = mac(b, f0, g9);
  a = mac(a, f1_2, g3); b = mac(b, f1, g8);
  a = mac(a, f2, g2); b = mac(b, f2, g7);
  a = mac(a, f3_2, g1); b = mac(b, f3, g6);
  a = mac(a, f4, g0); b = mac(b, f4, g5);
  a = mac(a, f5_2, g9_19); b = mac(b, f5, g4);
  a = mac(a, f6, g8_19); b = mac(b, f6, g3);
  a = mac(a, f7_2, g7_19); b = mac(b, f7, g2);
  a = mac(a, f8, g6_19); b = mac(b, f8, g1);
  a = mac(a, f9_2, g5_19); b = mac(b, f9, g0);
  fe_join(h, a, b);
}

NW_HD void fe_sq(fe& h, const fe& f) {
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t f0_2 = 2 * f0, f1_2 = 2 * f1, f2_2 = 2 * f2, f3_2 = 2 * f3, f4_2 = 2 * f4,
                 f5_2 = 2 * f5, f6_2 = 2 * f6, f7_2 = 2 * f7;
  const uint32_t f5_38 = 38 * f5, f6_19 = 19 * f6, f7_38 = 38 * f7, f8_19 = 19 * f8,
                 f9_38 = 38 * f9;
  // Two interleaved carry-folded chains: columns 0-4 (a) and 5-9 (b).
  uint64_t a = 0, b = 0;
  a = mac(a, f0, f0); b = mac(b, f0_2, f5);
  a = mac(a, f1_2, f9_38); b = mac(b, f1_2, f4);
  a = mac(a, f2_2, f8_19); b = mac(b, f2_2, f3);
  a = mac(a, f3_2, f7_38); b = mac(b, f6, f9_38);
  a = mac(a, f4_2, f6_19); b = mac(b, f7_2, f8_19);
  a = mac(a, f5, f5_38); h.v[5] = (uint32_t)b & M25; b >>= 25;
  h.v[0] = (uint32_t)a & M26; a >>= 26; b = mac(b, f0_2, f6);
  a = mac(a, f0_2, f1); b = mac(b, f1_2, f5_2);
  a = mac(a, f2, f9_38); b = mac(b, f2_2, f4);
  a = mac(a, f3_2, f8_19); b = mac(b, f3_2, f3);
  a = mac(a, f4, f7_38); b = mac(b, f7_2, f9_38);
  a = mac(a, f5_2, f6_19); b = mac(b, f8, f8_19);
  h.v[1] = (uint32_t)a & M25; a >>= 25; h.v[6] = (uint32_t)b & M26; b >>= 26;
  a = mac(a, f0_2, f2); b = mac(b, f0_2, f7);
  a = mac(a, f1_2, f1); b = mac(b, f1_2, f6);
  a = mac(a, f3_2, f9_38); b = mac(b, f2_2, f5);
  a = mac(a, f4_2, f8_19); b = mac(b, f3_2, f4);
  a = mac(a, f5_2, f7_38); b = mac(b, f8, f9_38);
  a = mac(a, f6, f6_19); h.v[7] = (uint32_t)b & M25; b >>= 25;
  h.v[2] = (uint32_t)a & M26; a >>= 26; b = mac(b, f0_2, f8);
  a = mac(a, f0_2, f3); b = mac(b, f1_2, f7_2);
  a = mac(a, f1_2, f2); b = mac(b, f2_2, f6);
  a = mac(a, f4, f9_38); b = mac(b, f3_2, f5_2);
  a = mac(a, f5_2, f8_19); b = mac(b, f4, f4);
  a = mac(a, f6, f7_38); b = mac(b, f9, f9_38);
  h.v[3] = (uint32_t)a & M25; a >>= 25; h.v[8] = (uint32_t)b & M26; b >>= 26;
  a = mac(a, f0_2, f4); b = mac(b, f0_2, f9);
  a = mac(a, f1_2, f3_2); b = mac(b, f1_2, f8);
  a = mac(a, f2, f2); b = mac(b, f2_2, f7);
  a = mac(a, f5_2, f9_38); b = mac(b, f3_2, f6);
  a = mac(a, f6_2, f8_19); b = mac(b, f4_2, f5);
  a = mac(a, f7, f7_38);
  fe_join(h, a, b);
}

// h = f^(2^n), rolled loop (keeps code size down inside the exponentiations).
NW_HD void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq(h, f);
#pragma unroll 1
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

// Load 32 bytes as curve25519-dalek FieldElement::from_bytes does: the low 255 bits,
// NOT reduced mod p (y >= p stays as is; arithmetic is mod p anyway).
NW_HD void fe_frombytes(fe& h, const uint32_t w[8]) {
  // w = 8 little-endian 32-bit words of the encoding.
  h.v[0] = w[0] & M26;                                        // bits   0..25
  h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & M25;                // bits  26..50
  h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & M26;               // bits  51..76
  h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & M25;               // bits  77..101
  h.v[4] = ((w[3] >> 6)) & M26;                               // bits 102..127
  h.v[5] = w[4] & M25;                                        // bits 128..152
  h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & M26;                // bits 153..178
  h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & M25;               // bits 179..203
  h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & M26;               // bits 204..229
  h.v[9] = (w[7] >> 6) & M25;                                 // bits 230..254
}

// Fully reduce to the canonical representative in [0, p) as 10 tight limbs.
NW_HD void fe_canonical(fe& t, const fe& f) {
  fe_copy(t, f);
  fe_carry(t);
  fe_carry(t);
  // t < 2^255 + small now; q = 1 iff t >= p.
  uint32_t q = (t.v[0] + 19) >> 26;
  q = (t.v[1] + q) >> 25;
  q = (t.v[2] + q) >> 26;
  q = (t.v[3] + q) >> 25;
  q = (t.v[4] + q) >> 26;
  q = (t.v[5] + q) >> 25;
  q = (t.v[6] + q) >> 26;
  q = (t.v[7] + q) >> 25;
  q = (t.v[8] + q) >> 26;
  q = (t.v[9] + q) >> 25;
  t.v[0] += 19 * q;
  uint32_t c;
  c = t.v[0] >> 26; t.v[1] += c; t.v[0] &= M26;
  c = t.v[1] >> 25; t.v[2] += c; t.v[1] &= M25;
  c = t.v[2] >> 26; t.v[3] += c; t.v[2] &= M26;
  c = t.v[3] >> 25; t.v[4] += c; t.v[3] &= M25;
  c = t.v[4] >> 26; t.v[5] += c; t.v[4] &= M26;
  c = t.v[5] >> 25; t.v[6] += c; t.v[5] &= M25;
  c = t.v[6] >> 26; t.v[7] += c; t.v[6] &= M26;
  c = t.v[7] >> 25; t.v[8] += c; t.v[7] &= M25;
  c = t.v[8] >> 26; t.v[9] += c; t.v[8] &= M26;
  t.v[9] &= M25;
}

// Canonical little-endian 32-byte encoding as 8 words.
NW_HD void fe_tobytes(uint32_t w[8], const fe& f) {
  fe t;
  fe_canonical(t, f);
  w[0] = t.v[0] | (t.v[1] << 26);
  w[1] = (t.v[1] >> 6) | (t.v[2] << 19);
  w[2] = (t.v[2] >> 13) | (t.v[3] << 13);
  w[3] = (t.v[3] >> 19) | (t.v[4] << 6);
  w[4] = t.v[5] | (t.v[6] << 25);
  w[5] = (t.v[6] >> 7) | (t.v[7] << 19);
  w[6] = (t.v[7] >> 13) | (t.v[8] << 12);
  w[7] = (t.v[8] >> 20) | (t.v[9] << 6);
}

NW_HD bool fe_iszero(const fe& f) {
  fe t;
  fe_canonical(t, f);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) acc |= t.v[i];
  return acc == 0;
}
NW_HD bool fe_eq(const fe& a, const fe& b) {
  fe d;
  fe_sub(d, a, b);
  return fe_iszero(d);
}
// "negative" = low bit of the canonical encoding (curve25519-dalek is_negative).
NW_HD uint32_t fe_isnegative(const fe& f) {
  fe t;
  fe_canonical(t, f);
  return t.v[0] & 1;
}
NW_HD void fe_cmov(fe& h, const fe& f, bool c) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = c ? f.v[i] : h.v[i];
}

// z^(2^250 - 1) (returned in out) and z^11 (returned in z11).
NW_HD void fe_pow2_250_1(fe& out, fe& z11, const fe& z) {
  fe z2, z9, t, z5, z10, z20, z50, z100;
  fe_sq(z2, z);                  // 2
  fe_sqn(t, z2, 2);              // 8
  fe_mul(z9, t, z);              // 9
  fe_mul(z11, z9, z2);           // 11
  fe_sq(t, z11);                 // 22
  fe_mul(z5, t, z9);             // 2^5 - 1
  fe_sqn(t, z5, 5);    fe_mul(z10, t, z5);     // 2^10 - 1
  fe_sqn(t, z10, 10);  fe_mul(z20, t, z10);    // 2^20 - 1
  fe_sqn(t, z20, 20);  fe_mul(t, t, z20);      // 2^40 - 1
  fe_sqn(t, t, 10);    fe_mul(z50, t, z10);    // 2^50 - 1
  fe_sqn(t, z50, 50);  fe_mul(z100, t, z50);   // 2^100 - 1
  fe_sqn(t, z100, 100); fe_mul(t, t, z100);    // 2^200 - 1
  fe_sqn(t, t, 50);    fe_mul(out, t, z50);    // 2^250 - 1
}
NW_HD void fe_invert(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 5);               // 2^255 - 32
  fe_mul(out, t, z11);           // 2^255 - 21 = p - 2
}
NW_HD void fe_pow22523(fe& out, const fe& z) {
  fe t, z11;
  fe_pow2_250_1(t, z11, z);
  fe_sqn(t, t, 2);               // 2^252 - 4
  fe_mul(out, t, z);             // 2^252 - 3 = (p - 5) / 8
}

}  // namespace nw
