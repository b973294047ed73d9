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
