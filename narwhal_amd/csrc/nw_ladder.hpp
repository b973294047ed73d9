// nw_ladder.hpp — scalar-multiplication ladders shared by the verification kernels.
//
// Signed fixed windows, recoded without a sequential pass (sc_recode): 4-bit digits over a
// 9-entry per-point table j*P (cached form), 8-bit digits over the 129-entry B table
// (affine niels, LDS). A joint ladder shares the 252 doublings between the two scalars,
// as dalek's Straus/vartime_double_scalar_mul_basepoint does [ext].
#pragma once
#include "nw_point.hpp"
#include "nw_scalar.hpp"

namespace nw {

// Select word j (wave-uniform j) of an 8-word register array without dynamic indexing.
NW_HD uint32_t sel8(const uint32_t a[8], int j) {
  uint32_t r = a[0];
#pragma unroll
  for (int t = 1; t < 8; ++t) r = (j == t) ? a[t] : r;
  return r;
}

// Table of j * P (j = 0..8) in cached form, for signed 4-bit digits.
NW_HD void build_table9(ge_cached tab[9], const ge& P, const fe& d2) {
  ge_cached_identity(tab[0]);
  ge_to_cached(tab[1], P, d2);
  ge acc;
  ge_dbl(acc, P, true);
  ge_to_cached(tab[2], acc, d2);
#pragma unroll 1
  for (int j = 3; j <= 8; ++j) {
    ge_add_cached(acc, acc, tab[1], true);
    ge_to_cached(tab[j], acc, d2);
  }
}

NW_HD void add_digit_cached(ge& acc, const ge_cached* tab, int d,
                                                 bool want_t) {
  int ad = d < 0 ? -d : d;
  ge_cached c = tab[ad];
  ge_cached_cneg(c, d < 0);
  ge_add_cached(acc, acc, c, want_t);
}

NW_HD void add_digit_niels(ge& acc, const ge_niels* s_btab, int e,
                                                bool want_t) {
  int ae = e < 0 ? -e : e;
  ge_niels nb = s_btab[ae];
  ge_niels_cneg(nb, e < 0);
  ge_add_niels(acc, acc, nb, want_t);
}

// acc = [b]B + [a]P  with a < 2^253 (4-bit signed digits over tab = j*P) and b < 2^253
// (8-bit signed digits over the LDS B table). Returned without T.
NW_HD void dsm_var_base(ge& acc, const ge_cached* tab, const sc& a,
                                             const sc& b, const ge_niels* s_btab) {
  uint32_t aa[8], bb[8];
  sc_recode(aa, a, 0x88888888u);
  sc_recode(bb, b, 0x80808080u);
  ge_identity(acc);
#pragma unroll 1
  for (int i = 63; i >= 0; --i) {
    if (i != 63) {
#pragma unroll 1
      for (int t = 0; t < 3; ++t) ge_dbl(acc, acc, false);
      ge_dbl(acc, acc, true);
    }
    const bool even = (i & 1) == 0;
    const int da = (int)((sel8(aa, i >> 3) >> ((i & 7) * 4)) & 15u) - 8;
    add_digit_cached(acc, tab, da, even);
    if (even) {
      const int db = (int)((sel8(bb, i >> 3) >> (((i >> 1) & 3) * 8)) & 255u) - 128;
      add_digit_niels(acc, s_btab, db, false);
    }
  }
}

// acc = [b]B for b < 2^253 (8-bit signed windows over the LDS B table), with T.
NW_HD void fixed_base_mul(ge& acc, const sc& b, const ge_niels* s_btab) {
  uint32_t bb[8];
  sc_recode(bb, b, 0x80808080u);
  ge_identity(acc);
#pragma unroll 1
  for (int j = 31; j >= 0; --j) {
    if (j != 31) {
#pragma unroll 1
      for (int t = 0; t < 7; ++t) ge_dbl(acc, acc, false);
      ge_dbl(acc, acc, true);
    }
    const int db = (int)((sel8(bb, j >> 2) >> ((j & 3) * 8)) & 255u) - 128;
    add_digit_niels(acc, s_btab, db, true);
  }
}

}  // namespace nw
