// nw_consts.hpp — curve constants and the fixed-base table, derived from their
// definitions (d = -121665/121666, sqrt(-1) = 2^((p-1)/4), B = (x >= 0, 4/5)) with the same
// arithmetic the kernels use. Computed once on the host and uploaded to constant memory.
#pragma once
#include "nw_point.hpp"

namespace nw {

NW_HD void fe_from_u32(fe& h, uint32_t x) {
  fe_0(h);
  h.v[0] = x & M26;
  h.v[1] = x >> 26;
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

}  // namespace nw
