// nw_quad.hpp — one edwards25519 point spread over the 4 lanes of a DPP quad, for the
// latency-bound single chains (the Pippenger Horner over windows in k_pip_final).
//
// A lone wave issues every VALU instruction at full cost whatever its active lanes, so a
// one-lane doubling chain pays ~4 squarings + 3 multiplications of issue per doubling. Here
// lane q of a quad holds coordinate q of the point (X, Y, Z, T) and the four independent
// multiplications of each formula stage run side by side, one per lane: a doubling is one
// squaring + one multiplication deep, an addition two multiplications deep. Operands move
// between the lanes of a quad with DPP quad_perm moves (no LDS traffic).
//
// Every lane multiplies exactly the operand pair the one-lane formulas in nw_point.hpp
// multiply (same order, same carried/uncarried forms), so the limb bounds checked by
// tests/test_field_bounds.py hold unchanged.
#pragma once
#include "nw_point.hpp"

namespace nw {

// quad_perm control: lane i of each quad reads lane s_i.
template <int S0, int S1, int S2, int S3>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
  constexpr int ctrl = S0 | (S1 << 2) | (S2 << 4) | (S3 << 6);
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xf, 0xf, false);
}

template <int S0, int S1, int S2, int S3>
__device__ __forceinline__ void fe_qperm(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 10; ++i) r.v[i] = qperm<S0, S1, S2, S3>(a.v[i]);
}

template <int K>
__device__ __forceinline__ void fe_bcast(fe& r, const fe& a) { fe_qperm<K, K, K, K>(r, a); }

// Lane-q select without branches: m[k] = all-ones in lane k of the quad, else 0 (a
// ternary chain here is compiled into divergent branches).
struct qmask { uint32_t m[4]; };
__device__ __forceinline__ qmask quad_mask(int q) {
  qmask k;
#pragma unroll
  for (int i = 0; i < 4; ++i) k.m[i] = q == i ? 0xffffffffu : 0u;
  return k;
}

__device__ __forceinline__ void fe_sel4(fe& r, const qmask& k, const fe& a0, const fe& a1,
                                        const fe& a2, const fe& a3) {
#pragma unroll
  for (int i = 0; i < 10; ++i)
    r.v[i] = (a0.v[i] & k.m[0]) | (a1.v[i] & k.m[1]) | (a2.v[i] & k.m[2]) | (a3.v[i] & k.m[3]);
}

// Second stage shared by doubling and addition: from (E, F, G, H) in every lane,
// X3 = E F, Y3 = G H, Z3 = F G, T3 = E H (lane q computes coordinate q).
__device__ __forceinline__ void quad_stage2(fe& v, const qmask& q, const fe& E, const fe& F, const fe& G,
                                            const fe& H) {
  fe a, b;
  fe_sel4(a, q, E, G, F, E);
  fe_sel4(b, q, F, H, G, H);
  fe_mul(v, a, b);
}

// v = coordinate q of 2P (ge_dbl, with T).
__device__ __forceinline__ void quad_dbl(fe& v, const qmask& q) {
  fe X, Y, in, s, A, B, C, t, E, F, G, H;
  fe_bcast<0>(X, v);
  fe_bcast<1>(Y, v);
  fe_add(in, X, Y);
#pragma unroll
  for (int i = 0; i < 10; ++i) in.v[i] = (in.v[i] & q.m[3]) | (v.v[i] & ~q.m[3]);
  fe_sq(s, in);            // A = X^2, B = Y^2, C = Z^2, t = (X + Y)^2
  fe_bcast<0>(A, s);
  fe_bcast<1>(B, s);
  fe_bcast<2>(C, s);
  fe_bcast<3>(t, s);
  fe_add(C, C, C);
  fe_add(H, A, B);
  fe_sub_nc(E, H, t);
  fe_sub(G, A, B);
  fe_add(F, G, C);
  quad_stage2(v, q, E, F, G, H);
}

// v = coordinate q of P + Q, where lane q holds component q of Q in the order
// (YmX, YpX, T2d, Z2) of a cached point (ge_add_cached, with T).
__device__ __forceinline__ void quad_add(fe& v, const qmask& q, const fe& tab) {
  fe X, Y, sw, ymx, ypx, a, b, m, A, B, C, D, E, F, G, H;
  fe_bcast<0>(X, v);
  fe_bcast<1>(Y, v);
  fe_qperm<0, 1, 3, 2>(sw, v);   // lane 2 gets T, lane 3 gets Z
  fe_sub_nc(ymx, Y, X);
  fe_add(ypx, Y, X);
  // a = (Y - X) YmX, b = (Y + X) YpX, c = T2d T, d = Z Z2 (operand order as ge_add_cached)
  fe_sel4(a, q, ymx, ypx, tab, sw);
  fe_sel4(b, q, tab, tab, sw, tab);
  fe_mul(m, a, b);
  fe_bcast<0>(A, m);
  fe_bcast<1>(B, m);
  fe_bcast<2>(C, m);
  fe_bcast<3>(D, m);
  fe_sub_nc(E, B, A);
  fe_sub(F, D, C);
  fe_add(G, D, C);
  fe_add(H, B, A);
  quad_stage2(v, q, E, F, G, H);
}

// Component q of a cached point, in quad_add's order.
__device__ __forceinline__ void quad_cached_component(fe& r, const qmask& q, const ge_cached& c) {
  fe_sel4(r, q, c.YmX, c.YpX, c.T2d, c.Z2);
}

// Component q of the affine niels point sign * n (Z2 = 2), in quad_add's order.
__device__ __forceinline__ void quad_niels_component(fe& r, const qmask& q, const ge_niels& n, bool neg) {
  fe two, nxy, a0, a1, a2;
  fe_0(two);
  two.v[0] = 2;
  fe_neg_nc(nxy, n.xy2d);
  const uint32_t ng = neg ? 0xffffffffu : 0u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    a0.v[i] = (n.ypx.v[i] & ng) | (n.ymx.v[i] & ~ng);
    a1.v[i] = (n.ymx.v[i] & ng) | (n.ypx.v[i] & ~ng);
    a2.v[i] = (nxy.v[i] & ng) | (n.xy2d.v[i] & ~ng);
  }
  fe_sel4(r, q, a0, a1, a2, two);
}

__device__ __forceinline__ void quad_identity(fe& v, const qmask& q) {
  fe_0(v);
  v.v[0] = (q.m[1] | q.m[2]) & 1u;
}

// X == 0 and Y == Z (curve25519-dalek is_identity), the same answer in every lane.
__device__ __forceinline__ bool quad_is_identity(const fe& v) {
  fe X, Y, Z;
  fe_bcast<0>(X, v);
  fe_bcast<1>(Y, v);
  fe_bcast<2>(Z, v);
  return fe_iszero(X) && fe_eq(Y, Z);
}

}  // namespace nw
