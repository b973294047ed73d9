// nw_strict.hpp — crypto::Signature::verify (crypto/src/lib.rs:200-204: ed25519
// Signature::from_bytes, dalek PublicKey::from_bytes, verify_strict [ext]) for one lane.
//
// Shared by k_verify_strict and the host self-check (tools/hostcheck.hip), so the exact
// code the GPU runs is also checked against the oracle on the CPU.
//
//   1. s high bits, s < l, decompress A and R (dalek semantics, y >= p accepted),
//      small-order tests (8P == 0 <=> y mod p in {0, 1, -1, y8, -y8} for a decoded P).
//   2. k = H(R || A || M) mod l (computed by the caller: SHA-512 is device code).
//   3. Half-size scalars (nw_scalar.hpp sc_half_split): u = v k (mod 8l), v odd, and
//      w = -v s mod l; then  R + [k]A - [s]B == 0  <=>  [v]R + [u]A + [w]B == 0.
//   4. One ladder of ~128 doublings: signed 4-bit windows over u (table j*A) and |v|
//      (table j*R, digits negated when v < 0), per-lane tables in private memory;
//      w by signed NW_BWIN-bit windows over two affine tables (j*B and j*2^128 B, bdigits
//      below): 16-bit windows over 2 x 32,769 entries in global memory (8.4 MB; 16 B
//      additions per verify), 20-bit (2 x 524,289, 134 MB; 13 additions), 24-bit
//      (2 x 8,388,609, 2.1 GB; 11 additions), or 8-bit over 2 x 129 entries in LDS (32).
#pragma once
#include "narwhal_amd.h"
#include "nw_kernels.h"

#ifndef NW_BWIN
#define NW_BWIN 24
#endif

#include "nw_ladder.hpp"

namespace nw {

struct strict_consts {
  curve_consts k;
  fe small_y[5];   // canonical y of the 8 small-order points: 0, 1, -1, y8, -y8
};

// 8P == identity for a decoded point (y as loaded; the x sign does not matter).
NW_HD bool small_order_by_y(const fe& y, const fe small_y[5]) {
  fe t;
  fe_canonical(t, y);
  bool hit = false;
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) d |= t.v[i] ^ small_y[c].v[i];
    hit |= d == 0;
  }
  return hit;
}

// The torsion subgroup E[8] of edwards25519 is cyclic of order 8: x[j], y[j] = the affine
// (canonical) coordinates of [j] T8, j = 0..7, for the order-8 point T8 with y = y8 and
// x >= 0 (nw_consts.hpp compute_torsion). torsion_index names a point of E[8] by its j, so
// sums of torsion points become sums of indices mod 8.
struct torsion_consts {
  fe x[8], y[8];
};
// j with P == [j] T8 (projective compare), or -1 when P is not a torsion point.
NW_HD int torsion_index(const ge& P, const torsion_consts& tc) {
  int r = -1;
#pragma unroll 1
  for (int j = 0; j < 8; ++j) {
    fe a, b;
    fe_mul(a, tc.x[j], P.Z);
    fe_mul(b, tc.y[j], P.Z);
    if (fe_eq(a, P.X) && fe_eq(b, P.Y)) r = j;
  }
  return r;
}

// Committee-key flag word (nw_kernels.h key_tables_t::ok): bit 0 = the key decodes, bit 1 =
// small order (8A == identity), bits 2..4 = lambda with [l] A == [lambda] T8 (the image of the
// key's torsion component; 0 iff A lies in the prime-order subgroup). dalek's verify_batch
// weights A by (z k mod l), not z k, so a key with lambda != 0 adds [-(z k div l) lambda] T8
// to the batch sum even for a vote that passes its strict check.
constexpr uint32_t kKeyDecoded = 1u, kKeySmall = 2u, kKeyLambdaShift = 2u, kKeyLambdaMask = 0x1cu;

NW_HD int digit4_of(const uint32_t* w, int nwords, int j) {
  uint32_t word = w[0];
  for (int t = 1; t < 8; ++t) word = (t < nwords && (j >> 3) == t) ? w[t] : word;
  return (int)((word >> ((j & 7) * 4)) & 15u) - 8;
}

NW_HD void add_table_digit(ge& acc, const ge_cached* tab, int d, bool want_t) {
  // tab[e - 1] = e * P, e = 1..8; d = 0 adds nothing.
  if (d != 0) {
    const int ad = d < 0 ? -d : d;
    ge_cached c = tab[ad - 1];
    ge_cached_cneg(c, d < 0);
    ge_add_cached(acc, acc, c, want_t);
  }
}

// (2X : 2Y : 2Z) from a cached entry (Y+X, Y-X, 2Z, 2dT), without T: a doubling's input.
NW_HD void ge_from_cached_not(ge& r, const ge_cached& c) {
  fe_sub(r.X, c.YpX, c.YmX);
  fe_add(r.Y, c.YpX, c.YmX);
  fe_carry(r.Y);
  fe_copy(r.Z, c.Z2);
}

// A per-lane table entry packed into one 128-byte line (the device kernel's tables; the host
// self-check runs both forms): the four coordinates
// of the cached form, each carried to limbs < 2^26 / 2^25 (limb 1 < 2^26) and packed into 8
// words (limb widths 26, 26, 26, 25, 26, 25, 26, 25, 26, 25 = 256 bits). A 160-byte entry
// spans two 128-byte lines, so each lookup fetches 256 bytes; a packed one fetches 128
// (20.2 -> 12 KB of HBM traffic per strict verification; the unpacking, 7 funnel shifts
// and 10 masks per coordinate, costs less than the second line: DESIGN.md 5).
struct alignas(16) ge_cached_pk { uint32_t w[32]; };

NW_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_alignbit(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}
NW_HD void fe_pack(uint32_t* w, const fe& f) {
  const uint32_t* v = f.v;
  w[0] = v[0] | v[1] << 26;
  w[1] = v[1] >> 6 | v[2] << 20;
  w[2] = v[2] >> 12 | v[3] << 14;
  w[3] = v[3] >> 18 | v[4] << 7;
  w[4] = v[4] >> 25 | v[5] << 1 | v[6] << 26;
  w[5] = v[6] >> 6 | v[7] << 20;
  w[6] = v[7] >> 12 | v[8] << 13;
  w[7] = v[8] >> 19 | v[9] << 7;
}
NW_HD void fe_unpack(fe& f, const uint32_t* w) {
  f.v[0] = w[0] & M26;
  f.v[1] = funnel(w[1], w[0], 26) & M26;
  f.v[2] = funnel(w[2], w[1], 20) & M26;
  f.v[3] = funnel(w[3], w[2], 14) & M25;
  f.v[4] = funnel(w[4], w[3], 7) & M26;
  f.v[5] = (w[4] >> 1) & M25;
  f.v[6] = funnel(w[5], w[4], 26) & M26;
  f.v[7] = funnel(w[6], w[5], 20) & M25;
  f.v[8] = funnel(w[7], w[6], 13) & M26;
  f.v[9] = w[7] >> 7;
}
NW_HD void tab_put(ge_cached* t, int j, const ge_cached& c) { t[j] = c; }
NW_HD void tab_put(ge_cached_pk* t, int j, const ge_cached& c) {
  fe t2;
  fe_copy(t2, c.T2d);
  fe_carry(t2);   // a product's limbs 1 and 6 may sit just above their width
  fe_pack(t[j].w, c.YpX);
  fe_pack(t[j].w + 8, c.YmX);
  fe_pack(t[j].w + 16, c.Z2);
  fe_pack(t[j].w + 24, t2);
}
NW_HD void tab_get(const ge_cached* t, int j, ge_cached& e) { e = t[j]; }
NW_HD void tab_get(const ge_cached_pk* t, int j, ge_cached& e) {
  fe_unpack(e.YpX, t[j].w);
  fe_unpack(e.YmX, t[j].w + 8);
  fe_unpack(e.Z2, t[j].w + 16);
  fe_unpack(e.T2d, t[j].w + 24);
}

#ifndef NW_TAB_DBL
#define NW_TAB_DBL 0   // 1: four doublings + three mixed additions (0.5 % / 0.9 % slower, r02b / r06w)
#endif

template <class Tab>
NW_HD void build_table8(Tab* tab, const ge& P, const fe& d2) {
  ge_cached c1;
  ge_to_cached(c1, P, d2);
  tab_put(tab, 0, c1);
#if NW_TAB_DBL
  // P is affine (decompressed, Z = 1), so its additions are mixed (2 Z1 instead of Z1 Z2).
  // Four doublings and three mixed additions instead of one doubling and six additions,
  // as one rolled chain (one copy of each routine in the code object):
  //   2P = 2(P), 3P = 2P + P, 6P = 2(3P), 4P = 2(2P)*, 5P = 4P + P, 8P = 2(4P)*, 7P = 8P - P
  // (* restarted from the cached entry, (2X : 2Y : 2Z) without T, which a doubling ignores).
  {
    ge cur = P;
    ge_cached cj;
#pragma unroll 1
    for (int st = 0; st < 7; ++st) {
      const bool dbl = st == 0 || st == 2 || st == 3 || st == 5;
      const int dst = st == 0 ? 1 : st == 1 ? 2 : st == 2 ? 5 : st == 3 ? 3 : st == 4 ? 4 : st == 5 ? 7 : 6;
      if (st == 3 || st == 5) {   // (the entry read back in whatever form the table holds)
        ge_cached back;
        tab_get(tab, st == 3 ? 1 : 3, back);
        ge_from_cached_not(cur, back);
      }
      if (st == 6) ge_cached_cneg(c1, true);
      if (dbl) ge_dbl(cur, cur, true);
      else ge_add_any(cur, cur, c1, true, true);
      ge_to_cached(cj, cur, d2);
      tab_put(tab, dst, cj);
    }
    return;
  }
#endif
  ge acc;
  ge_dbl(acc, P, true);
  ge_cached cj;
  ge_to_cached(cj, acc, d2);
  tab_put(tab, 1, cj);
#pragma unroll 1
  for (int j = 3; j <= 8; ++j) {
    // P is affine (Z = 1): 2 Z1 Z2 = 2 Z1, one multiplication fewer than a cached addition
    ge_add_any(acc, acc, c1, true, true);
    ge_to_cached(cj, acc, d2);
    tab_put(tab, j - 1, cj);
  }
}

// Inputs of one strict verification, fetched when needed (so nothing but the decompression
// is live across the decompression): A(w) / R(w) / S(w) give the 8 LE words of the public
// key, of R and of s; k(x) gives k = H(R || A || M) mod l. The kernel's source reloads
// from global memory; the host self-check's returns copies of its arrays.
struct strict_src_arrays {
  static constexpr bool kPre = false;   // A and R decompressed here (see strict_verify_core)
  const uint32_t* a;
  const uint32_t* r;
  const uint32_t* s;
  const uint32_t* k;
  NW_HD void A(uint32_t w[8]) const { for (int i = 0; i < 8; ++i) w[i] = a[i]; }
  NW_HD void R(uint32_t w[8]) const { for (int i = 0; i < 8; ++i) w[i] = r[i]; }
  NW_HD void S(uint32_t w[8]) const { for (int i = 0; i < 8; ++i) w[i] = s[i]; }
  NW_HD void K(uint32_t w[8]) const { for (int i = 0; i < 8; ++i) w[i] = k[i]; }
};

// The B term's tables: entry ad of j * 2^(128 h) * B (h = 0, 1) into e's YpX / YmX / T2d.
// btab_pair: two 129-entry arrays (8-bit windows, LDS); btab_wide: one array of 2 x n
// padded entries (BW >= 16, global memory: k_btab_build on the device; the host self-check
// builds the 16-bit one with nw_consts.hpp compute_wide_btab).
struct btab_pair {
  const ge_niels* t0;
  const ge_niels* t1;
  NW_HD void operator()(int h, int ad, ge_cached& e) const {
    const ge_niels& nb = (h == 0 ? t0 : t1)[ad];
    fe_copy(e.YpX, nb.ypx);
    fe_copy(e.YmX, nb.ymx);
    fe_copy(e.T2d, nb.xy2d);
  }
};
struct btab_wide {
  const ge_niels_pad* t;
  uint32_t n;   // entries per half: 2^(bw-1) + 1
  NW_HD const ge_niels_pad* entry(int h, int ad) const { return t + (h ? n : 0u) + (uint32_t)ad; }
  NW_HD void operator()(int h, int ad, ge_cached& e) const {
    const ge_niels& nb = t[(h ? n : 0u) + (uint32_t)ad].n;
    fe_copy(e.YpX, nb.ypx);
    fe_copy(e.YmX, nb.ymx);
    fe_copy(e.T2d, nb.xy2d);
  }
};

// Signed BW-bit digits of w (< 2^253) for the B term: NB = ceil(253 / BW) digits, digit m at
// bit BW m. All are signed (bias 2^(BW-1)) except, when NB * BW > 256, the top one: it is
// taken unsigned (< 2^13 + 2), so the biased sum still fits 256 bits. Digits below bit 128
// use table 0 (j * B) at ladder window BW m / 4; the others table 1 (j * 2^128 B) at window
// (BW m - 128) / 4 — every position is a multiple of 4 for BW in {8, 16, 20, 24}.
template <int BW>
struct bdigits {
  static_assert(BW == 8 || BW == 16 || BW == 20 || BW == 24, "B windows of 8/16/20/24 bits");
  static constexpr int NB = (253 + BW - 1) / BW;
  static constexpr bool TOP_UNSIGNED = NB * BW > 256;
  static constexpr int NSIGNED = TOP_UNSIGNED ? NB - 1 : NB;
  static constexpr uint32_t ENTRIES = (1u << (BW - 1)) + 1;   // |d| <= 2^(BW-1)
  NW_HD static constexpr uint32_t bias_word(int i) {
    uint32_t b = 0;
    for (int m = 0; m < NSIGNED; ++m) {
      const int p = BW * m + BW - 1;
      if ((p >> 5) == i) b |= 1u << (p & 31);
    }
    return b;
  }
  // out = w + sum over signed digits of 2^(BW-1) 2^(BW m)
  NW_HD static void recode(uint32_t out[8], const sc& w) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (uint64_t)w.w[i] + bias_word(i);
      out[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  // digit m (wave-uniform) of the recoded words, word i read by get(i)
  template <class Get>
  NW_HD static int digit_g(Get get, int m) {
    const int p = BW * m, wi = p >> 5, sh = p & 31;
    const uint32_t lo = get(wi), hi = wi < 7 ? get(wi + 1) : 0u;
    const uint32_t v = (uint32_t)(((((uint64_t)hi) << 32) | lo) >> sh) & ((1u << BW) - 1);
    return m < NSIGNED ? (int)v - (1 << (BW - 1)) : (int)v;
  }
  NW_HD static int digit(const uint32_t wd[8], int m) {
    return digit_g([&](int i) { return sel8(wd, i); }, m);
  }
};

// The B tables computed on demand (host self-check only: fixed-base product + inversion
// per lookup), for window widths whose tables the host does not hold.
struct btab_lazy {
  const ge_niels* btab8;   // j * B, j = 0..128 (fixed_base_mul's table)
  const fe* d2;
  NW_HD void operator()(int h, int ad, ge_cached& e) const {
    sc s;
#pragma unroll
    for (int i = 0; i < 8; ++i) s.w[i] = 0;
    s.w[h ? 4 : 0] = (uint32_t)ad;
    ge P;
    fixed_base_mul(P, s, btab8);
    ge_niels nb;
    ge_to_niels(nb, P, *d2);
    fe_copy(e.YpX, nb.ypx);
    fe_copy(e.YmX, nb.ymx);
    fe_copy(e.T2d, nb.xy2d);
  }
};

// The B comb for keyed verifications: kBCombT tables j * 2^(W m) * B (W = kBCombW), so
// [s]B = sum_m T_m[d_m] over s's signed W-bit digits (bdigits) with no doublings. bcomb_wide: the
// device copy (global memory, padded entries); bcomb_lazy: entries computed per lookup
// (host self-check).
// B comb width (NW_BCOMBW): 24-bit digits over 11 tables j * 2^(24 m) * B, j = 0..2^23
// (11.8 GB per device, 11 additions for [s]B) or 16-bit over 16 tables (67 MB, 16 additions).
#ifndef NW_BCOMBW
#define NW_BCOMBW 24
#endif
constexpr int kBCombW = NW_BCOMBW;
constexpr int kBCombT = bdigits<NW_BCOMBW>::NB;
constexpr uint32_t kBCombN = bdigits<NW_BCOMBW>::ENTRIES;
// Committee-key comb digits at the tables' runtime width (nw_kernels.h keyspec): k + bias
// recoded once, digit t = bits W t .. W t + W - 1, signed (minus 2^(W-1)) except the top one
// when the digits overrun 256 bits — bdigits<W>'s recoding with W a value.
NW_HD void key_recode(uint32_t kd[8], const sc& k, const keyspec& ks) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)k.w[i] + ks.bias[i];
    kd[i] = (uint32_t)c;
    c >>= 32;
  }
}
NW_HD int key_digit(const uint32_t kd[8], int t, const keyspec& ks) {
  const uint32_t p = ks.W * (uint32_t)t, wi = p >> 5, sh = p & 31;
  const uint32_t lo = sel8(kd, (int)wi), hi = wi < 7 ? sel8(kd, (int)wi + 1) : 0u;
  const uint32_t v = (uint32_t)(((((uint64_t)hi) << 32) | lo) >> sh) & ((1u << ks.W) - 1u);
  return (uint32_t)t < ks.nsigned ? (int)v - (1 << (ks.W - 1)) : (int)v;
}
struct bcomb_wide {
  const ge_niels_pad* t;
  NW_HD const ge_niels_pad* entry(int m, int ad) const {
    return t + (uint32_t)m * kBCombN + (uint32_t)ad;
  }
  NW_HD void operator()(int m, int ad, ge_cached& e) const {
    const ge_niels& nb = t[(uint32_t)m * kBCombN + (uint32_t)ad].n;
    fe_copy(e.YpX, nb.ypx);
    fe_copy(e.YmX, nb.ymx);
    fe_copy(e.T2d, nb.xy2d);
  }
};
struct bcomb_lazy {
  const ge_niels* btab8;
  const fe* d2;
  NW_HD void operator()(int m, int ad, ge_cached& e) const {
    sc s;
#pragma unroll
    for (int i = 0; i < 8; ++i) s.w[i] = 0;
    const int bit = kBCombW * m, wi = bit >> 5, sh = bit & 31;
    s.w[wi] = (uint32_t)ad << sh;
    if (sh && wi < 7) s.w[wi + 1] = (uint32_t)ad >> (32 - sh);
    ge P;
    fixed_base_mul(P, s, btab8);
    ge_niels nb;
    ge_to_niels(nb, P, *d2);
    fe_copy(e.YpX, nb.ypx);
    fe_copy(e.YmX, nb.ymx);
    fe_copy(e.T2d, nb.xy2d);
  }
};

// Table-entry prefetch for the strict ladder. pf_none: each addition reads its entry from
// its table when it runs (host self-check; NW_STRICT_PF=0). The device's LDS prefetcher
// (nw_kernels.hip pf_lds) loads the NEXT addition's entry straight into LDS
// (global_load_lds_dwordx4, no registers) while the current addition or the window's four
// doublings run, so the ladder's ~77 dependent table loads per verification stop stalling
// the wave. issue(src, chunks): 16-byte chunks at src (8: a packed per-lane entry or a
// ge_niels_pad; 10: an unpacked ge_cached); get(e, niels): wait for it and read it (niels:
// Y+x, Y-x, xy2d into YpX, YmX, T2d).
// A prefetcher may also hold the ladder's digit words (lds_digits: dput(k, word) once after
// the recoding, dget(k) per addition; words 0-7 u, 8-12 |v|, 13-20 w): the words are read
// with a wave-uniform index, which the compiler otherwise serves from a scratch array (a
// dependent scratch load per addition).
struct pf_none {
  static constexpr bool enabled = false;
  static constexpr bool lds_digits = false;
  NW_HD void issue(const void*, int) const {}
  NW_HD void get(ge_cached&, bool) const {}
  NW_HD void get_signed(ge_cached&, bool) const {}
  NW_HD void dput(int, uint32_t) const {}
  NW_HD uint32_t dget(int) const { return 0; }
};

// A committee key's comb tables: keytab_wide reads the device copy (keytab[ks.nent t + j]
// = j * 2^(W t) A, affine niels, built by k_key_tabs); keytab_lazy computes an entry per
// lookup from A (host self-check: the full 16-bit tables are 67 MB per key).
struct keytab_wide {
  const ge_niels_pad* t;
  keyspec ks;
  NW_HD const ge_niels_pad* entry(int tab, int j) const {
    return t + (uint32_t)tab * ks.nent + (uint32_t)j;
  }
  NW_HD void operator()(int tab, int j, ge_niels& e) const {
    e = t[(uint32_t)tab * ks.nent + (uint32_t)j].n;
  }
};
struct keytab_lazy {
  const ge* A;
  const fe* d2;
  keyspec ks;
  NW_HD void operator()(int tab, int j, ge_niels& e) const {
    ge P = *A;
    for (int d = 0; d < (int)ks.W * tab; ++d) ge_dbl(P, P, true);
    ge_cached c;
    ge_to_cached(c, P, *d2);
    ge acc;
    ge_identity(acc);
    for (int bit = (int)ks.W - 1; bit >= 0; --bit) {
      ge_dbl(acc, acc, true);
      if ((j >> bit) & 1) ge_add_cached(acc, acc, c, true);
    }
    ge_to_niels(e, acc, *d2);
  }
};

// acc = [s]B - [k]A for k, s < l: -[k]A as k's ceil(253 / W) W-bit digits against the
// key's comb tables (kt), [s]B as s's 16 signed 16-bit digits against the B comb (bc). No
// doublings.
#ifndef NW_KEYED_SPLIT
#define NW_KEYED_SPLIT 0   // 1: the A and B terms in two interleaved accumulators (ILP)
#endif
template <class BComb, class KeyTab, class PF = pf_none>
NW_HD void keyed_comb_sum(ge& acc, const sc& k, const sc& s, const BComb& bc,
                          const KeyTab& kt, const fe& d2, const PF& pf = PF{}) {
  uint32_t kd[8], sd[8];
  const keyspec& ks = kt.ks;
  key_recode(kd, k, ks);              // k < l: ceil(253 / W) W-bit digits
  bdigits<kBCombW>::recode(sd, s);    // s < l: kBCombT digits of kBCombW bits
  ge_identity(acc);
  if constexpr (PF::enabled) {
    // the same additions in the same order, each entry requested one addition ahead
    // (pf_lds: global_load_lds into a per-lane LDS slot while the current addition runs)
    const int KT = (int)ks.ntab, NS = KT + kBCombT;
    auto step_src = [&](int st, int& d) -> const void* {
      if (st < KT) {
        d = key_digit(kd, st, ks);
        return d ? static_cast<const void*>(kt.entry(st, d < 0 ? -d : d)) : nullptr;
      }
      d = bdigits<kBCombW>::digit(sd, st - KT);
      return d ? static_cast<const void*>(bc.entry(st - KT, d < 0 ? -d : d)) : nullptr;
    };
    {
      int d0;
      const void* s0 = step_src(0, d0);
      if (s0) pf.issue(s0, 8);
    }
#pragma unroll 1
    for (int st = 0; st < NS; ++st) {
      int d;
      const void* cur = step_src(st, d);
      ge_cached e;
      if (cur) pf.get(e, true);
      if (st + 1 < NS) {
        int dn;
        const void* nx = step_src(st + 1, dn);
        if (nx) pf.issue(nx, 8);
      }
      if (cur) {
        ge_cached_cneg(e, st < KT ? d > 0 : d < 0);   // -[k]A: key digits negated
        ge_add_any(acc, acc, e, true, true);
      }
    }
    (void)d2;
    return;
  }
#if NW_KEYED_SPLIT
  // two independent chains, one step of each per iteration: -[k]A in acc, [s]B in accB,
  // joined by one cached addition (T3 not needed by the callers' comparisons)
  ge accB;
  ge_identity(accB);
#pragma unroll 1
  for (int t = 0; t < ((int)ks.ntab > kBCombT ? (int)ks.ntab : kBCombT); ++t) {
    if (t < (int)ks.ntab) {
      const int d = key_digit(kd, t, ks);
      if (d != 0) {
        ge_niels nb;
        kt(t, d < 0 ? -d : d, nb);
        ge_niels_cneg(nb, d > 0);
        ge_add_niels(acc, acc, nb, true);
      }
    }
    if (t < kBCombT) {
      const int e = bdigits<kBCombW>::digit(sd, t);
      if (e != 0) {
        ge_cached c;
        bc(t, e < 0 ? -e : e, c);
        ge_cached_cneg(c, e < 0);
        ge_add_any(accB, accB, c, true, true);
      }
    }
  }
  ge_cached cb;
  ge_to_cached(cb, accB, d2);
  ge_add_cached(acc, acc, cb, false);
  return;
#else
  (void)d2;
#endif
  // -[k]A: digit t of k against table t, negated
#pragma unroll 1
  for (int t = 0; t < (int)ks.ntab; ++t) {
    const int d = key_digit(kd, t, ks);
    if (d != 0) {
      ge_niels nb;
      kt(t, d < 0 ? -d : d, nb);
      ge_niels_cneg(nb, d > 0);
      ge_add_niels(acc, acc, nb, true);
    }
  }
  // +[s]B
#pragma unroll 1
  for (int m = 0; m < kBCombT; ++m) {
    const int d = bdigits<kBCombW>::digit(sd, m);
    if (d != 0) {
      ge_cached e;
      bc(m, d < 0 ? -d : d, e);
      ge_cached_cneg(e, d < 0);
      ge_add_any(acc, acc, e, true, true);
    }
  }
}

// Keyed check of a certificate vote WITHOUT decompressing R (pass / fail only: a failing
// vote sends its certificate to its own verify_batch, which names the failure). With
// R' = [s]B - [k]A and y_R, sign = R's encoding (y taken unreduced as dalek does, so y >= p
// means y - p), dalek's verify_strict passes iff s has no high bits, A decodes, s < l, R
// decodes, neither R nor A is small and R' == decode(R). Since R' is a curve point,
// Y' == y_R Z' means R' = (+-x0, y_R) for the root x0 >= 0 of y_R (so R decodes, to
// (sign ? -x0 : x0, y_R)); R' == decode(R) then iff x0 == 0 (X' == 0) or the parity of
// X'/Z' equals the sign bit. Returns kVotePass / kVoteFail, or kVotePending (| sign) when
// only that parity is left: the caller batches the inversions of Z' (k_votes_keyed_inv).
constexpr uint32_t kVotePass = 0, kVoteFail = 1, kVotePending = 2;
template <class BComb, class KeyTab, class Src, class PF = pf_none>
NW_HD uint32_t keyed_vote_check(const Src& src, const strict_consts& K, const BComb& bc,
                                const KeyTab& keytab, uint32_t keyflags, fe& X, fe& Z,
                                const PF& pf = PF{}) {
  const bool okA = (keyflags & kKeyDecoded) != 0, smallA = (keyflags & kKeySmall) != 0;
  // a key with a torsion component: a strict pass does not make its batch term vanish
  // (dalek weights A by z k mod l), so its votes take the certificate's own verify_batch
  const bool torsionA = (keyflags & kKeyLambdaMask) != 0;
  uint32_t Sw[8];
  src.S(Sw);
  sc s;
#pragma unroll
  for (int j = 0; j < 8; ++j) s.w[j] = Sw[j];
  if ((Sw[7] >> 29) != 0 || !okA || smallA || torsionA || !sc_is_canonical(s)) return kVoteFail;
  uint32_t Rw[8];
  src.R(Rw);
  const uint32_t sign = Rw[7] >> 31;
  fe yR;
  fe_frombytes(yR, Rw);
  if (small_order_by_y(yR, K.small_y)) return kVoteFail;   // R small (if it decodes at all)
  uint32_t kw[8];
  src.K(kw);
  sc k;
#pragma unroll
  for (int j = 0; j < 8; ++j) k.w[j] = kw[j];
  ge acc;
  keyed_comb_sum(acc, k, s, bc, keytab, K.k.d2, pf);
  fe t;
  fe_mul(t, yR, acc.Z);
  if (!fe_eq(t, acc.Y)) return kVoteFail;
  if (fe_iszero(acc.X)) return kVotePass;
  fe_copy(X, acc.X);
  fe_copy(Z, acc.Z);
  return kVotePending | sign;
}

// Keyed strict verification: A is a committee key with comb tables j * 2^(W t) A
// (keytab_wide / keytab_lazy; affine niels), keyflags bit 0 = decoded, bit 1 = small
// order. Then R' = [s]B - [k]A is 16 + 256 / W table additions with no doublings and no
// scalar split, and the equation is dalek's own projective comparison R == R' (R decompressed,
// Z = 1). Same checks and order as strict_verify_core; A is neither decompressed nor
// tabulated per signature.
template <class BComb, class KeyTab, class Src>
NW_HD int strict_keyed_comb(const Src& src, const strict_consts& K, const BComb& bc,
                            const KeyTab& keytab, uint32_t keyflags) {
  const bool okA = (keyflags & kKeyDecoded) != 0, smallA = (keyflags & kKeySmall) != 0;
  ge R;
  bool okR, smallR;
  {
    uint32_t x[8];
    src.R(x);
    okR = ge_frombytes(R, x, K.k);
    smallR = small_order_by_y(R.Y, K.small_y);
  }
  uint32_t Sw[8];
  src.S(Sw);
  sc s;
#pragma unroll
  for (int j = 0; j < 8; ++j) s.w[j] = Sw[j];
  const bool s_high = (Sw[7] >> 29) != 0;
  const bool s_canon = sc_is_canonical(s);
  // Reference order: crypto/src/lib.rs:201 (s high bits), 202 (decompress A), then dalek
  // verify_strict: check_scalar, decompress R, small order (R || A), equation.
  if (s_high) return NW_ERR_S_HIGH_BITS;
  if (!okA) return NW_ERR_A_DECODE;
  if (!s_canon) return NW_ERR_S_NONCANONICAL;
  if (!okR) return NW_ERR_R_DECODE;
  if (smallR) return NW_ERR_R_SMALL_ORDER;
  if (smallA) return NW_ERR_A_SMALL_ORDER;
  uint32_t kw[8];
  src.K(kw);
  sc k;
#pragma unroll
  for (int j = 0; j < 8; ++j) k.w[j] = kw[j];
  ge acc;
  keyed_comb_sum(acc, k, s, bc, keytab, K.k.d2);
  return ge_eq_affine(acc, R) ? NW_OK : NW_ERR_EQUATION;
}


// Status of one strict verification. wave_max maps this lane's ladder length (in 4-bit
// windows) to the wave's maximum (identity on the host). tabA/tabR: 8 entries each of
// per-lane scratch. bt: j*B and j*2^128 B, j = 0..2^(BW-1) (btab_pair / btab_wide).
// NW_STRICT_STOP (instrumentation builds only, tools/strict_phases.sh; 0 = the kernel): cut
// the verification after a phase so that PMC instruction counts of the cut builds split the
// kernel's work by phase: 1 the two decompressions, 2 + the per-lane tables, 3 + SHA-512 and
// Barrett (k), 4 + the scalar split and recodings, 5 + the ladder's doublings only (no
// additions), 6 + the A and R additions (no B additions). The status is then a digest of the
// state, not a verdict.
#ifndef NW_STRICT_STOP
#define NW_STRICT_STOP 0
#endif
// NW_PF_SWAP (default 1; 0 = the round-5 form): a per-lane entry's sign taken in the
// prefetcher's LDS read (pf_lds::get_signed) instead of 20 selects after it.
#ifndef NW_PF_SWAP
#define NW_PF_SWAP 1
#endif
// NW_ADD_NEGC (default 1): the ladder's additions as ge_add_any_negc (no carry pass on f).
// Both together: +0.4 % / +0.7 % in one process on two boxes (profiles/r06d, r06e).
#ifndef NW_ADD_NEGC
#define NW_ADD_NEGC 1
#endif
// The checks before the equation, as k_strict_triage runs them (config 4 in two passes,
// nw_kernels.hip): s's high bits and canonical form, A's and R's decompression and small
// order, in strict_verify_core's order. Returns the status of an item that fails one of
// them, NW_OK otherwise; xa / xr get the x of A and R (the rest of each point is its
// encoding's y, Z = 1 and T = x y: exactly what ge_frombytes returned).
template <class Src>
NW_HD int strict_triage(const Src& src, const strict_consts& K, fe& xa, fe& xr) {
  uint32_t Sw[8];
  src.S(Sw);
  const bool s_high = (Sw[7] >> 29) != 0;
  sc s;
#pragma unroll
  for (int t = 0; t < 8; ++t) s.w[t] = Sw[t];
  const bool s_canon = sc_is_canonical(s);
  bool okA = false, okR = false, smallA = false, smallR = false;
  // A, then R, in one rolled loop (one copy of the square-root chain: registers, code size)
#pragma unroll 1
  for (int pt = 0; pt < 2; ++pt) {
    uint32_t w[8];
    if (pt) src.R(w); else src.A(w);
    ge P;
    const bool ok = ge_frombytes(P, w, K.k);
    const bool small = small_order_by_y(P.Y, K.small_y);
    if (pt == 0) { okA = ok; smallA = small; xa = P.X; } else { okR = ok; smallR = small; xr = P.X; }
  }
  return s_high ? NW_ERR_S_HIGH_BITS : !okA ? NW_ERR_A_DECODE
       : !s_canon ? NW_ERR_S_NONCANONICAL : !okR ? NW_ERR_R_DECODE
       : smallR ? NW_ERR_R_SMALL_ORDER : smallA ? NW_ERR_A_SMALL_ORDER : NW_OK;
}

template <int BW, class BTab, class Src, class WaveMax, class PF = pf_none, class Tab = ge_cached>
NW_HD int strict_verify_core(const Src& src, const strict_consts& K, const BTab& bt,
                             Tab* tabA, Tab* tabR,
                             WaveMax wave_max, const PF& pf = PF{}) {
  using BD = bdigits<BW>;
  // Decompress A, then R, in one rolled loop (one copy of the sqrt_ratio_i chain in the
  // code object): P, its small-order flag and its 8-entry table j * P. Only the point is
  // live here: the scalars are computed afterwards (register pressure).
  bool okA = false, smallA = false, okR = false, smallR = false;
#pragma unroll 1
  for (int pt = 0; pt < 2; ++pt) {
    ge P;
    bool ok;
    if constexpr (Src::kPre) {
      // the point was decompressed by an earlier pass (k_strict_triage): the same limbs
      ok = src.point(pt, P);
    } else {
      uint32_t x[8];
      if (pt) src.R(x); else src.A(x);
      ok = ge_frombytes(P, x, K.k);
    }
    const bool small = small_order_by_y(P.Y, K.small_y);
    if (pt == 0) { okA = ok; smallA = small; } else { okR = ok; smallR = small; }
    if (NW_STRICT_STOP == 1) continue;
    build_table8(pt ? tabR : tabA, P, K.k.d2);
  }
  if (NW_STRICT_STOP == 1 || NW_STRICT_STOP == 2)
    return (okA ? 1 : 0) + (okR ? 2 : 0) + (smallA ? 4 : 0) + (smallR ? 8 : 0);

  uint32_t Sw[8], kw[8];
  src.S(Sw);
  src.K(kw);
  const bool s_high = (Sw[7] >> 29) != 0;
  sc s, k;
#pragma unroll
  for (int j = 0; j < 8; ++j) { s.w[j] = Sw[j]; k.w[j] = kw[j]; }
  if (NW_STRICT_STOP == 3) return (int)((kw[0] ^ kw[7] ^ Sw[0]) & 15u) + (okA ? 16 : 0);
  const bool s_canon = sc_is_canonical(s);
  // v < 0: [v]R = [|v|](-R), taken as negated R digits (the table holds j * R)
  sc_half h;
  sc_half_split(h, k);

  // w = -v s mod l (s zeroed when invalid: the verdict is already decided)
  sc vm, w;
#pragma unroll
  for (int j = 0; j < 8; ++j) vm.w[j] = j < 5 ? h.v[j] : 0u;
  if (!s_canon || s_high) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s.w[j] = 0;
  }
  sc_mul(w, vm, s);
  if (!h.vneg) sc_neg(w, w);
  // signed digits: u, |v| in 4-bit windows; w0 = w mod 2^128, w1 = w >> 128 in BW-bit
  // windows (one signed recoding of the whole w: digit m of w1 is digit m + 128 / BW of w,
  // the carry out of w0's top digit flows into w1's bottom one)
  sc ur, vr;
#pragma unroll
  for (int j = 0; j < 8; ++j) { ur.w[j] = h.u[j]; vr.w[j] = vm.w[j]; }
  uint32_t ud[8], vd[8], wd[8];
  const uint32_t ubias = 0x88888888u;
  sc_recode(ud, ur, ubias);
  sc_recode(vd, vr, 0x88888888u);
  BD::recode(wd, w);
  // ladder length in 4-bit windows: up to the highest nonzero signed digit of u and |v|
  // (digit j is nonzero iff nibble j of the recoded word is not 8), at least 32 for the
  // two 128-bit halves of w
  uint32_t xu[8], xv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { xu[j] = ud[j] ^ ubias; xv[j] = vd[j] ^ 0x88888888u; }
  const int bu = bn_bits(xu, 8), bv = bn_bits(xv, 5);
  int W = ((bu > bv ? bu : bv) + 3) / 4;
  if (W < 32) W = 32;
  W = wave_max(W);
  if (NW_STRICT_STOP == 4) return W + (int)((ud[0] ^ vd[0] ^ wd[0] ^ wd[7]) & 15u) + (okR ? 64 : 0);

  // One rolled doubling and one addition routine serve every term (code size: the ladder
  // body stays inside the instruction cache). Per 4-bit window j: 4 doublings, then the
  // A digit, the R digit and, on j < 32, the B digits at this window (bdigits: at most one
  // per table).
  ge acc;
  ge_identity(acc);
  if constexpr (PF::enabled) {
    // The same additions in the same order as below; the entry of addition (j, slot) is
    // requested one addition ahead (window j's first one before its doublings).
    if constexpr (PF::lds_digits) {
#pragma unroll
      for (int t = 0; t < 8; ++t) { pf.dput(t, ud[t]); pf.dput(13 + t, wd[t]); }
#pragma unroll
      for (int t = 0; t < 5; ++t) pf.dput(8 + t, vd[t]);
    }
    // digit j of u / |v| (4-bit, biased by 8) and digit m of w
    auto dig4 = [&](int base, int nw, const uint32_t* arr, int j) -> int {
      if constexpr (PF::lds_digits) {
        const uint32_t word = (j >> 3) < nw ? pf.dget(base + (j >> 3)) : 0x88888888u;
        return (int)((word >> ((j & 7) * 4)) & 15u) - 8;
      } else {
        return digit4_of(arr, nw, j);
      }
    };
    auto digw = [&](int m) -> int {
      if constexpr (PF::lds_digits) return BD::digit_g([&](int i) { return pf.dget(13 + i); }, m);
      else return BD::digit(wd, m);
    };
    auto slot_src = [&](int j, int slot, int& d, bool& niels) -> const void* {
      const int p0 = 4 * j, p1 = 4 * j + 128;
      const bool has0 = j < 32 && p0 % BW == 0;
      niels = slot >= 2;
      if (slot == 0) {
        d = dig4(0, 8, ud, j);
      } else if (slot == 1) {
        d = j < 40 ? dig4(8, 5, vd, j) : 0;
        if (h.vneg) d = -d;
      } else {
        const bool t1 = slot == 3 || !has0;
        d = digw(t1 ? p1 / BW : p0 / BW);
        return d ? static_cast<const void*>(bt.entry(t1 ? 1 : 0, d < 0 ? -d : d)) : nullptr;
      }
      const int ad = d < 0 ? -d : d;
      return d ? static_cast<const void*>((slot == 0 ? tabA : tabR) + (ad - 1)) : nullptr;
    };
    auto nslots_of = [&](int j) {
      const int p0 = 4 * j, p1 = 4 * j + 128;
      const bool has0 = j < 32 && p0 % BW == 0;
      const bool has1 = j < 32 && p1 % BW == 0 && p1 / BW < BD::NB;
      return 2 + (has0 ? 1 : 0) + (has1 ? 1 : 0);
    };
    {
      int d0;
      bool nl0;
      const void* s0 = slot_src(W - 1, 0, d0, nl0);
      if (s0 && NW_STRICT_STOP != 5) pf.issue(s0, nl0 ? 8 : int(sizeof(Tab) / 16));
    }
#pragma unroll 1
    for (int j = W - 1; j >= 0; --j) {
      if (j != W - 1) {
#pragma unroll 1
        for (int t = 0; t < 4; ++t) ge_dbl(acc, acc, t == 3);
      }
      if (NW_STRICT_STOP == 5) continue;
      const int nslots = NW_STRICT_STOP == 6 ? 2 : nslots_of(j);
#pragma unroll 1
      for (int slot = 0; slot < nslots; ++slot) {
        int d;
        bool niels;
        const void* cur = slot_src(j, slot, d, niels);
        ge_cached e;
#if NW_PF_SWAP
        if (cur) {
          if (niels) pf.get(e, true);
          else pf.get_signed(e, d < 0);
        }
#else
        if (cur) pf.get(e, niels);
#endif
        // request the next addition's entry before this one runs
        const int j2 = slot + 1 < nslots ? j : j - 1, s2 = slot + 1 < nslots ? slot + 1 : 0;
        if (j2 >= 0) {
          int d2;
          bool n2;
          const void* nx = slot_src(j2, s2, d2, n2);
          if (nx) pf.issue(nx, n2 ? 8 : int(sizeof(Tab) / 16));
        }
        if (cur) {
          // NW_ADD_NEGC: 2dT negated when the digit is positive (ge_add_any_negc)
          const bool tneg = NW_ADD_NEGC ? d > 0 : d < 0;
#if NW_PF_SWAP
          if (niels) {
            if (NW_ADD_NEGC) ge_cached_cneg_negc(e, d < 0);
            else ge_cached_cneg(e, d < 0);
          } else {   // Y+X / Y-X already swapped by the read: -2dT only
            fe t;
            fe_neg_nc(t, e.T2d);
            fe_cmov(e.T2d, t, tneg);
          }
#else
          if (NW_ADD_NEGC) ge_cached_cneg_negc(e, d < 0);
          else ge_cached_cneg(e, d < 0);
#endif
          if (NW_ADD_NEGC) ge_add_any_negc(acc, acc, e, niels, slot != nslots - 1);
          else ge_add_any(acc, acc, e, niels, slot != nslots - 1);
        }
      }
    }
  } else {
#pragma unroll 1
  for (int j = W - 1; j >= 0; --j) {
    if (j != W - 1) {
#pragma unroll 1
      for (int t = 0; t < 4; ++t) ge_dbl(acc, acc, t == 3);
    }
    const int p0 = 4 * j, p1 = 4 * j + 128;
    const bool has0 = j < 32 && p0 % BW == 0;
    const bool has1 = j < 32 && p1 % BW == 0 && p1 / BW < BD::NB;
    const int nslots = 2 + (has0 ? 1 : 0) + (has1 ? 1 : 0);
#pragma unroll 1
    for (int slot = 0; slot < nslots; ++slot) {
      int d;
      if (slot == 0) {
        d = digit4_of(ud, 8, j);
      } else if (slot == 1) {
        d = j < 40 ? digit4_of(vd, 5, j) : 0;
        if (h.vneg) d = -d;
      } else {
        // the table-0 digit first (when present), then the table-1 digit
        const bool t1 = slot == 3 || !has0;
        d = BD::digit(wd, t1 ? p1 / BW : p0 / BW);
      }
      if (d != 0) {
        const int ad = d < 0 ? -d : d;
        ge_cached e;
        if (slot < 2) {
          tab_get(slot == 0 ? tabA : tabR, ad - 1, e);
        } else {
          bt((slot == 3 || !has0) ? 1 : 0, ad, e);
        }
        if (NW_ADD_NEGC) {
          ge_cached_cneg_negc(e, d < 0);
          ge_add_any_negc(acc, acc, e, slot >= 2, slot != nslots - 1);
        } else {
          ge_cached_cneg(e, d < 0);
          ge_add_any(acc, acc, e, slot >= 2, slot != nslots - 1);
        }
      }
    }
  }
  }
  const bool eq = ge_is_identity(acc);
  // Reference order: crypto/src/lib.rs:201 (s high bits), 202 (decompress A), then dalek
  // verify_strict: check_scalar, decompress R, small order (R || A), equation.
  if (s_high) return NW_ERR_S_HIGH_BITS;
  if (!okA) return NW_ERR_A_DECODE;
  if (!s_canon) return NW_ERR_S_NONCANONICAL;
  if (!okR) return NW_ERR_R_DECODE;
  if (smallR) return NW_ERR_R_SMALL_ORDER;
  if (smallA) return NW_ERR_A_SMALL_ORDER;
  if (!eq) return NW_ERR_EQUATION;
  return NW_OK;
}

}  // namespace nw
