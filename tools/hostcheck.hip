// hostcheck.hip — TEST INFRASTRUCTURE. Exposes the device arithmetic headers (compiled as
// host code) through a C ABI so tests/test_hostcheck.py can compare the exact field /
// point / scalar / ladder code the kernels run against the CPU oracle, without a GPU.
// SHA-512 is device-only, so the verification entry takes k = H(R||A||M) mod l as input.
#include <string.h>
#include "../narwhal_amd/csrc/nw_consts.hpp"
#include "../narwhal_amd/csrc/nw_ladder.hpp"

using namespace nw;

static curve_consts K;
static ge_niels BT[129];
static strict_consts SK;
static ge_niels B128[129];
static ge_niels_pad* BTW = nullptr;   // 16-bit-window tables (the kernel's default)
static const uint32_t BTW_N = (1u << 15) + 1;
static bool ready = false;
static void init() {
  if (!ready) {
    compute_consts(K, BT);
    compute_strict_consts(SK, B128);
    BTW = new ge_niels_pad[2 * BTW_N];
    compute_wide_btab(BTW, 16);
    ready = true;
  }
}

static void load8(uint32_t w[8], const uint8_t* b) { memcpy(w, b, 32); }
static void store8(uint8_t* b, const uint32_t w[8]) { memcpy(b, w, 32); }

extern "C" {

int hc_decompress(const uint8_t in[32], uint8_t out[32]) {
  init();
  uint32_t w[8]; load8(w, in);
  ge p;
  if (!ge_frombytes(p, w, K)) return 0;
  uint32_t o[8]; ge_tobytes(o, p); store8(out, o);
  return 1;
}

int hc_is_small_order(const uint8_t in[32]) {
  init();
  uint32_t w[8]; load8(w, in);
  ge p;
  if (!ge_frombytes(p, w, K)) return -1;
  return ge_is_small_order(p) ? 1 : 0;
}

void hc_reduce512(const uint8_t in[64], uint8_t out[32]) {
  uint32_t x[16]; memcpy(x, in, 64);
  sc r; sc_reduce512(r, x); store8(out, r.w);
}

void hc_scalar_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  sc x, y, r; load8(x.w, a); load8(y.w, b); sc_mul(r, x, y); store8(out, r.w);
}

void hc_scalar_add(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  sc x, y, r; load8(x.w, a); load8(y.w, b); sc_add(r, x, y); store8(out, r.w);
}

int hc_scalar_canonical(const uint8_t a[32]) { sc x; load8(x.w, a); return sc_is_canonical(x); }

void hc_fixed_base(const uint8_t s[32], uint8_t out[32]) {
  init();
  sc x; load8(x.w, s);
  ge r; fixed_base_mul(r, x, BT);
  uint32_t o[8]; ge_tobytes(o, r); store8(out, o);
}

// [b]B + [a]P
int hc_dsm(const uint8_t a[32], const uint8_t P[32], const uint8_t b[32], uint8_t out[32]) {
  init();
  uint32_t w[8]; load8(w, P);
  ge p;
  if (!ge_frombytes(p, w, K)) return 0;
  ge_cached tab[9]; build_table9(tab, p, K.d2);
  sc x, y; load8(x.w, a); load8(y.w, b);
  ge r; dsm_var_base(r, tab, x, y, BT);
  uint32_t o[8]; ge_tobytes(o, r); store8(out, o);
  return 1;
}

// Strict verification with the kernel's check order; k supplied (device-only SHA).
int hc_verify_strict(const uint8_t pk[32], const uint8_t sig[64], const uint8_t k32[32]) {
  init();
  uint32_t Aw[8], Rw[8], Sw[8];
  load8(Aw, pk); load8(Rw, sig); load8(Sw, sig + 32);
  const bool s_high = (Sw[7] >> 29) != 0;
  sc s; memcpy(s.w, Sw, 32);
  const bool s_canon = sc_is_canonical(s);
  ge A, R;
  const bool okA = ge_frombytes(A, Aw, K);
  const bool okR = ge_frombytes(R, Rw, K);
  const bool smallA = ge_is_small_order(A), smallR = ge_is_small_order(R);
  sc k; load8(k.w, k32);
  ge mA; ge_neg(mA, A);
  ge_cached tab[9]; build_table9(tab, mA, K.d2);
  if (!s_canon || s_high) memset(s.w, 0, 32);
  ge acc; dsm_var_base(acc, tab, k, s, BT);
  const bool eq = ge_eq_affine(acc, R);
  if (s_high) return 1;
  if (!okA) return 3;
  if (!s_canon) return 2;
  if (!okR) return 4;
  if (smallR) return 6;
  if (smallA) return 5;
  if (!eq) return 7;
  return 0;
}


// Half-size scalar split (nw_scalar.hpp): u (32 bytes), |v| (20 bytes), sign.
int hc_half_split(const uint8_t k32[32], uint8_t u32[32], uint8_t v20[20]) {
  sc k; load8(k.w, k32);
  sc_half h; sc_half_split(h, k);
  memcpy(u32, h.u, 32); memcpy(v20, h.v, 20);
  return h.vneg ? 1 : 0;
}

// The same split by single Euclid steps only (the reference for the Lehmer rounds).
int hc_half_split_onestep(const uint8_t k32[32], uint8_t u32[32], uint8_t v20[20]) {
  sc k; load8(k.w, k32);
  sc_half h; sc_half_split<false>(h, k);
  memcpy(u32, h.u, 32); memcpy(v20, h.v, 20);
  return h.vneg ? 1 : 0;
}

// The kernel's strict verification (nw_strict.hpp), k supplied (device-only SHA), with
// B windows of bw = 16 bits (wide tables; the host-built copy), 8 bits (LDS tables) or
// 20 / 24 bits (entries computed per lookup). bw < 0: |bw| with the per-lane tables packed
// into 128-byte entries (ge_cached_pk, NW_PACK_TAB).
int hc_verify_strict_half(const uint8_t pk[32], const uint8_t sig[64], const uint8_t k32[32],
                          int bw) {
  init();
  uint32_t Aw[8], Rw[8], Sw[8];
  load8(Aw, pk); load8(Rw, sig); load8(Sw, sig + 32);
  uint32_t kw[8]; load8(kw, k32);
  ge_cached ta[8], tr[8];
  const strict_src_arrays src{Aw, Rw, Sw, kw};
  auto id = [](int w) { return w; };
  if (bw < 0) {
    ge_cached_pk pa[8], pr[8];
    if (bw == -24) return strict_verify_core<24>(src, SK, btab_lazy{BT, &SK.k.d2}, pa, pr, id);
    return strict_verify_core<16>(src, SK, btab_wide{BTW, BTW_N}, pa, pr, id);
  }
  if (bw == 8) return strict_verify_core<8>(src, SK, btab_pair{BT, B128}, ta, tr, id);
  if (bw == 20) return strict_verify_core<20>(src, SK, btab_lazy{BT, &SK.k.d2}, ta, tr, id);
  if (bw == 24) return strict_verify_core<24>(src, SK, btab_lazy{BT, &SK.k.d2}, ta, tr, id);
  return strict_verify_core<16>(src, SK, btab_wide{BTW, BTW_N}, ta, tr, id);
}

// Config 4 in two passes, on the host: strict_triage (k_strict_triage's checks), then, for an
// item that passes them, strict_verify_core on the stored x of A and R (the kPre source, as
// k_verify_strict_pre's strict_src_pre) with B windows of |bw| bits and packed tables as
// hc_verify_strict_half(bw < 0). Must equal the one-pass status for every input.
struct src_arrays_pre : strict_src_arrays {
  static constexpr bool kPre = true;
  fe xa, xr;
  bool point(int pt, ge& P) const {
    uint32_t w[8];
    if (pt) R(w); else A(w);
    fe_frombytes(P.Y, w);
    P.X = pt ? xr : xa;
    fe_1(P.Z);
    fe_mul(P.T, P.X, P.Y);
    return true;
  }
};
int hc_verify_strict_twopass(const uint8_t pk[32], const uint8_t sig[64], const uint8_t k32[32],
                             int bw) {
  init();
  uint32_t Aw[8], Rw[8], Sw[8], kw[8];
  load8(Aw, pk); load8(Rw, sig); load8(Sw, sig + 32); load8(kw, k32);
  src_arrays_pre src{};
  src.a = Aw; src.r = Rw; src.s = Sw; src.k = kw;
  const int st = strict_triage(static_cast<const strict_src_arrays&>(src), SK, src.xa, src.xr);
  if (st != NW_OK) return st;
  ge_cached_pk pa[8], pr[8];
  auto id = [](int w) { return w; };
  if (bw == -24) return strict_verify_core<24>(src, SK, btab_lazy{BT, &SK.k.d2}, pa, pr, id);
  return strict_verify_core<16>(src, SK, btab_wide{BTW, BTW_N}, pa, pr, id);
}

// The keyed strict path (nw_strict.hpp strict_keyed_comb): the key's comb table entries
// j * 2^(W t) A computed per lookup (keytab_lazy) by the definition the device's k_key_base /
// k_key_tabs tabulate, the B comb likewise. Returns the status; -1 when A does not decode is reported through the
// key flags exactly as the device does (status 3).
static uint32_t keyed_key(ge& A, const uint32_t Aw[8]) {
  const bool dec = ge_frombytes(A, Aw, K);
  uint32_t lam = 0;
  if (dec) {   // [l] A == [lambda] T8, as k_key_base computes it
    static torsion_consts tc;
    static bool have = false;
    if (!have) { compute_torsion(tc); have = true; }
    ge_cached Pc;
    ge_to_cached(Pc, A, K.d2);
    ge acc;
    ge_identity(acc);
    for (int bit = 252; bit >= 0; --bit) {
      ge_dbl(acc, acc, true);
      if ((L_W[bit >> 5] >> (bit & 31)) & 1u) ge_add_cached(acc, acc, Pc, true);
    }
    const int j = torsion_index(acc, tc);
    lam = j > 0 ? (uint32_t)j : 0u;
  }
  return (dec ? kKeyDecoded : 0u) | (dec && ge_is_small_order(A) ? kKeySmall : 0u) |
         (lam << kKeyLambdaShift);
}

// lambda of a key (bits 2..4 of the flag word): [l] A == [lambda] T8; -1 if A does not decode.
int hc_key_lambda(const uint8_t pk[32]) {
  init();
  uint32_t Aw[8];
  load8(Aw, pk);
  ge A;
  const uint32_t f = keyed_key(A, Aw);
  return (f & kKeyDecoded) ? (int)((f & kKeyLambdaMask) >> kKeyLambdaShift) : -1;
}

// Comb width of the keyed checks' (lazily computed) key tables: 16 or 20 (the widths the
// device builds, nw_api.cpp key_width).
static uint32_t g_key_w = 16;
int hc_set_key_width(int w) {
  if (w != 16 && w != 20 && w != 24) return -1;
  g_key_w = (uint32_t)w;
  return 0;
}

int hc_verify_strict_keyed(const uint8_t pk[32], const uint8_t sig[64], const uint8_t k32[32]) {
  init();
  uint32_t Aw[8], Rw[8], Sw[8], kw[8];
  load8(Aw, pk); load8(Rw, sig); load8(Sw, sig + 32); load8(kw, k32);
  ge A;
  const uint32_t flags = keyed_key(A, Aw);
  const strict_src_arrays src{Aw, Rw, Sw, kw};
  return strict_keyed_comb(src, SK, bcomb_lazy{BT, &SK.k.d2}, keytab_lazy{&A, &SK.k.d2, keyspec_for(g_key_w)}, flags);
}

// The certificate-vote keyed check without R decompression (nw_strict.hpp
// keyed_vote_check) followed by what k_votes_keyed_inv does for a pending vote (here one
// inversion per vote): 0 = the vote passes, 1 = it fails.
int hc_keyed_vote_check(const uint8_t pk[32], const uint8_t sig[64], const uint8_t k32[32]) {
  init();
  uint32_t Aw[8], Rw[8], Sw[8], kw[8];
  load8(Aw, pk); load8(Rw, sig); load8(Sw, sig + 32); load8(kw, k32);
  ge A;
  const uint32_t flags = keyed_key(A, Aw);
  const strict_src_arrays src{Aw, Rw, Sw, kw};
  fe X, Z;
  const uint32_t st = keyed_vote_check(src, SK, bcomb_lazy{BT, &SK.k.d2},
                                       keytab_lazy{&A, &SK.k.d2, keyspec_for(g_key_w)}, flags, X, Z);
  if (st < kVotePending) return (int)st;
  fe zi, x;
  fe_invert(zi, Z);
  fe_mul(x, X, zi);
  return fe_isnegative(x) == (st & 1) ? 0 : 1;
}

// Entry j of the wide B table half h (ypx || ymx || xy2d as 30 limbs), for the table test.
void hc_wide_btab_entry(int h, uint32_t j, uint32_t out[30]) {
  init();
  memcpy(out, &BTW[(h ? BTW_N : 0u) + j].n, 120);
}

}
