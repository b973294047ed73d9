// nw_host.cpp — the engine's host verification path (nw_host.h): the certificate service's
// hedge. Everything below the message layer is the kernels' own NW_HD arithmetic
// (nw_field.hpp radix-2^25.5 field, nw_point.hpp group law and dalek decompression,
// nw_scalar.hpp Barrett reduction, nw_strict.hpp strict ladder and small-order tests)
// compiled for the CPU; the oracle (oracle/) is never linked.
//
// Why a host path at all: the primary verifies one message at a time on its single Core task
// (/root/reference/primary/src/core.rs:338-346), so a device job that stalls (the box's
// host-memory access episodes) stalls the whole primary. The service
// (nw_service.cpp) answers a request here as well once its job is late, and the first
// verdict wins; verdicts are the device's (same checks, same order, same status / index).
//
// Work per signature on one core: a committee key's signature is a keyed comb check,
// [s]B - [k]A from 8-bit comb tables (32 + 32 mixed additions, no doublings; in five 51-bit
// limbs, nw_host_f51.hpp, since a 64x64-bit product is the CPU's native one), then one
// decompression of R (headers, votes) or, for certificate votes, the compressed-R compare
// of nw_strict.hpp keyed_vote_check with one inversion per certificate (Montgomery's trick);
// any other key takes the kernels'
// half-size strict ladder (nw_strict.hpp strict_verify_core<8>). A certificate whose votes
// do not all pass exactly is re-verified as dalek's verify_batch with fresh CSPRNG z (Straus).
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "nw_host.h"
#include "nw_host_f51.hpp"
#include "nw_consts.hpp"
#include "nw_sha512.hpp"

namespace nw {
namespace host {
namespace {

// ---------------------------------------------------------------------------------------
// SHA-512 (FIPS 180-4), host
// ---------------------------------------------------------------------------------------
constexpr uint64_t kShaK[80] = NW_SHA512_K_INIT;

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint64_t be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}

void sha_block(uint64_t h[8], const uint8_t* blk) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) w[t] = be64(blk + 8 * t);
  for (int t = 16; t < 80; ++t) {
    const uint64_t s0 = rotr(w[t - 15], 1) ^ rotr(w[t - 15], 8) ^ (w[t - 15] >> 7);
    const uint64_t s1 = rotr(w[t - 2], 19) ^ rotr(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], k = h[7];
  for (int t = 0; t < 80; ++t) {
    const uint64_t t1 = k + (rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41)) + ((e & f) ^ (~e & g)) +
                        kShaK[t] + w[t];
    const uint64_t t2 = (rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
    k = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += k;
}

// SHA-512 of the concatenation of up to three byte ranges.
void sha512(uint8_t out[64], const uint8_t* p0, size_t n0, const uint8_t* p1 = nullptr,
            size_t n1 = 0, const uint8_t* p2 = nullptr, size_t n2 = 0) {
  uint64_t h[8];
  for (int i = 0; i < 8; ++i) h[i] = SHA512_H0[i];
  uint8_t buf[128];
  size_t nb = 0;
  const uint8_t* ps[3] = {p0, p1, p2};
  const size_t ns[3] = {n0, n1, n2};
  for (int r = 0; r < 3; ++r) {
    const uint8_t* p = ps[r];
    size_t n = ns[r];
    while (n) {
      if (nb == 0 && n >= 128) {
        sha_block(h, p);
        p += 128;
        n -= 128;
        continue;
      }
      const size_t take = std::min(n, 128 - nb);
      memcpy(buf + nb, p, take);
      nb += take;
      p += take;
      n -= take;
      if (nb == 128) {
        sha_block(h, buf);
        nb = 0;
      }
    }
  }
  const uint64_t bits = 8 * (uint64_t)(n0 + n1 + n2);
  buf[nb++] = 0x80;
  if (nb > 112) {
    memset(buf + nb, 0, 128 - nb);
    sha_block(h, buf);
    nb = 0;
  }
  memset(buf + nb, 0, 120 - nb);
  for (int i = 0; i < 8; ++i) buf[120 + i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_block(h, buf);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(h[i] >> (56 - 8 * j));
}

// ---------------------------------------------------------------------------------------
// ChaCha20 keystream (DJB layout: 64-bit block counter, 64-bit nonce), the z_i of
// verify_batch: z_i = bytes [16 i, 16 i + 16) of the stream (nw_chacha.hpp's device layout)
// ---------------------------------------------------------------------------------------
inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
void chacha20_stream(const uint32_t key[8], uint8_t* out, size_t len) {
  for (uint64_t blk = 0; len; ++blk) {
    const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1],
                            key[2], key[3], key[4], key[5], key[6], key[7], (uint32_t)blk,
                            (uint32_t)(blk >> 32), 0u, 0u};
    uint32_t x[16];
    memcpy(x, s, sizeof x);
    for (int r = 0; r < 10; ++r) {
      auto qr = [&x](int a, int b, int c, int d) {
        x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 16);
        x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 12);
        x[a] += x[b]; x[d] = rotl32(x[d] ^ x[a], 8);
        x[c] += x[d]; x[b] = rotl32(x[b] ^ x[c], 7);
      };
      qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
      qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    uint8_t ks[64];
    for (int j = 0; j < 16; ++j) {
      const uint32_t v = x[j] + s[j];
      memcpy(ks + 4 * j, &v, 4);
    }
    const size_t take = std::min<size_t>(len, 64);
    memcpy(out, ks, take);
    out += take;
    len -= take;
  }
}

bool os_random(void* buf, size_t n) {
  size_t got = 0;
  while (got < n) {
    const ssize_t r = getrandom(static_cast<char*>(buf) + got, n - got, 0);
    if (r <= 0) return false;
    got += (size_t)r;
  }
  return true;
}

// ---------------------------------------------------------------------------------------
// Constants and 8-bit comb tables
// ---------------------------------------------------------------------------------------
constexpr int kComb = 32, kCombN = 129;   // tables j * 2^(8 t) P, t < 32, j = 0..128

// out[129 t + j] = j * 2^(8 t) P (affine niels), each table's 128 inversions batched into
// one (Montgomery's trick; Z never vanishes under the complete twisted Edwards formulas).
void comb8(ge_niels* out, const ge& P, const fe& d2) {
  ge base = P;
  ge pts[128];
  fe pre[128];
  for (int t = 0; t < kComb; ++t) {
    ge_cached cb;
    ge_to_cached(cb, base, d2);
    pts[0] = base;
    for (int j = 1; j < 128; ++j) ge_add_cached(pts[j], pts[j - 1], cb, true);
    fe_copy(pre[0], pts[0].Z);
    for (int j = 1; j < 128; ++j) fe_mul(pre[j], pre[j - 1], pts[j].Z);
    fe inv;
    fe_invert(inv, pre[127]);
    for (int j = 127; j >= 0; --j) {
      fe zi;
      if (j) {
        fe_mul(zi, inv, pre[j - 1]);
        fe_mul(inv, inv, pts[j].Z);
      } else {
        fe_copy(zi, inv);
      }
      ge_to_niels_zi(out[kCombN * t + j + 1], pts[j], zi, d2);
    }
    ge_niels_identity(out[kCombN * t]);
    for (int d = 0; d < 8; ++d) ge_dbl(base, base, d == 7);
  }
}

struct Consts {
  strict_consts SK;
  ge_niels BT[129], B128[129];
  torsion_consts tc;
  std::vector<f51::niels> BC;   // j * 2^(8 t) B
};

// the same field element in five 51-bit limbs (through its canonical bytes)
void to51(f51::fe& h, const fe& f) {
  uint32_t w[8];
  fe_tobytes(w, f);
  f51::frombytes(h, reinterpret_cast<const uint8_t*>(w));
}
void to51(f51::niels& h, const ge_niels& n) {
  to51(h.ypx, n.ypx);
  to51(h.ymx, n.ymx);
  to51(h.xy2d, n.xy2d);
}
// comb8 into 51-bit limbs
void comb8_51(std::vector<f51::niels>& out, const ge& P, const fe& d2) {
  std::vector<ge_niels> t((size_t)kComb * kCombN);
  comb8(t.data(), P, d2);
  out.resize(t.size());
  for (size_t i = 0; i < t.size(); ++i) to51(out[i], t[i]);
}
const Consts& consts() {
  static const Consts* c = [] {
    Consts* k = new Consts;
    compute_strict_consts(k->SK, k->B128);
    curve_consts kk;
    compute_consts(kk, k->BT);
    compute_torsion(k->tc);
    fe a, b, t;
    fe_from_u32(a, 4);
    fe_from_u32(b, 5);
    fe_invert(t, b);
    fe_mul(a, a, t);
    uint32_t yw[8];
    fe_tobytes(yw, a);
    ge B;
    ge_frombytes(B, yw, k->SK.k);
    comb8_51(k->BC, B, k->SK.k.d2);
    return k;
  }();
  return *c;
}

inline void load8(uint32_t w[8], const uint8_t* b) { memcpy(w, b, 32); }
inline void load_sc(sc& s, const uint8_t* b) { memcpy(s.w, b, 32); }

// k = SHA-512(R || A || M) mod l
void hram(sc& k, const uint8_t R[32], const uint8_t A[32], const uint8_t* m, size_t len) {
  uint8_t h[64];
  sha512(h, R, 32, A, 32, m, len);
  uint32_t x[16];
  memcpy(x, h, 64);
  sc_reduce512(k, x);
}

// signed 8-bit digit m of a recoded scalar (sc_recode with 0x80808080)
inline int digit8(const uint32_t d[8], int m) {
  return (int)((d[m >> 2] >> ((m & 3) * 8)) & 255u) - 128;
}

// acc = [s]B - [k]A from the 8-bit combs of A (ka) and B: 64 mixed additions, no doublings
void comb_sum(f51::pt& acc, const sc& k, const sc& s, const f51::niels* ka,
              const f51::niels* bc) {
  uint32_t kd[8], sd[8];
  sc_recode(kd, k, 0x80808080u);
  sc_recode(sd, s, 0x80808080u);
  f51::pt_identity(acc);
  for (int m = 0; m < kComb; ++m) {
    const int dk = digit8(kd, m), ds = digit8(sd, m);
    if (dk) {
      f51::niels n = ka[kCombN * m + (dk < 0 ? -dk : dk)];
      f51::niels_cneg(n, dk > 0);
      f51::add_niels(acc, acc, n);
    }
    if (ds) {
      f51::niels n = bc[kCombN * m + (ds < 0 ? -ds : ds)];
      f51::niels_cneg(n, ds < 0);
      f51::add_niels(acc, acc, n);
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Committee
// ---------------------------------------------------------------------------------------
struct KeyInfo {
  uint32_t flags = 0;          // kKeyDecoded | kKeySmall | lambda << kKeyLambdaShift
  std::vector<f51::niels> comb;  // 32 x 129 when decoded
};

struct Committee {
  size_t nauth = 0;
  std::vector<uint8_t> pks;
  std::vector<uint32_t> stakes;
  std::vector<uint64_t> wo;
  std::vector<uint32_t> wi;
  uint32_t quorum = 0;
  std::vector<KeyInfo> keys;
  // BTreeMap<PublicKey, Authority>::get: index or -1
  long find(const uint8_t pk[32]) const {
    long lo = 0, hi = (long)nauth - 1;
    while (lo <= hi) {
      const long mid = (lo + hi) / 2;
      const int c = memcmp(pks.data() + 32 * mid, pk, 32);
      if (c == 0) return mid;
      if (c < 0) lo = mid + 1;
      else hi = mid - 1;
    }
    return -1;
  }
  uint32_t stake(long a) const { return a < 0 ? 0u : stakes[a]; }
};

namespace {
// flags of a key as k_key_base computes them: decoded, small order, and lambda with
// [l]A == [lambda]T8 (the torsion image a strict pass does not cancel in a batch)
void key_info(KeyInfo& ki, const uint8_t pk[32]) {
  const Consts& C = consts();
  uint32_t w[8];
  load8(w, pk);
  ge A;
  if (!ge_frombytes(A, w, C.SK.k)) {
    ki.flags = 0;
    return;
  }
  ge_cached Pc;
  ge_to_cached(Pc, A, C.SK.k.d2);
  ge acc;
  ge_identity(acc);
  for (int bit = 252; bit >= 0; --bit) {
    ge_dbl(acc, acc, true);
    if ((L_W[bit >> 5] >> (bit & 31)) & 1u) ge_add_cached(acc, acc, Pc, true);
  }
  const int j = torsion_index(acc, C.tc);
  const uint32_t lam = j > 0 ? (uint32_t)j : 0u;
  ki.flags = kKeyDecoded | (ge_is_small_order(A) ? kKeySmall : 0u) | (lam << kKeyLambdaShift);
  comb8_51(ki.comb, A, C.SK.k.d2);
}
}  // namespace

Committee* committee_new(const nw_committee* c) {
  std::unique_ptr<Committee> h(new (std::nothrow) Committee);
  if (!h) return nullptr;
  const size_t na = c ? c->nauth : 0;
  h->nauth = na;
  h->pks.assign(c && na ? c->pks : nullptr, c && na ? c->pks + 32 * na : nullptr);
  h->stakes.assign(c && na ? c->stakes : nullptr, c && na ? c->stakes + na : nullptr);
  if (na) h->wo.assign(c->worker_offsets, c->worker_offsets + na + 1);
  else h->wo.assign(1, 0);
  const uint64_t nwk = h->wo[na];
  if (nwk) h->wi.assign(c->worker_ids, c->worker_ids + nwk);
  uint32_t total = 0;   // config::Stake is u32 (Committee::quorum_threshold, lib.rs:167-173)
  for (size_t a = 0; a < na; ++a) total += h->stakes[a];
  h->quorum = 2u * total / 3u + 1u;
  (void)consts();
  h->keys.resize(na);
  // the keys' tables, spread over a few threads (~2-5 ms of one core per key)
  const size_t nt = std::min<size_t>(na, std::max(1u, std::min(8u, std::thread::hardware_concurrency())));
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (size_t a = t; a < na; a += nt) key_info(h->keys[a], h->pks.data() + 32 * a);
    });
  for (auto& x : th) x.join();
  return h.release();
}

void committee_free(Committee* c) { delete c; }

// ---------------------------------------------------------------------------------------
// Signatures
// ---------------------------------------------------------------------------------------
int verify_strict(const uint8_t msg32[32], const uint8_t pk[32], const uint8_t sig[64]) {
  const Consts& C = consts();
  sc k;
  hram(k, sig, pk, msg32, 32);
  uint32_t Aw[8], Rw[8], Sw[8];
  load8(Aw, pk);
  load8(Rw, sig);
  load8(Sw, sig + 32);
  const strict_src_arrays src{Aw, Rw, Sw, k.w};
  ge_cached ta[8], tr[8];
  return strict_verify_core<8>(src, C.SK, btab_pair{C.BT, C.B128}, ta, tr, [](int w) { return w; });
}

namespace {
// Signature::verify with a committee key (the keyed comb; same checks and order as
// nw_strict.hpp strict_keyed_comb)
int verify_strict_keyed(const KeyInfo& key, const uint8_t msg32[32], const uint8_t pk[32],
                        const uint8_t sig[64]) {
  const Consts& C = consts();
  uint32_t Rw[8];
  load8(Rw, sig);
  ge R;
  const bool okR = ge_frombytes(R, Rw, C.SK.k);
  const bool smallR = okR && small_order_by_y(R.Y, C.SK.small_y);
  sc s;
  load_sc(s, sig + 32);
  if (sig[63] & 0xE0) return NW_ERR_S_HIGH_BITS;
  if (!(key.flags & kKeyDecoded)) return NW_ERR_A_DECODE;
  if (!sc_is_canonical(s)) return NW_ERR_S_NONCANONICAL;
  if (!okR) return NW_ERR_R_DECODE;
  if (smallR) return NW_ERR_R_SMALL_ORDER;
  if (key.flags & kKeySmall) return NW_ERR_A_SMALL_ORDER;
  sc k;
  hram(k, sig, pk, msg32, 32);
  f51::pt acc;
  comb_sum(acc, k, s, key.comb.data(), C.BC.data());
  // projective equality against the affine R: X == x_R Z, Y == y_R Z
  f51::fe xr, yr, t;
  to51(xr, R.X);
  to51(yr, R.Y);
  f51::mul(t, xr, acc.Z);
  if (!f51::eq(t, acc.X)) return NW_ERR_EQUATION;
  f51::mul(t, yr, acc.Z);
  return f51::eq(t, acc.Y) ? NW_OK : NW_ERR_EQUATION;
}

// A vote whose R == [s]B - [k]A exactly (and which dalek's verify_strict accepts) adds
// nothing to ANY random linear combination: the compressed-R check of nw_strict.hpp
// keyed_vote_check. Returns 0 = fails (decide by the full verify_batch), 1 = passes, or
// 2 | sign = passes iff the parity of X'/Z' equals sign: the caller batches those
// inversions (Montgomery's trick, as k_votes_keyed_inv does on the device).
uint32_t vote_check(const KeyInfo& key, const uint8_t digest[32], const uint8_t pk[32],
                    const uint8_t sig[64], f51::fe& X, f51::fe& Z) {
  const Consts& C = consts();
  if ((sig[63] & 0xE0) || !(key.flags & kKeyDecoded) || (key.flags & kKeySmall) ||
      (key.flags & kKeyLambdaMask))
    return 0;
  sc s;
  load_sc(s, sig + 32);
  if (!sc_is_canonical(s)) return 0;
  uint32_t Rw[8];
  load8(Rw, sig);
  const uint32_t sign = Rw[7] >> 31;
  fe yR;
  fe_frombytes(yR, Rw);
  if (small_order_by_y(yR, C.SK.small_y)) return 0;
  sc k;
  hram(k, sig, pk, digest, 32);
  f51::pt acc;
  comb_sum(acc, k, s, key.comb.data(), C.BC.data());
  // y' == y_R: the encoding's y as given (bit 255 cleared, reduced mod p as dalek's
  // decompression reads it)
  f51::fe y51, t;
  to51(y51, yR);
  f51::mul(t, y51, acc.Z);
  if (!f51::eq(t, acc.Y)) return 0;
  if (f51::iszero(acc.X)) return 1;
  X = acc.X;
  Z = acc.Z;
  return 2 | sign;
}

// Every vote passes (each R == [s]B - [k]A with dalek's strict checks), the parities with
// one inversion for all of them.
bool votes_pass(const Committee& com, const uint8_t digest[32], const uint8_t* pks,
                const uint8_t* sigs, size_t n) {
  std::vector<f51::fe> X(n), Z(n), pre(n);
  std::vector<uint32_t> sign(n);
  size_t m = 0;   // pending parities
  for (size_t i = 0; i < n; ++i) {
    const long a = com.find(pks + 32 * i);
    if (a < 0) return false;
    const uint32_t r = vote_check(com.keys[a], digest, pks + 32 * i, sigs + 64 * i, X[m], Z[m]);
    if (r == 0) return false;
    if (r & 2) sign[m++] = r & 1;
  }
  if (m == 0) return true;
  pre[0] = Z[0];
  for (size_t i = 1; i < m; ++i) f51::mul(pre[i], pre[i - 1], Z[i]);
  f51::fe inv;
  f51::invert(inv, pre[m - 1]);
  for (size_t i = m; i-- > 0;) {
    f51::fe zi, x;
    if (i) {
      f51::mul(zi, inv, pre[i - 1]);
      f51::mul(inv, inv, Z[i]);
    } else {
      zi = inv;
    }
    f51::mul(x, X[i], zi);
    if (f51::isnegative(x) != sign[i]) return false;
  }
  return true;
}

// dalek verify_batch, every step: per vote s high bits / A decode (first failure), s < l over
// all, R decode over all, then sum z_i R_i + (z_i k_i mod l) A_i - (sum z_i s_i mod l) B ==
// identity, by a Straus ladder (4-bit signed windows over 9-entry tables, 8-bit B digits).
int verify_batch_full(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs,
                      size_t n, const uint8_t* z16, uint64_t* fail_index) {
  const Consts& C = consts();
  *fail_index = n;
  if (n == 0) return NW_OK;
  std::vector<ge> P(2 * n);   // R_0..R_{n-1}, A_0..A_{n-1}
  for (size_t i = 0; i < n; ++i) {
    uint32_t w[8];
    if (sigs[64 * i + 63] & 0xE0) { *fail_index = i; return NW_ERR_S_HIGH_BITS; }
    load8(w, pks + 32 * i);
    if (!ge_frombytes(P[n + i], w, C.SK.k)) { *fail_index = i; return NW_ERR_A_DECODE; }
  }
  for (size_t i = 0; i < n; ++i) {
    sc s;
    load_sc(s, sigs + 64 * i + 32);
    if (!sc_is_canonical(s)) { *fail_index = i; return NW_ERR_S_NONCANONICAL; }
  }
  for (size_t i = 0; i < n; ++i) {
    uint32_t w[8];
    load8(w, sigs + 64 * i);
    if (!ge_frombytes(P[i], w, C.SK.k)) { *fail_index = i; return NW_ERR_R_DECODE; }
  }
  std::vector<uint8_t> zb;
  if (!z16) {
    uint32_t key[8];
    if (!os_random(key, sizeof key)) return NW_E_DEVICE;   // no CSPRNG: no verdict
    zb.resize(16 * n);
    chacha20_stream(key, zb.data(), zb.size());
    z16 = zb.data();
  }
  std::vector<uint32_t> dig(8 * 2 * n);   // 4-bit signed digits of z_i and c_i
  sc bsum;
  memset(bsum.w, 0, 32);
  for (size_t i = 0; i < n; ++i) {
    sc z, k, s, t;
    memset(z.w, 0, 32);
    memcpy(z.w, z16 + 16 * i, 16);
    hram(k, sigs + 64 * i, pks + 32 * i, digest, 32);
    load_sc(s, sigs + 64 * i + 32);
    sc_mul(t, z, k);
    sc_recode(&dig[8 * i], z, 0x88888888u);
    sc_recode(&dig[8 * (n + i)], t, 0x88888888u);
    sc_mul(t, z, s);
    sc_add(bsum, bsum, t);
  }
  sc nb;
  sc_neg(nb, bsum);
  uint32_t bd[8];
  sc_recode(bd, nb, 0x80808080u);
  std::vector<ge_cached> tab(9 * 2 * n);
  for (size_t j = 0; j < 2 * n; ++j) build_table9(&tab[9 * j], P[j], C.SK.k.d2);
  ge acc;
  ge_identity(acc);
  for (int i = 63; i >= 0; --i) {
    if (i != 63)
      for (int t = 0; t < 4; ++t) ge_dbl(acc, acc, true);
    for (size_t j = 0; j < 2 * n; ++j) {
      const int d = (int)((dig[8 * j + (i >> 3)] >> ((i & 7) * 4)) & 15u) - 8;
      if (d) add_digit_cached(acc, &tab[9 * j], d, true);
    }
    if ((i & 1) == 0) {
      const int d = (int)((bd[i >> 3] >> (((i >> 1) & 3) * 8)) & 255u) - 128;
      if (d) add_digit_niels(acc, C.BT, d, true);
    }
  }
  return ge_is_identity(acc) ? NW_OK : NW_ERR_EQUATION;
}
}  // namespace

int verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                 const uint8_t* z16, const Committee* com, uint64_t* fail_index) {
  uint64_t fi = n;
  int st = NW_OK;
  const bool all = n > 0 && com != nullptr && votes_pass(*com, digest, pks, sigs, n);
  if (!all) st = verify_batch_full(digest, pks, sigs, n, z16, &fi);
  else fi = n;
  if (fail_index) *fail_index = fi;
  return st;
}

// ---------------------------------------------------------------------------------------
// Messages (primary/src/messages.rs)
// ---------------------------------------------------------------------------------------
namespace {
inline uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline uint64_t le64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}
}  // namespace

int header_verify(const Committee& c, const uint8_t* hb, size_t hlen, uint32_t np,
                  const uint8_t id[32], const uint8_t sig[64], uint64_t* index) {
  *index = 0;
  uint8_t h[64];
  sha512(h, hb, hlen);   // Hash for Header: the bytes as given (messages.rs:70-84)
  if (memcmp(h, id, 32) != 0) return NW_DAG_INVALID_HEADER_ID;
  const long a = c.find(hb);
  if (c.stake(a) == 0) {
    *index = UINT64_MAX;
    return NW_DAG_UNKNOWN_AUTHORITY;
  }
  for (uint32_t e = 0; e < np; ++e) {   // Committee::worker(author, id) for every payload entry
    const uint32_t wid = le32(hb + 40 + 36 * (size_t)e + 32);
    bool found = false;
    for (uint64_t w = c.wo[a]; w < c.wo[a + 1] && !found; ++w) found = c.wi[w] == wid;
    if (!found) {
      *index = e;
      return NW_DAG_MALFORMED_HEADER;
    }
  }
  const int st = verify_strict_keyed(c.keys[a], id, hb, sig);
  return st ? NW_DAG_INVALID_SIGNATURE + st : NW_OK;
}

int vote_verify(const Committee& c, const uint8_t id[32], uint64_t round,
                const uint8_t origin[32], const uint8_t author[32], const uint8_t sig[64]) {
  const long a = c.find(author);
  if (c.stake(a) == 0) return NW_DAG_UNKNOWN_AUTHORITY;
  uint8_t rb[8], h[64];
  for (int i = 0; i < 8; ++i) rb[i] = (uint8_t)(round >> (8 * i));
  sha512(h, id, 32, rb, 8, origin, 32);   // Hash for Vote (messages.rs:145-153)
  const int st = verify_strict_keyed(c.keys[a], h, author, sig);
  return st ? NW_DAG_INVALID_SIGNATURE + st : NW_OK;
}

int certificate_verify(const Committee& c, const uint8_t* hb, size_t hlen, uint32_t np,
                       const uint8_t id[32], const uint8_t hsig[64], const uint8_t* vote_pks,
                       const uint8_t* vote_sigs, size_t nvotes, const uint8_t* z16,
                       uint64_t* index) {
  *index = 0;
  const uint64_t round = le64(hb + 32);
  // Genesis certificates are always valid (messages.rs:191-193): (id, round, origin) ==
  // (0, 0, an authority), Certificate's equality
  bool idzero = true;
  for (int i = 0; i < 32; ++i) idzero &= id[i] == 0;
  if (idzero && round == 0 && c.find(hb) >= 0) return NW_OK;
  int st = header_verify(c, hb, hlen, np, id, hsig, index);
  if (st) return st;
  // quorum (messages.rs:198-210): reuse, then voting rights, in vote order
  std::vector<uint8_t> used(c.nauth, 0);
  uint32_t weight = 0;
  for (size_t v = 0; v < nvotes; ++v) {
    const long a = c.find(vote_pks + 32 * v);
    if (a >= 0 && used[a]) {
      *index = v;
      return NW_DAG_AUTHORITY_REUSE;
    }
    if (c.stake(a) == 0) {
      *index = v;
      return NW_DAG_UNKNOWN_AUTHORITY;
    }
    used[a] = 1;
    weight += c.stakes[a];
  }
  if (weight < c.quorum) return NW_DAG_REQUIRES_QUORUM;
  uint8_t rb[8], h[64];
  for (int i = 0; i < 8; ++i) rb[i] = (uint8_t)(round >> (8 * i));
  sha512(h, id, 32, rb, 8, hb, 32);   // Hash for Certificate (messages.rs:226-234)
  uint64_t fi = 0;
  st = verify_batch(h, vote_pks, vote_sigs, nvotes, z16, &c, &fi);
  if (st < 0) return st;
  if (st) {
    *index = fi;
    return NW_DAG_INVALID_VOTES + st;
  }
  return NW_OK;
}

}  // namespace host
}  // namespace nw

// ---------------------------------------------------------------------------------------
// C ABI (include/narwhal_amd.h "host verification path")
// ---------------------------------------------------------------------------------------
extern "C" {

int nw_host_verify_strict_many(const uint8_t* msgs, size_t msg_stride, const uint8_t* pks,
                               const uint8_t* sigs, size_t n, int32_t* status_out) {
  if (n && (!msgs || !pks || !sigs || !status_out)) return NW_E_INVALID_ARG;
  for (size_t i = 0; i < n; ++i)
    status_out[i] = nw::host::verify_strict(msgs + msg_stride * i, pks + 32 * i, sigs + 64 * i);
  return 0;
}

int nw_host_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                              const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                              int32_t* status_out, uint64_t* fail_index_out) {
  if (nbatches && (!digests || !offsets || !status_out)) return NW_E_INVALID_ARG;
  for (size_t b = 0; b < nbatches; ++b) {
    const uint64_t o = offsets[b], cnt = offsets[b + 1] - o;
    uint64_t fi = 0;
    const int st = nw::host::verify_batch(digests + 32 * b, pks + 32 * o, sigs + 64 * o, cnt,
                                          z16 ? z16 + 16 * o : nullptr, nullptr, &fi);
    if (st < 0) return st;
    status_out[b] = st;
    if (fail_index_out) fail_index_out[b] = fi;
  }
  return 0;
}

int nw_host_certificates_verify_many(const nw_committee* committee, const nw_certificates* cs,
                                     const uint8_t* z16, int headers_only, int32_t* status_out,
                                     uint64_t* index_out) {
  if (!committee || !cs || (cs->n && !status_out)) return NW_E_INVALID_ARG;
  std::unique_ptr<nw::host::Committee, void (*)(nw::host::Committee*)> c(
      nw::host::committee_new(committee), nw::host::committee_free);
  if (!c) return NW_E_OUT_OF_MEMORY;
  for (size_t i = 0; i < cs->n; ++i) {
    const uint8_t* hb = cs->header_bytes + cs->header_offsets[i];
    const size_t hl = cs->header_offsets[i + 1] - cs->header_offsets[i];
    uint64_t ix = 0;
    int st;
    if (headers_only) {
      st = nw::host::header_verify(*c, hb, hl, cs->payload_counts[i], cs->ids + 32 * i,
                                   cs->header_sigs + 64 * i, &ix);
    } else {
      const uint64_t vb = cs->vote_offsets[i], nv = cs->vote_offsets[i + 1] - vb;
      st = nw::host::certificate_verify(*c, hb, hl, cs->payload_counts[i], cs->ids + 32 * i,
                                        cs->header_sigs + 64 * i, cs->vote_pks + 32 * vb,
                                        cs->vote_sigs + 64 * vb, nv, z16 ? z16 + 16 * vb : nullptr,
                                        &ix);
    }
    if (st < 0) return st;
    status_out[i] = st;
    if (index_out) index_out[i] = ix;
  }
  return 0;
}

int nw_host_votes_verify_many(const nw_committee* committee, const uint8_t* ids,
                              const uint64_t* rounds, const uint8_t* origins,
                              const uint8_t* authors, const uint8_t* sigs, size_t n,
                              int32_t* status_out) {
  if (!committee || (n && (!ids || !rounds || !origins || !authors || !sigs || !status_out)))
    return NW_E_INVALID_ARG;
  std::unique_ptr<nw::host::Committee, void (*)(nw::host::Committee*)> c(
      nw::host::committee_new(committee), nw::host::committee_free);
  if (!c) return NW_E_OUT_OF_MEMORY;
  for (size_t i = 0; i < n; ++i)
    status_out[i] = nw::host::vote_verify(*c, ids + 32 * i, rounds[i], origins + 32 * i,
                                          authors + 32 * i, sigs + 64 * i);
  return 0;
}

}  // extern "C"
