// nw_kernels.hip — gfx950 kernels for Narwhal's crypto hot path.
//
//   k_sha512_digest32     Digest(Sha512(m)[..32]) for many messages, one lane per message
//                         (worker/src/processor.rs:38, primary/src/messages.rs:70-84 ...).
//   k_verify_strict       crypto::Signature::verify (crypto/src/lib.rs:200-204), one lane per
//                         signature: decompress A and R, small-order tests, k = H(R||A||M)
//                         mod l, half-size scalars, [v]R + [u]A + [w]B == 0 by one joint
//                         signed-window ladder (A and R tables in per-lane scratch, w in
//                         24-bit windows over device-built global tables), identity test.
//   k_btab_build          the strict kernel's B tables, once per device.
//   (crypto::Signature::verify_batch lives in nw_batch.hip.)
//
// Everything here is integer VALU work; no MFMA (modular arithmetic is not a contraction).
#include "nw_kernels.h"
#include "nw_point.hpp"
#include "nw_scalar.hpp"
#include "nw_sha512.hpp"
#include "nw_ladder.hpp"
#include "nw_consts.hpp"

#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>

namespace nw {

struct dev_consts {
  curve_consts k;
  ge_niels btab[129];   // j * B, j = 0..128, affine niels (signed 8-bit windows)
  strict_consts sk;     // nw_strict.hpp: small-order y values
  ge_niels b128[129];   // j * 2^128 B
};

__constant__ dev_consts g_consts;

static constexpr int BT_WORDS = 129 * 30;

// ---------------------------------------------------------------------------------------
// Small helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Copy a 129-entry niels table from constant memory into LDS (all threads of the block).
__device__ __forceinline__ void load_table(ge_niels* dst_tab, const ge_niels* src_tab) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(src_tab);
  uint32_t* dst = reinterpret_cast<uint32_t*>(dst_tab);
  for (int i = threadIdx.x; i < BT_WORDS; i += blockDim.x) dst[i] = src[i];
}
__device__ __forceinline__ void load_btab(ge_niels* s_btab) { load_table(s_btab, g_consts.btab); }

// Maximum of a per-lane value 0 <= w < 128 over the ACTIVE lanes of the wave (wave-uniform
// result), bit by bit with ballots, so it is exact inside divergent code too (a lane shuffle
// would read inactive lanes' stale registers).
struct WaveMax {
  __device__ int operator()(int w) const {
    int r = 0;
#pragma unroll
    for (int b = 6; b >= 0; --b) {
      const int c = r | (1 << b);
      if (__ballot(w >= c) != 0) r = c;
    }
    return r;
  }
};

// SHA-512 of the 96-byte R || A || M (one block) -> 16 LE words of the digest.
__device__ __forceinline__ void hram96(uint32_t x[16], const uint32_t R[8], const uint32_t A[8],
                                       const uint32_t M[8]) {
  uint64_t w[16], st[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = ((uint64_t)bswap32(R[2 * i]) << 32) | bswap32(R[2 * i + 1]);
    w[4 + i] = ((uint64_t)bswap32(A[2 * i]) << 32) | bswap32(A[2 * i + 1]);
    w[8 + i] = ((uint64_t)bswap32(M[2 * i]) << 32) | bswap32(M[2 * i + 1]);
  }
  w[12] = 0x8000000000000000ULL;
  w[13] = 0;
  w[14] = 0;
  w[15] = 96 * 8;
  sha512_init(st);
  sha512_compress(st, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x[2 * i] = bswap32((uint32_t)(st[i] >> 32));
    x[2 * i + 1] = bswap32((uint32_t)st[i]);
  }
}

// ---------------------------------------------------------------------------------------
// SHA-512 digests of many messages (lane per message)
// ---------------------------------------------------------------------------------------
// One lane per message (sha512_digest32_lane, nw_sha512.hpp: full blocks double-buffered,
// so a lone wave per SIMD -- config 3: 65,536 messages = 1,024 waves -- does not stall on
// each block's HBM latency).
__global__ __launch_bounds__(256) void k_sha512_digest32(const uint8_t* __restrict__ data,
                                                         const uint64_t* __restrict__ offsets,
                                                         const uint64_t* __restrict__ lengths,
                                                         uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* msg = data + offsets[i];
  const uint64_t len = lengths ? lengths[i] : offsets[i + 1] - offsets[i];
  sha512_digest32_lane(msg, len, out + 8 * i);
}

// ---------------------------------------------------------------------------------------
// Strict verification
// ---------------------------------------------------------------------------------------

// Makes p opaque to the optimiser: a load through the result is not merged with an earlier
// load of the same address, so inputs are re-fetched where they are needed instead of
// being kept live (and spilled) across the decompression.
template <class T>
__device__ __forceinline__ const T* opaque_ptr(const T* p) {
  asm volatile("" : "+v"(p));
  return p;
}

// strict_verify_core's inputs for item i, fetched from global memory when needed.
struct strict_src_global {
  static constexpr bool kPre = false;
  const uint32_t* pk;    // 8 words
  const uint32_t* sig;   // 16 words: R || s
  const uint32_t* msg;   // 8 words
  __device__ void A(uint32_t w[8]) const {
    const uint32_t* p = opaque_ptr(pk);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = p[j];
  }
  __device__ void R(uint32_t w[8]) const {
    const uint32_t* p = opaque_ptr(sig);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = p[j];
  }
  __device__ void S(uint32_t w[8]) const {
    const uint32_t* p = opaque_ptr(sig);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = p[8 + j];
  }
  // k = SHA-512(R || A || M) mod l over the raw bytes
  __device__ void K(uint32_t kw[8]) const {
    uint32_t Aw[8], Rw[8], Mw[8], hx[16];
    A(Aw);
    R(Rw);
    const uint32_t* m = opaque_ptr(msg);
#pragma unroll
    for (int j = 0; j < 8; ++j) Mw[j] = m[j];
    hram96(hx, Rw, Aw, Mw);
    sc k;
    sc_reduce512(k, hx);
#pragma unroll
    for (int j = 0; j < 8; ++j) kw[j] = k.w[j];
  }
};

// The same inputs with A's and R's x already decompressed (k_strict_triage): x limb k of
// point pt (0 = A, 1 = R) of survivor q at xs[(10 pt + k) cap + q]. y is the encoding's own
// (fe_frombytes), Z = 1, T = x y: exactly the point ge_frombytes returned.
struct strict_src_pre : strict_src_global {
  static constexpr bool kPre = true;
  const uint32_t* xs;
  uint64_t cap, q;
  __device__ bool point(int pt, ge& P) const {
    uint32_t w[8];
    if (pt) R(w); else A(w);
    fe_frombytes(P.Y, w);
    const uint32_t* x = opaque_ptr(xs) + (uint64_t)(10 * pt) * cap + q;
#pragma unroll
    for (int k = 0; k < 10; ++k) P.X.v[k] = x[(uint64_t)k * cap];
    fe_1(P.Z);
    fe_mul(P.T, P.X, P.Y);
    return true;
  }
};

// Limb planes of the pending votes of a slice: X' limb k at planes[k S + i], Z' limb k at
// planes[(10 + k) S + i] (coalesced in both kernels); state[i] = kVote* of vote v0 + i.
struct vote_planes_t {
  uint32_t* planes;
  uint32_t* state;
  uint64_t S;
  const uint32_t* perm;   // slice position -> slice vote (key-major order), or nullptr
};

#ifndef NW_KEYED_WAVES
#define NW_KEYED_WAVES 1
#endif
// The strict ladder's LDS prefetcher (nw_strict.hpp pf_none for the contract): one
// 128-byte slot per lane (8 chunks of 16 B, chunk k of lane l at s_pf[k][l]: the lanes of a
// wave write and read 16 consecutive bytes each, conflict-free), 32 KB per 256-thread block.
// Every entry is one 128-byte line: a B-table entry (affine niels, ge_niels_pad) or a
// per-lane entry packed to 128 B (ge_cached_pk; unpacked here).
#ifndef NW_STRICT_PF
#define NW_STRICT_PF 1
#endif
// (The keyed comb checks through the same slots measured slower)
#if NW_STRICT_PF && NW_BWIN != 8
// The ladder's digit words (u, |v|, w recoded: 21 per lane) live in LDS too, 21 KB per block:
// read with a wave-uniform index once per addition, they were otherwise a scratch array (a
// dependent scratch load per addition; scratch 272 -> 180 B per lane, +0.2 % in the same
// process, profiles/r05w). 53 KB per block: three blocks per CU fit the 160 KB.
__shared__ uint4 s_pf[8][256];
__shared__ uint32_t s_dig[21][256];
struct pf_lds {
  static constexpr bool enabled = true;
  static constexpr bool lds_digits = true;
  uint32_t wave;   // wave index in the block (uniform)
  __device__ void dput(int k, uint32_t v) const { s_dig[k][threadIdx.x] = v; }
  __device__ uint32_t dget(int k) const { return s_dig[k][threadIdx.x]; }
  __device__ void issue(const void* src, int chunks) const {
    const uint4* g = static_cast<const uint4*>(src);
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this lane's last slot read is done
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < chunks) __builtin_amdgcn_global_load_lds(g + k, &s_pf[k][wave * 64], 16, 0, 0);
  }
  __device__ void get(ge_cached& e, bool niels) const {
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the DMA into LDS has landed
    asm volatile("" ::: "memory");
    const uint32_t l = threadIdx.x;
    uint32_t p[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 v = s_pf[k][l];
      p[4 * k] = v.x; p[4 * k + 1] = v.y; p[4 * k + 2] = v.z; p[4 * k + 3] = v.w;
    }
    if (niels) {   // y+x, y-x, xy2d (-> YpX, YmX, T2d; Z2 unused)
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        e.YpX.v[i] = p[i];
        e.YmX.v[i] = p[10 + i];
        e.T2d.v[i] = p[20 + i];
      }
      return;
    }
    fe_unpack(e.YpX, p);
    fe_unpack(e.YmX, p + 8);
    fe_unpack(e.Z2, p + 16);
    fe_unpack(e.T2d, p + 24);
  }
  // A packed per-lane entry read as -entry when neg (NW_PF_SWAP): Y+X and Y-X trade places
  // through the LDS address (chunks 0-1 <-> 2-3), so the caller negates only 2dT.
  __device__ void get_signed(ge_cached& e, bool neg) const {
    __builtin_amdgcn_s_waitcnt(0x0F70);
    asm volatile("" ::: "memory");
    const uint32_t l = threadIdx.x;
    const uint32_t a = neg ? 2u : 0u;
    uint32_t p[32];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 v = s_pf[k < 4 ? (k ^ a) : k][l];
      p[4 * k] = v.x; p[4 * k + 1] = v.y; p[4 * k + 2] = v.z; p[4 * k + 3] = v.w;
    }
    fe_unpack(e.YpX, p);
    fe_unpack(e.YmX, p + 8);
    fe_unpack(e.Z2, p + 16);
    fe_unpack(e.T2d, p + 24);
  }
};
#endif

// Persistent: the grid covers the resident waves once and strides over the items, so the
// per-lane tables j*A, j*R live in a fixed workspace (16 packed entries x 128 B per lane slot,
// lane-contiguous: a lookup reads one 128-byte line per lane instead of 40 scattered dwords).
#ifndef NW_STRICT_WAVES
#define NW_STRICT_WAVES 3
#endif
// KEYED = false: arbitrary keys only, every item through the half-size ladder (config 4,
// nw_verify_strict_many): the instance carries neither the keyed comb branch nor the list
// mode, so their registers and code do not weigh on the ladder. KEYED = true: committee
// keys take the keyed comb, and `list` (the keyed fast path's leftovers) is honoured.
template <bool KEYED>
__global__ __launch_bounds__(256, NW_STRICT_WAVES) void k_verify_strict(const uint32_t* __restrict__ msgs,
                                                       uint32_t msg_stride_words,
                                                       const uint32_t* __restrict__ pks,
                                                       const uint32_t* __restrict__ sigs,
                                                       uint64_t n, int32_t* __restrict__ status,
                                                       uint64_t* __restrict__ bitmap,
                                                       ge_cached_pk* __restrict__ tabs,
                                                       key_tables_t keys,
                                                       const ge_niels_pad* __restrict__ btw,
                                                       const ge_niels_pad* __restrict__ bcomb,
                                                       const uint32_t* __restrict__ list,
                                                       const uint32_t* __restrict__ list_count) {
  // list mode (keyed fast path's leftovers): items list[0 .. *list_count), no bitmap words
  if (!KEYED) list = nullptr;
  if (list) n = *list_count;
#if NW_BWIN == 8
  __shared__ ge_niels s_btab[129];
  __shared__ ge_niels s_b128[129];
  load_table(s_btab, g_consts.btab);
  load_table(s_b128, g_consts.b128);
  __syncthreads();
  const btab_pair bt{s_btab, s_b128};
  (void)btw;
#else
  const btab_wide bt{btw, bdigits<NW_BWIN>::ENTRIES};
#endif
  ge_cached_pk* tabA = tabs + 16 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  ge_cached_pk* tabR = tabA + 8;
#pragma unroll 1
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n;
       base += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t gi = base + threadIdx.x;
    const bool active = gi < n;
    const uint64_t i = list ? list[active ? gi : n - 1] : active ? gi : n - 1;
    const strict_src_global src{pks + 8 * i, sigs + 16 * i, msgs + (uint64_t)msg_stride_words * i};
    const uint32_t kk = KEYED && keys.vote_key ? keys.vote_key[i] : kNoKey;
    const ge_niels_pad* keytab = kk != kNoKey ? keys.tabs + keys.ks.tab * (uint64_t)kk : nullptr;
    // committee keys: [s]B - [k]A from comb tables, no ladder; others: the half-size ladder
    int st;
    if (KEYED && keytab) {
      st = strict_keyed_comb(src, g_consts.sk, bcomb_wide{bcomb}, keytab_wide{keytab, keys.ks},
                             keys.ok[kk]);
    } else {
#if NW_STRICT_PF && NW_BWIN != 8
      st = strict_verify_core<NW_BWIN>(src, g_consts.sk, bt, tabA, tabR, WaveMax{},
                                       pf_lds{(uint32_t)__builtin_amdgcn_readfirstlane(
                                           threadIdx.x >> 6)});
#else
      st = strict_verify_core<NW_BWIN>(src, g_consts.sk, bt, tabA, tabR, WaveMax{});
#endif
    }
    if (active) status[i] = st;
    if (list) continue;
    const uint64_t mask = __ballot(active && st == NW_OK);
    if ((threadIdx.x & 63) == 0 && gi < n) bitmap[gi >> 6] = mask;
  }
}

// ---- config 4's strict verification in two passes (NW_STRICT_TRIAGE, default on) ----
// Every check before the equation (s's high bits and canonical form, A's and R's
// decompression and small order) needs only the two square roots, ~15 % of a verification;
// an item that fails one of them (7 of the 12 invalid classes of the mixed corpus, ~6.5 % of
// its items) still ran the whole ladder in k_verify_strict, whose lanes all take the same
// path. k_strict_triage runs the checks for a slice of items, one lane per item, writes the
// verdict of every item that fails one (same order as strict_verify_core: crypto/src/lib.rs
// 201-202, then dalek's verify_strict), and appends the others to a list with the x of A and
// R; k_verify_strict_pre runs strict_verify_core on the list, loading those points instead
// of decompressing them (strict_src_pre). Statuses are the same codes for every item.
#ifndef NW_TRIAGE_WAVES
#define NW_TRIAGE_WAVES 4   // waves per SIMD (129 VGPRs unbounded: 3)
#endif
__global__ __launch_bounds__(256, NW_TRIAGE_WAVES) void k_strict_triage(
    const uint32_t* __restrict__ msgs, uint32_t msg_stride_words, const uint32_t* __restrict__ pks,
    const uint32_t* __restrict__ sigs, uint64_t i0, uint64_t ns, int32_t* __restrict__ status,
    uint32_t* __restrict__ xs, uint64_t cap, uint32_t* __restrict__ list,
    uint32_t* __restrict__ count) {
  (void)msgs;
  (void)msg_stride_words;
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = j < ns;
  const uint64_t i = i0 + (active ? j : 0);
  const strict_src_global src{pks + 8 * i, sigs + 16 * i, nullptr};
  fe xa, xr;
  const int st = strict_triage(src, g_consts.sk, xa, xr);
  if (active && st != NW_OK) status[i] = st;
  const bool keep = active && st == NW_OK;
  const uint64_t m = __ballot(keep);
  if (m == 0) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t rank = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
  const uint32_t leader = (uint32_t)__builtin_ctzll(m);
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(count, (uint32_t)__builtin_popcountll(m));
  base = (uint32_t)__shfl((int)base, (int)leader);
  if (!keep) return;
  const uint64_t pos = (uint64_t)base + rank;
  list[pos] = (uint32_t)j;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    xs[(uint64_t)k * cap + pos] = xa.v[k];
    xs[(uint64_t)(10 + k) * cap + pos] = xr.v[k];
  }
}

// The list's items (persistent, as k_verify_strict): strict_verify_core on the points
// k_strict_triage decompressed; *count is read on the device.
__global__ __launch_bounds__(256, NW_STRICT_WAVES) void k_verify_strict_pre(
    const uint32_t* __restrict__ msgs, uint32_t msg_stride_words, const uint32_t* __restrict__ pks,
    const uint32_t* __restrict__ sigs, uint64_t i0, const uint32_t* __restrict__ list,
    const uint32_t* __restrict__ count, const uint32_t* __restrict__ xs, uint64_t cap,
    int32_t* __restrict__ status, ge_cached_pk* __restrict__ tabs,
    const ge_niels_pad* __restrict__ btw) {
  const uint64_t n = *count;
#if NW_BWIN == 8
  __shared__ ge_niels s_btab[129];
  __shared__ ge_niels s_b128[129];
  load_table(s_btab, g_consts.btab);
  load_table(s_b128, g_consts.b128);
  __syncthreads();
  const btab_pair bt{s_btab, s_b128};
  (void)btw;
#else
  const btab_wide bt{btw, bdigits<NW_BWIN>::ENTRIES};
#endif
  ge_cached_pk* tabA = tabs + 16 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  ge_cached_pk* tabR = tabA + 8;
#pragma unroll 1
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n;
       base += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q0 = base + threadIdx.x;
    const bool active = q0 < n;
    const uint64_t q = active ? q0 : n - 1;
    const uint64_t i = i0 + list[q];
    const strict_src_pre src{{pks + 8 * i, sigs + 16 * i, msgs + (uint64_t)msg_stride_words * i},
                             xs, cap, q};
#if NW_STRICT_PF && NW_BWIN != 8
    const int st = strict_verify_core<NW_BWIN>(src, g_consts.sk, bt, tabA, tabR, WaveMax{},
                                               pf_lds{(uint32_t)__builtin_amdgcn_readfirstlane(
                                                   threadIdx.x >> 6)});
#else
    const int st = strict_verify_core<NW_BWIN>(src, g_consts.sk, bt, tabA, tabR, WaveMax{});
#endif
    if (active) status[i] = st;
  }
}

// Keyed fast path of launch_verify_strict (committee-key signers: Header::verify authors,
// Vote::verify voters). k_strict_keyed runs the certificate votes' check (nw_strict.hpp
// keyed_vote_check: [s]B - [k]A from the comb tables, compared with R in compressed form,
// no square root) on every keyed item of a slice; a pass IS dalek's verify_strict Ok
// (status 0), everything else — fails, non-committee signers, parity mismatches found by
// k_strict_keyed_inv — is appended to a list (k_strict_keyed_list) and verified by
// k_verify_strict in list mode, which names the exact failing check (status 1..7). With
// honest streams the list is short, so the ~265-squaring decompression of R is skipped
// for almost every signature.
__global__ __launch_bounds__(256, NW_KEYED_WAVES) void k_strict_keyed(
    const uint32_t* __restrict__ msgs, uint32_t msg_stride_words, const uint32_t* __restrict__ pks,
    const uint32_t* __restrict__ sigs, uint64_t i0, uint64_t ns, int32_t* __restrict__ status,
    key_tables_t keys, const ge_niels_pad* __restrict__ bcomb, vote_planes_t vp) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ns) return;
  const uint64_t gi = i0 + i;
  const uint32_t kk = keys.vote_key[gi];
  uint32_t st = kVoteFail;
  if (kk != kNoKey) {
    const strict_src_global src{pks + 8 * gi, sigs + 16 * gi,
                                msgs + (uint64_t)msg_stride_words * gi};
    fe X, Z;
    st = keyed_vote_check(src, g_consts.sk, bcomb_wide{bcomb},
                          keytab_wide{keys.tabs + keys.ks.tab * (uint64_t)kk, keys.ks}, keys.ok[kk], X, Z);
    if (st >= kVotePending) {
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        vp.planes[(uint64_t)k * vp.S + i] = X.v[k];
        vp.planes[(uint64_t)(10 + k) * vp.S + i] = Z.v[k];
      }
    }
  }
  if (st == kVotePass) status[gi] = NW_OK;
  vp.state[i] = st;
}

// Parity of the pending items (Montgomery's trick per strided chunk, as k_votes_keyed_inv):
// a match is status 0, a mismatch goes to the list.
__global__ __launch_bounds__(256) void k_strict_keyed_inv(uint64_t i0, uint64_t ns,
                                                          uint64_t nchunks,
                                                          int32_t* __restrict__ status,
                                                          vote_planes_t vp) {
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nchunks) return;
  auto load = [&](fe& f, int base, uint64_t i) {
#pragma unroll
    for (int k = 0; k < 10; ++k) f.v[k] = vp.planes[(uint64_t)(base + k) * vp.S + i];
  };
  fe acc;
  fe_1(acc);
  uint64_t last = ~0ull;
#pragma unroll 1
  for (uint64_t i = lane; i < ns; i += nchunks) {
    if (vp.state[i] < kVotePending) continue;
    fe X, Z, W;
    load(X, 0, i);
    load(Z, 10, i);
    fe_mul(W, X, acc);
#pragma unroll
    for (int k = 0; k < 10; ++k) vp.planes[(uint64_t)k * vp.S + i] = W.v[k];
    fe_mul(acc, acc, Z);
    last = i;
  }
  if (last == ~0ull) return;
  fe inv;
  fe_invert(inv, acc);
#pragma unroll 1
  for (uint64_t i = last;; i -= nchunks) {
    const uint32_t st = vp.state[i];
    if (st >= kVotePending) {
      fe W, Z, x;
      load(W, 0, i);
      load(Z, 10, i);
      fe_mul(x, W, inv);
      if (fe_isnegative(x) != (st & 1)) vp.state[i] = kVoteFail;
      else status[i0 + i] = NW_OK;
      fe_mul(inv, inv, Z);
    }
    if (i < nchunks) break;
  }
}

// Failed / unkeyed items of the slice -> list (one atomic per wave).
__global__ __launch_bounds__(256) void k_strict_keyed_list(uint64_t i0, uint64_t ns,
                                                           const uint32_t* __restrict__ state,
                                                           uint32_t* __restrict__ list,
                                                           uint32_t* __restrict__ count) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool f = i < ns && state[i] == kVoteFail;
  const uint64_t m = __ballot(f);
  if (m == 0) return;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t base = 0;
  if (lane == (uint32_t)(__ffsll((unsigned long long)m) - 1))
    base = atomicAdd(count, (uint32_t)__popcll(m));
  base = (uint32_t)__shfl((int)base, __ffsll((unsigned long long)m) - 1);
  if (f) list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint32_t)(i0 + i);
}

// Verdict bitmap from the statuses (bit i set iff status[i] == 0), 64 items per wave.
__global__ __launch_bounds__(256) void k_status_bitmap(const int32_t* __restrict__ status,
                                                       uint64_t n, uint64_t* __restrict__ bitmap) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t m = __ballot(i < n && status[i] == NW_OK);
  if ((threadIdx.x & 63) == 0 && i < n) bitmap[i >> 6] = m;
}

// Certificate votes checked one by one with the keyed comb (Certificate::verify's
// Signature::verify_batch, messages.rs:212, without merging). A vote whose strict check
// passes satisfies R == [s]B - [k]A exactly, so its term of any random linear combination
// vanishes: a certificate all of whose votes pass is Ok under verify_batch too. Every other
// certificate keeps cert_ok = 0 and gets its own verify_batch (launch_verify_batch with
// skip_group_ok = cert_ok, one certificate per group), so statuses and fail indices are the
// per-certificate path's. Certificates already decided by an earlier check are left alone
// (their batch status is never read).
//
// R is never decompressed (nw_strict.hpp keyed_vote_check): R' = [s]B - [k]A is compared
// with R's encoding through Y' == y_R Z' and the parity of X'/Z'. The parity needs 1/Z':
// k_votes_keyed writes X', Z' of the votes that got that far into limb planes, and
// k_votes_keyed_inv inverts them in batches (Montgomery's trick, one lane per strided chunk
// of votes: 4 multiplications per vote and one inversion per chunk instead of the ~265
// squarings of a decompression per vote).
__global__ __launch_bounds__(256) void k_votes_keyed_init(const uint64_t* __restrict__ cvo,
                                                          uint64_t ncert,
                                                          uint32_t* __restrict__ cert_ok) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncert) cert_ok[c] = cvo[c + 1] > cvo[c] ? 1u : 0u;   // no votes: its own batch
}


// Key-major order of a slice's votes (k_vk_hist / k_vk_scan / k_vk_scatter: a counting sort
// by committee key; the votes of already-decided certificates and non-members go to one
// last bin whose lanes do no comb work). With 16-bit key tables (67 MB per key) a wave whose
// lanes name ~64 different keys gathers from the whole committee's tables (6.7 GB at
// N = 100: HBM and TLB bound); sorted, the chip works on one or two keys' tables at a time,
// which stay in the last-level caches.
constexpr uint32_t kVkMaxBins = 1024;
constexpr uint32_t kVkSortMinKeys = 32;
__device__ __forceinline__ uint32_t vk_bin(const uint32_t* __restrict__ vote_cert,
                                           const uint32_t* __restrict__ vote_key, uint64_t v,
                                           const int32_t* __restrict__ pre1,
                                           const int32_t* __restrict__ pre2,
                                           const int32_t* __restrict__ hdr_st, uint32_t nkeys) {
  const uint32_t c = vote_cert[v];
  if (pre1[c] != 0 || (hdr_st && hdr_st[c] != 0) || pre2[c] != 0) return nkeys;
  const uint32_t k = vote_key[v];
  return k < nkeys ? k : nkeys;
}
// Blocks take contiguous chunks of kVkChunk votes: one global atomic per (block, bin), not
// per (256 votes, bin) — with ~100 bins per block the per-block form made the 26M global
// atomics of N = 100 serialize on 100 addresses (4.9 ms per pass).
constexpr uint32_t kVkChunk = 16384;
__global__ __launch_bounds__(256) void k_vk_hist(const uint32_t* __restrict__ vote_cert,
                                                 const uint32_t* __restrict__ vote_key,
                                                 uint64_t v0, uint64_t nv,
                                                 const int32_t* __restrict__ pre1,
                                                 const int32_t* __restrict__ pre2,
                                                 const int32_t* __restrict__ hdr_st,
                                                 uint32_t nkeys, uint32_t* __restrict__ gh) {
  __shared__ uint32_t h[kVkMaxBins];
  for (uint32_t b = threadIdx.x; b <= nkeys; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint64_t c0 = (uint64_t)blockIdx.x * kVkChunk;
  const uint64_t c1 = c0 + kVkChunk < nv ? c0 + kVkChunk : nv;
  for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x)
    atomicAdd(&h[vk_bin(vote_cert, vote_key, v0 + i, pre1, pre2, hdr_st, nkeys)], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b <= nkeys; b += blockDim.x)
    if (h[b]) atomicAdd(&gh[b], h[b]);
}
__global__ __launch_bounds__(64) void k_vk_scan(uint32_t* __restrict__ gh, uint32_t nbins) {
  if (threadIdx.x != 0) return;
  uint32_t acc = 0;
  for (uint32_t b = 0; b < nbins; ++b) {
    const uint32_t c = gh[b];
    gh[b] = acc;
    acc += c;
  }
}
// Same chunks: count again, reserve the block's range in every bin (one atomic each), then
// hand out positions inside the ranges with LDS cursors.
__global__ __launch_bounds__(256) void k_vk_scatter(const uint32_t* __restrict__ vote_cert,
                                                    const uint32_t* __restrict__ vote_key,
                                                    uint64_t v0, uint64_t nv,
                                                    const int32_t* __restrict__ pre1,
                                                    const int32_t* __restrict__ pre2,
                                                    const int32_t* __restrict__ hdr_st,
                                                    uint32_t nkeys, uint32_t* __restrict__ cursor,
                                                    uint32_t* __restrict__ perm) {
  __shared__ uint32_t h[kVkMaxBins];
  for (uint32_t b = threadIdx.x; b <= nkeys; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint64_t c0 = (uint64_t)blockIdx.x * kVkChunk;
  const uint64_t c1 = c0 + kVkChunk < nv ? c0 + kVkChunk : nv;
  for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x)
    atomicAdd(&h[vk_bin(vote_cert, vote_key, v0 + i, pre1, pre2, hdr_st, nkeys)], 1u);
  __syncthreads();
  for (uint32_t x = threadIdx.x; x <= nkeys; x += blockDim.x)
    if (h[x]) h[x] = atomicAdd(&cursor[x], h[x]);   // this block's range in bin x
  __syncthreads();
  for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
    const uint32_t b = vk_bin(vote_cert, vote_key, v0 + i, pre1, pre2, hdr_st, nkeys);
    perm[atomicAdd(&h[b], 1u)] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256, NW_KEYED_WAVES) void k_votes_keyed(
    const uint32_t* __restrict__ cert_digest, const uint32_t* __restrict__ vote_cert,
    uint64_t v0, uint64_t nv, const uint32_t* __restrict__ pks,
    const uint32_t* __restrict__ sigs, const int32_t* __restrict__ pre1,
    const int32_t* __restrict__ pre2, const int32_t* __restrict__ hdr_st, key_tables_t keys,
    const ge_niels_pad* __restrict__ bcomb, uint32_t* __restrict__ cert_ok, vote_planes_t vp) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nv) return;
  const uint64_t v = v0 + (vp.perm ? vp.perm[i] : i);
  const uint32_t c = vote_cert[v];
  uint32_t st = kVotePass;
  if (pre1[c] == 0 && (!hdr_st || hdr_st[c] == 0) && pre2[c] == 0) {
    const uint32_t kk = keys.vote_key[v];
    if (kk == kNoKey) {   // not a committee key (cannot happen for an undecided certificate)
      st = kVoteFail;
    } else {
      const strict_src_global src{pks + 8 * v, sigs + 16 * v, cert_digest + 8 * (uint64_t)c};
      fe X, Z;
      st = keyed_vote_check(src, g_consts.sk, bcomb_wide{bcomb},
                            keytab_wide{keys.tabs + keys.ks.tab * (uint64_t)kk, keys.ks}, keys.ok[kk], X, Z);
      if (st >= kVotePending) {
#pragma unroll
        for (int k = 0; k < 10; ++k) {
          vp.planes[(uint64_t)k * vp.S + i] = X.v[k];
          vp.planes[(uint64_t)(10 + k) * vp.S + i] = Z.v[k];
        }
      }
    }
    if (st == kVoteFail) cert_ok[c] = 0;   // same value from every failing lane
  }
  vp.state[i] = st;
}

// After votes were checked concurrently with the headers (hdr_st not yet known to them):
// a certificate whose header failed is decided by its header, so it skips its own
// verify_batch (cert_ok = 1 is the skip flag there).
__global__ __launch_bounds__(256) void k_cert_ok_headers(const int32_t* __restrict__ hdr_st,
                                                         uint64_t ncert,
                                                         uint32_t* __restrict__ cert_ok) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < ncert && hdr_st[c] != 0) cert_ok[c] = 1u;
}

// One lane per chunk {i = j * nchunks + lane}: Montgomery's trick over the chunk's pending
// votes. Forward: W_i = X'_i * (product of the earlier Z'), acc *= Z'_i (W_i over X'_i);
// one inversion of the product; backward: x_i = W_i * inv, inv *= Z'_i. A vote whose x
// parity differs from its sign bit fails its certificate.
__global__ __launch_bounds__(256) void k_votes_keyed_inv(const uint32_t* __restrict__ vote_cert,
                                                         uint64_t v0, uint64_t nv,
                                                         uint64_t nchunks,
                                                         uint32_t* __restrict__ cert_ok,
                                                         vote_planes_t vp) {
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= nchunks) return;
  auto load = [&](fe& f, int base, uint64_t i) {
#pragma unroll
    for (int k = 0; k < 10; ++k) f.v[k] = vp.planes[(uint64_t)(base + k) * vp.S + i];
  };
  fe acc;
  fe_1(acc);
  uint64_t last = ~0ull;
#pragma unroll 1
  for (uint64_t i = lane; i < nv; i += nchunks) {
    if (vp.state[i] < kVotePending) continue;
    fe X, Z, W;
    load(X, 0, i);
    load(Z, 10, i);
    fe_mul(W, X, acc);
#pragma unroll
    for (int k = 0; k < 10; ++k) vp.planes[(uint64_t)k * vp.S + i] = W.v[k];
    fe_mul(acc, acc, Z);
    last = i;
  }
  if (last == ~0ull) return;
  fe inv;
  fe_invert(inv, acc);
#pragma unroll 1
  for (uint64_t i = last;; i -= nchunks) {
    const uint32_t st = vp.state[i];
    if (st >= kVotePending) {
      fe W, Z, x;
      load(W, 0, i);
      load(Z, 10, i);
      fe_mul(x, W, inv);
      if (fe_isnegative(x) != (st & 1))
        cert_ok[vote_cert[v0 + (vp.perm ? vp.perm[i] : i)]] = 0;
      fe_mul(inv, inv, Z);
    }
    if (i < nchunks) break;
  }
}

// ---------------------------------------------------------------------------------------
// Key generation and signing (crypto::generate_keypair / Signature::new, lib.rs:167-191;
// dalek Keypair::generate + ExpandedSecretKey::sign = RFC 8032)
// ---------------------------------------------------------------------------------------
// SHA-512 of nwords64 whole 64-bit words (<= 13, one block), words given big-endian.
__device__ __forceinline__ void sha512_words(uint64_t st[8], const uint64_t* m, int nwords64) {
  uint64_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = i < nwords64 ? m[i] : 0;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i == nwords64) w[i] = 0x8000000000000000ULL;
  w[15] = (uint64_t)nwords64 * 64;
  sha512_init(st);
  sha512_compress(st, w);
}

__device__ __forceinline__ uint64_t be64_of_le_words(const uint32_t* x, int i) {
  return ((uint64_t)bswap32(x[2 * i]) << 32) | bswap32(x[2 * i + 1]);
}

// Expanded secret: a = clamp(H(seed)[0..32]) mod l, prefix = H(seed)[32..64] (LE words).
__device__ __forceinline__ void expand_seed(sc& a, uint32_t prefix[8], const uint32_t seed[8]) {
  uint64_t m[4], st[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) m[i] = be64_of_le_words(seed, i);
  sha512_words(st, m, 4);
  uint32_t h[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[2 * i] = bswap32((uint32_t)(st[i] >> 32));
    h[2 * i + 1] = bswap32((uint32_t)st[i]);
  }
  h[0] &= 0xfffffff8u;
  h[7] = (h[7] & 0x7fffffffu) | 0x40000000u;
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = i < 8 ? h[i] : 0u;
  sc_reduce512(a, x);   // [a]B = [a mod l]B
#pragma unroll
  for (int i = 0; i < 8; ++i) prefix[i] = h[8 + i];
}

__global__ __launch_bounds__(256) void k_keypair(const uint32_t* __restrict__ seeds, uint64_t n,
                                                 uint32_t* __restrict__ pks) {
  __shared__ ge_niels s_btab[129];
  load_btab(s_btab);
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t seed[8], prefix[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) seed[j] = seeds[8 * i + j];
  sc a;
  expand_seed(a, prefix, seed);
  ge A;
  fixed_base_mul(A, a, s_btab);
  uint32_t Aw[8];
  ge_tobytes(Aw, A);
#pragma unroll
  for (int j = 0; j < 8; ++j) pks[8 * i + j] = Aw[j];
}

// sks: crypto::SecretKey bytes (seed || pk), stride sk_stride_words (16, or 0 = one key).
__global__ __launch_bounds__(256) void k_sign(const uint32_t* __restrict__ sks,
                                              uint32_t sk_stride_words,
                                              const uint32_t* __restrict__ msgs,
                                              uint32_t msg_stride_words, uint64_t n,
                                              uint32_t* __restrict__ sigs) {
  __shared__ ge_niels s_btab[129];
  load_btab(s_btab);
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t seed[8], pk[8], M[8], prefix[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    seed[j] = sks[(uint64_t)sk_stride_words * i + j];
    pk[j] = sks[(uint64_t)sk_stride_words * i + 8 + j];
    M[j] = msgs[(uint64_t)msg_stride_words * i + j];
  }
  sc a;
  expand_seed(a, prefix, seed);
  // r = H(prefix || M) mod l
  uint64_t m[8], st[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = be64_of_le_words(prefix, j);
    m[4 + j] = be64_of_le_words(M, j);
  }
  sha512_words(st, m, 8);
  uint32_t hx[16];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hx[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    hx[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
  sc r;
  sc_reduce512(r, hx);
  ge R;
  fixed_base_mul(R, r, s_btab);
  uint32_t Rw[8];
  ge_tobytes(Rw, R);
  hram96(hx, Rw, pk, M);
  sc k, ka, s;
  sc_reduce512(k, hx);
  sc_mul(ka, k, a);
  sc_add(s, ka, r);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sigs[16 * i + j] = Rw[j];
    sigs[16 * i + 8 + j] = s.w[j];
  }
}

}  // namespace nw

namespace nw {
// The strict kernel's wide B tables, built on the device once per process and device, in
// padded affine niels form, one lane per entry: fixed-base product over the 8-bit LDS table,
// then one inversion.
// out[h * n + j] = j * 2^(shift h) * B for h < ntab (shift 128: the ladder's two tables;
// shift 16: the keyed comb's sixteen).
__global__ __launch_bounds__(256) void k_btab_build(ge_niels_pad* __restrict__ out, uint32_t n,
                                                    uint32_t ntab, uint32_t shift) {
  __shared__ ge_niels s_btab[129];
  load_btab(s_btab);
  __syncthreads();
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (uint64_t)ntab * n) return;
  const uint32_t h = (uint32_t)(g / n), j = (uint32_t)(g % n);
  sc s;
#pragma unroll
  for (int i = 0; i < 8; ++i) s.w[i] = 0;
  const uint32_t bit = shift * h, wi = bit >> 5, sh = bit & 31;   // j < 2^24, bit <= 240
  s.w[wi] = j << sh;
  if (sh && wi < 7) s.w[wi + 1] = j >> (32 - sh);
  ge P;
  fixed_base_mul(P, s, s_btab);
  ge_niels nb;
  ge_to_niels(nb, P, g_consts.k.d2);
  out[g].n = nb;
  out[g].pad[0] = out[g].pad[1] = 0;
}
}  // namespace nw

// ---------------------------------------------------------------------------------------
// Host side: constants and launchers
// ---------------------------------------------------------------------------------------
namespace nw {

// The strict kernel's wide B tables (k_btab_build), one copy per device, indexed by HIP
// device id, built on the device the first time a strict launch needs them there (24-bit
// windows: 2 x 8,388,609 entries = 2.15 GB and ~0.2 s per device; lazily, so a process
// that initialises every device but verifies on one builds one table).
static constexpr int kMaxDevIds = 64;
static std::atomic<ge_niels_pad*> g_btw[kMaxDevIds];
static std::mutex g_btw_mu[kMaxDevIds];   // per device: devices build in parallel
static constexpr uint32_t kBtwPerHalf = bdigits<NW_BWIN>::ENTRIES;

static std::atomic<ge_niels_pad*> g_bcomb[kMaxDevIds];

hipError_t table_malloc(void** p, size_t bytes) {
  *p = nullptr;
  if (const char* e = getenv("NW_DEVICE_MEM_LIMIT")) {
    const unsigned long long lim = strtoull(e, nullptr, 10);
    if (lim && bytes > lim) return hipErrorOutOfMemory;
  }
  const hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    // reported by the return value; leave no last error behind for the next launch check
    *p = nullptr;
    (void)hipGetLastError();
  }
  return e;
}


// Table set `which` of the current device (0: the ladder's 2 x kBtwPerHalf; 1: the keyed
// comb's kBCombT x kBCombN: 11 x 8,388,609 = 11.8 GB at 24-bit digits), built on first use.
static hipError_t btab_for_current_device(int which, const ge_niels_pad** out) {
  *out = nullptr;
  if (which == 0 && NW_BWIN == 8) return hipSuccess;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kMaxDevIds) return hipErrorInvalidDevice;
  std::atomic<ge_niels_pad*>& slot = which ? g_bcomb[dev] : g_btw[dev];
  if ((*out = slot.load(std::memory_order_acquire))) return hipSuccess;
  std::lock_guard<std::mutex> lock(g_btw_mu[dev]);
  if ((*out = slot.load(std::memory_order_relaxed))) return hipSuccess;
  const uint32_t n = which ? kBCombN : kBtwPerHalf, ntab = which ? kBCombT : 2;
  const uint32_t shift = which ? (uint32_t)kBCombW : 128;
  void* p = nullptr;
  const uint64_t entries = (uint64_t)ntab * n;
  e = table_malloc(&p, entries * sizeof(ge_niels_pad));
  if (e != hipSuccess) return e;
  hipStream_t s = nullptr;
  e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_btab_build, dim3((unsigned)((entries + 255) / 256)), dim3(256), 0, s,
                       static_cast<ge_niels_pad*>(p), n, ntab, shift);
    e = hipGetLastError();
    const hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    (void)hipStreamDestroy(s);
  }
  if (e != hipSuccess) { (void)hipFree(p); return e; }
  slot.store(static_cast<ge_niels_pad*>(p), std::memory_order_release);
  *out = static_cast<ge_niels_pad*>(p);
  return hipSuccess;
}

hipError_t bcomb_table(const ge_niels_pad** out) { return btab_for_current_device(1, out); }

hipError_t prepare_strict_tables() {
  const ge_niels_pad* p = nullptr;
  hipError_t e = btab_for_current_device(0, &p);
  return e != hipSuccess ? e : btab_for_current_device(1, &p);
}

hipError_t upload_consts() {
  static dev_consts host;
  static std::once_flag once;
  std::call_once(once, [] {
    compute_consts(host.k, host.btab);
    compute_strict_consts(host.sk, host.b128);
  });
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_consts), &host, sizeof(host), 0,
                                   hipMemcpyHostToDevice);
  if (e == hipSuccess) e = upload_batch_consts();
  return e != hipSuccess ? e : upload_small_consts();
}

static inline unsigned grid_for(uint64_t n, unsigned block) {
  return (unsigned)((n + block - 1) / block);
}

hipError_t launch_sha512_digest32(const uint8_t* data, const uint64_t* offsets,
                                  const uint64_t* lengths, uint64_t n, uint32_t* out,
                                  hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sha512_digest32, dim3(grid_for(n, 256)), dim3(256), 0, stream, data,
                     offsets, lengths, n, out);
  return hipGetLastError();
}

// Resident 256-thread blocks of k_verify_strict on the current device (occupancy query,
// once per device; concurrent first calls compute the same value).
static unsigned strict_grid() {
  static std::atomic<int> cached[64];
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cached[dev].load(std::memory_order_acquire)) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_verify_strict<false>, 256, 0) !=
            hipSuccess || per_cu <= 0)
      per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    cached[dev].store(per_cu * cus, std::memory_order_release);
  }
  return (unsigned)cached[dev].load(std::memory_order_acquire);
}

// The keyed fast path reuses the per-lane table region for its limb planes (84 B per item of
// a slice) and keeps its list (4 B per item) and count in a tail after it.
constexpr uint64_t kKeyedSliceMax = 1ull << 22;
// (sized for 160-byte entries; the packed ones use 128 of each 160)
static size_t strict_tabs_bytes() { return (size_t)strict_grid() * 256 * 16 * sizeof(ge_cached); }
// The two-pass path's slice (k_strict_triage / k_verify_strict_pre): x of A and R (20 words)
// and a list entry per item, after the keyed path's region (1.4 GB, once per device). Large:
// config 4's 12.5M items are one slice, so the second pass's last, partly filled round over
// the resident lanes comes once per launch.
constexpr uint64_t kTriageSlice = 1ull << 24;
static size_t strict_keyed_region_bytes() { return 4 * kKeyedSliceMax + 256; }
size_t strict_workspace_bytes() {
  return strict_tabs_bytes() + strict_keyed_region_bytes() + 84 * kTriageSlice + 256;
}
bool strict_triage_on() {   // NW_STRICT_TRIAGE=0: one pass (k_verify_strict), A/B hook
  static const bool v = [] {
    const char* e = getenv("NW_STRICT_TRIAGE");
    return !(e && e[0] == '0');
  }();
  return v;
}

hipError_t launch_verify_strict(const uint32_t* msgs, uint32_t msg_stride_words,
                                const uint32_t* pks, const uint32_t* sigs, uint64_t n,
                                int32_t* status, uint64_t* bitmap, void* workspace,
                                hipStream_t stream, const key_tables_t* keys) {
  if (n == 0) return hipSuccess;
  const unsigned grid = std::min<uint64_t>(strict_grid(), grid_for(n, 256));
  const key_tables_t kt = keys ? *keys : key_tables_t{nullptr, nullptr, nullptr, {}};
  const ge_niels_pad* btw = nullptr;
  const ge_niels_pad* bcomb = nullptr;
  hipError_t eb = btab_for_current_device(0, &btw);
  if (eb == hipSuccess && kt.vote_key) eb = btab_for_current_device(1, &bcomb);
  if (eb != hipSuccess) return eb;
  const char* kf = getenv("NW_STRICT_KEYED_FAST");
  if (!kt.vote_key && strict_triage_on()) {
    char* const ws = static_cast<char*>(workspace);
    char* const tri = ws + strict_tabs_bytes() + strict_keyed_region_bytes();
    uint32_t* const xs = reinterpret_cast<uint32_t*>(tri);
    uint32_t* const list = xs + 20 * kTriageSlice;
    uint32_t* const count = list + kTriageSlice;
    // equal slices of at most kTriageSlice items
    const uint64_t nsl = (n + kTriageSlice - 1) / kTriageSlice;
    const uint64_t per = (n + nsl - 1) / nsl;
    for (uint64_t i0 = 0; i0 < n; i0 += per) {
      const uint64_t ns = std::min(per, n - i0);
      hipError_t e = hipMemsetAsync(count, 0, 4, stream);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_strict_triage, dim3(grid_for(ns, 256)), dim3(256), 0, stream, msgs,
                         msg_stride_words, pks, sigs, i0, ns, status, xs, kTriageSlice, list,
                         count);
      hipLaunchKernelGGL(k_verify_strict_pre,
                         dim3(std::min<uint64_t>(strict_grid(), grid_for(ns, 256))), dim3(256),
                         0, stream, msgs, msg_stride_words, pks, sigs, i0, list, count, xs,
                         kTriageSlice, status, static_cast<ge_cached_pk*>(workspace), btw);
    }
    if (bitmap)
      hipLaunchKernelGGL(k_status_bitmap, dim3(grid_for(n, 256)), dim3(256), 0, stream, status,
                         n, bitmap);
    return hipGetLastError();
  }
  if (!kt.vote_key) {
    hipLaunchKernelGGL(k_verify_strict<false>, dim3(grid), dim3(256), 0,
                       stream, msgs,
                       msg_stride_words, pks, sigs, n, status, bitmap,
                       static_cast<ge_cached_pk*>(workspace), kt, btw, bcomb, nullptr, nullptr);
    return hipGetLastError();
  }
  if (kf && kf[0] == '0') {
    hipLaunchKernelGGL(k_verify_strict<true>, dim3(grid), dim3(256), 0, stream, msgs,
                       msg_stride_words, pks, sigs, n, status, bitmap,
                       static_cast<ge_cached_pk*>(workspace), kt, btw, bcomb, nullptr, nullptr);
    return hipGetLastError();
  }
  // keyed fast path (k_strict_keyed above), slice by slice through the workspace
  const uint64_t S = std::min<uint64_t>(kKeyedSliceMax, strict_tabs_bytes() / (4 * 21)) & ~63ull;
  uint32_t* base = static_cast<uint32_t*>(workspace);
  uint32_t* list = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + strict_tabs_bytes());
  uint32_t* count = list + kKeyedSliceMax;
  const vote_planes_t vp{base, base + 20 * S, S, nullptr};
  for (uint64_t i0 = 0; i0 < n; i0 += S) {
    const uint64_t ns = std::min(S, n - i0);
    hipError_t e = hipMemsetAsync(count, 0, 4, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_strict_keyed, dim3(grid_for(ns, 256)), dim3(256), 0, stream, msgs,
                       msg_stride_words, pks, sigs, i0, ns, status, kt, bcomb, vp);
    const uint64_t nchunks = std::min<uint64_t>(ns, 256ull * 4 * 2 * 64);
    hipLaunchKernelGGL(k_strict_keyed_inv, dim3(grid_for(nchunks, 256)), dim3(256), 0, stream,
                       i0, ns, nchunks, status, vp);
    hipLaunchKernelGGL(k_strict_keyed_list, dim3(grid_for(ns, 256)), dim3(256), 0, stream, i0,
                       ns, vp.state, list, count);
    // the leftovers: full verification (exact status codes), the tables over the planes
    hipLaunchKernelGGL(k_verify_strict<true>, dim3(std::min<uint64_t>(strict_grid(), grid_for(ns, 256))),
                       dim3(256), 0, stream, msgs, msg_stride_words, pks, sigs, ns, status,
                       bitmap, static_cast<ge_cached_pk*>(workspace), kt, btw, bcomb, list, count);
  }
  if (bitmap)
    hipLaunchKernelGGL(k_status_bitmap, dim3(grid_for(n, 256)), dim3(256), 0, stream, status, n,
                       bitmap);
  return hipGetLastError();
}

size_t votes_keyed_bytes_per_vote() { return 4 * 22; }   // 20 limb planes, state, perm
size_t votes_keyed_fixed_bytes() { return 4 * kVkMaxBins; }   // key histogram / cursors

hipError_t launch_votes_keyed(const uint32_t* cert_digest, const uint64_t* cvo, uint64_t ncert,
                              const uint32_t* vote_cert, const uint32_t* pks,
                              const uint32_t* sigs, uint64_t nvotes, const int32_t* pre1,
                              const int32_t* pre2, const int32_t* hdr_st,
                              const key_tables_t& keys, uint32_t nkeys, uint32_t* cert_ok,
                              void* scratch, size_t scratch_bytes, hipStream_t stream) {
  if (ncert == 0) return hipSuccess;
  if (!keys.vote_key || !keys.tabs || !keys.ok || !vote_cert) return hipErrorInvalidValue;
  const ge_niels_pad* bcomb = nullptr;
  hipError_t eb = btab_for_current_device(1, &bcomb);
  if (eb != hipSuccess) return eb;
  hipLaunchKernelGGL(k_votes_keyed_init, dim3(grid_for(ncert, 256)), dim3(256), 0, stream, cvo,
                     ncert, cert_ok);
  // slices of S votes through the scratch (the caller's verify_batch workspace, free until
  // the failed certificates' batches run)
  if (nvotes == 0) return hipGetLastError();   // e.g. genesis certificates: no votes
  if (scratch_bytes < votes_keyed_fixed_bytes()) return hipErrorInvalidValue;
  const uint64_t cap = (scratch_bytes - votes_keyed_fixed_bytes()) / votes_keyed_bytes_per_vote();
  const uint64_t S = nvotes <= cap ? nvotes : cap & ~63ull;
  if (nvotes && S == 0) return hipErrorInvalidValue;
  uint32_t* gh = static_cast<uint32_t*>(scratch);
  uint32_t* base = gh + kVkMaxBins;
  // key-major order for committees whose tables overflow the caches (>= 32 keys: 2.1 GB of
  // 16-bit tables; config 2 N = 100: 7.58 -> 9.11 M certs/s in round 3; N = 50 22.4 -> 23.3
  // in round 5, profiles/r05kw2, though round 3 measured it slower there) — below that the
  // cert-major order's coalesced signature reads win (round 3: N = 4 / 10: 143 / 74
  // unsorted vs 137 / 72 sorted). NW_VOTES_KEY_MAJOR=1 / 0 forces it on / off.
  const char* km = getenv("NW_VOTES_KEY_MAJOR");
  const bool sort = nkeys + 1 <= kVkMaxBins &&
                    (km ? km[0] == '1' : nkeys >= kVkSortMinKeys);
  uint32_t* perm = base + 21 * S;
  const vote_planes_t vp{base, base + 20 * S, S, sort ? perm : nullptr};
  for (uint64_t v0 = 0; v0 < nvotes; v0 += S) {
    const uint64_t nv = std::min(S, nvotes - v0);
    if (sort) {
      hipError_t e = hipMemsetAsync(gh, 0, 4 * (nkeys + 1), stream);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_vk_hist, dim3(grid_for(nv, kVkChunk)), dim3(256), 0, stream, vote_cert,
                         keys.vote_key, v0, nv, pre1, pre2, hdr_st, nkeys, gh);
      hipLaunchKernelGGL(k_vk_scan, dim3(1), dim3(64), 0, stream, gh, nkeys + 1);
      hipLaunchKernelGGL(k_vk_scatter, dim3(grid_for(nv, kVkChunk)), dim3(256), 0, stream, vote_cert,
                         keys.vote_key, v0, nv, pre1, pre2, hdr_st, nkeys, gh, perm);
    }
    hipLaunchKernelGGL(k_votes_keyed, dim3(grid_for(nv, 256)), dim3(256), 0, stream,
                       cert_digest, vote_cert, v0, nv, pks, sigs, pre1, pre2, hdr_st, keys, bcomb,
                       cert_ok, vp);
    // chunks: ~2 waves per SIMD of lanes, each over nv / nchunks votes (>= 1)
    const uint64_t nchunks = std::min<uint64_t>(nv, 256ull * 4 * 2 * 64);
    hipLaunchKernelGGL(k_votes_keyed_inv, dim3(grid_for(nchunks, 256)), dim3(256), 0, stream,
                       vote_cert, v0, nv, nchunks, cert_ok, vp);
  }
  return hipGetLastError();
}

hipError_t launch_cert_ok_headers(const int32_t* hdr_st, uint64_t ncert, uint32_t* cert_ok,
                                  hipStream_t stream) {
  if (ncert == 0) return hipSuccess;
  hipLaunchKernelGGL(k_cert_ok_headers, dim3(grid_for(ncert, 256)), dim3(256), 0, stream, hdr_st,
                     ncert, cert_ok);
  return hipGetLastError();
}

hipError_t launch_keypair(const uint32_t* seeds, uint64_t n, uint32_t* pks, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_keypair, dim3(grid_for(n, 256)), dim3(256), 0, stream, seeds, n, pks);
  return hipGetLastError();
}

hipError_t launch_sign(const uint32_t* sks, uint32_t sk_stride_words, const uint32_t* msgs,
                       uint32_t msg_stride_words, uint64_t n, uint32_t* sigs,
                       hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_sign, dim3(grid_for(n, 256)), dim3(256), 0, stream, sks, sk_stride_words,
                     msgs, msg_stride_words, n, sigs);
  return hipGetLastError();
}

}  // namespace nw
