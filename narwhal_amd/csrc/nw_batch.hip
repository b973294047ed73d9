// nw_batch.hip — crypto::Signature::verify_batch (crypto/src/lib.rs:206-219 -> dalek
// verify_batch [ext]) for many independent batches: a chunked Straus multi-scalar
// multiplication for small batches (certificates), a Pippenger bucket MSM (k_pip_*, below)
// for batches of at least NW_BATCH_PIPPENGER_MIN votes:
//
//   sum_i z_i R_i + sum_i (z_i k_i mod l) A_i - (sum_i z_i s_i mod l) B == identity
//
//   k_bv_plan_*   a block scan per slice: splits every batch into ceil(n_b / C) balanced
//                 chunks (block-wide scan) and lists the batches that need a combine step.
//   k_bv_items    one lane per vote: parse/decode flags, k_i = H(R||A||M) mod l, z_i
//                 (ChaCha20 or injected), c_i = z_i k_i, b_i = z_i s_i, signed 4-bit
//                 digits of c_i and z_i, and the tables j*A_i, j*R_i (j = 1..8, cached form)
//                 written to HBM.
//   k_bv_chunks   one lane per chunk: a Straus ladder shared by the chunk's 2m points and
//                 B — 252 doublings per chunk instead of per vote — adding table entries
//                 per 4-bit window and [-(sum b)]B by 8-bit windows over the LDS B table.
//                 A batch that is a single chunk is finished here (identity test + first
//                 failure in reference order).
//   k_bv_combine  one wave per multi-chunk (or empty) batch: sums the chunk points, the
//                 first failures, and tests the total.
//
// Work per vote: 2 decompressions, ~97 table additions and the tables (SURVEY 8(d):
// 64,000 MAC/vote at n >= 10k); the 252 doublings and the B term are shared per chunk.
#include "narwhal_amd.h"
#include "nw_kernels.h"
#include "nw_point.hpp"
#include "nw_scalar.hpp"
#include "nw_sha512.hpp"
#include "nw_ladder.hpp"
#include "nw_consts.hpp"
#include "nw_strict.hpp"
#include "nw_lp.hpp"
#include "nw_chacha.hpp"

#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <vector>

namespace nw {

namespace {

struct batch_consts {
  curve_consts k;
  ge_niels btab[129];   // j * B
  ge_niels b128[129];   // j * 2^128 B (short ladders of keyed chunks)
  torsion_consts tor;   // [j] T8 (k_key_base: a committee key's lambda)
  uint32_t l[8];        // the group order l, little-endian words
};
__constant__ batch_consts g_bc;
// j * 2^(8 w) * B (nw_consts.hpp compute_comb): [-sum b_i]B in 32 additions, no doublings
__device__ ge_niels g_comb[32 * 129];

constexpr int BT_WORDS = 129 * 30;
constexpr uint64_t kSliceUnits = 4ull << 20;   // items + batches per slice (workspace bound)

// Test hooks (tests/test_gpu_batch.py): NW_BATCH_SLICE_UNITS shrinks the slice, and
// NW_BATCH_CHUNK fixes the chunk size, so small inputs exercise every path.
uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  const unsigned long long x = strtoull(v, nullptr, 10);
  return x ? (uint64_t)x : dflt;
}
// as env_u64, but a set value of 0 counts (switches whose "off" is 0)
uint64_t env_u64_zero(const char* name, uint64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return (uint64_t)strtoull(v, nullptr, 10);
}
// (never above kSliceUnits: k_bv_plan_top scans at most 4096 plan blocks)
uint64_t slice_units() { return std::min(env_u64("NW_BATCH_SLICE_UNITS", kSliceUnits), kSliceUnits); }
constexpr uint32_t kMaxChunk = 128;
constexpr uint32_t kNone = 0xffffffffu;

// Per-vote record written by k_bv_items (96 bytes).
struct bv_item {
  uint32_t c[8];     // c_i = z_i k_i mod l, recoded: + 0x88..8 (signed 4-bit digits), or
                     // for a keyed vote + 0x80..80 (signed 8-bit digits, 16 low + 16 high)
  uint32_t z[5];     // z_i + 0x88..8 (33 digits)
  uint32_t flags;    // BF_* (check FAILED)
  uint32_t key;      // key-table index of A_i, or kNoKey
  uint32_t pad;
  uint32_t b[8];     // z_i s_i mod l
};

struct bv_chunk {
  uint64_t start;    // first item (global index)
  uint32_t batch;
  uint32_t count;
};

struct bv_chunk_out {
  ge P;              // partial sum (with T)
  uint32_t first[3]; // first failing item per class, relative to the batch start
  uint32_t pad;
};

enum : uint32_t { BF_S_HIGH = 1, BF_A_DECODE = 2, BF_S_NONCANON = 4, BF_R_DECODE = 8 };

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void load_btab(ge_niels* s_btab) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&g_bc.btab[0]);
  uint32_t* dst = reinterpret_cast<uint32_t*>(s_btab);
  for (int i = threadIdx.x; i < BT_WORDS; i += blockDim.x) dst[i] = src[i];
}

__device__ __forceinline__ void hram96(uint32_t x[16], const uint32_t R[8], const uint32_t A[8],
                                       const uint32_t M[8]) {
  uint64_t w[16], st[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = ((uint64_t)bswap(R[2 * i]) << 32) | bswap(R[2 * i + 1]);
    w[4 + i] = ((uint64_t)bswap(A[2 * i]) << 32) | bswap(A[2 * i + 1]);
    w[8 + i] = ((uint64_t)bswap(M[2 * i]) << 32) | bswap(M[2 * i + 1]);
  }
  w[12] = 0x8000000000000000ULL;
  w[13] = 0;
  w[14] = 0;
  w[15] = 96 * 8;
  sha512_init(st);
  sha512_compress(st, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x[2 * i] = bswap((uint32_t)(st[i] >> 32));
    x[2 * i + 1] = bswap((uint32_t)st[i]);
  }
}

// ------------------------------------------------------------------------------ plan
// Plan of a slice of batches [b0, b1), three passes of 1024-batch blocks (a decoupled
// block scan; one workgroup looping over a million batches took 3.3 ms):
//   k_bv_plan_local  per batch: chunk count k_b = ceil(n_b / C) (0 for an empty or a
//                    Pippenger batch), whether it needs k_bv_combine (k_b != 1, not
//                    Pippenger), whether it is a Pippenger batch; per-block totals.
//   k_bv_plan_top    one workgroup: exclusive scan of the block totals, and the slice's
//                    chunk total in chunk_start[nb].
//   k_bv_plan_apply  per batch: chunk_start (nb + 1 entries), the combine list (multi,
//                    multi_first) and the Pippenger list.
// k_bv_expand: one lane per chunk writes its descriptor (balanced split of the batch).
// Batches settled elsewhere (skip.group_ok[b / skip.per_group] != 0: their certificate
// group passed the merged check, launch_cert_groups) get no chunks and status Ok.
struct batch_skip_t {
  const uint32_t* group_ok;
  uint64_t per_group;
};
__device__ __forceinline__ bool skipped(const batch_skip_t& sk, uint64_t b) {
  return sk.group_ok && sk.group_ok[b / sk.per_group] != 0;
}

__device__ __forceinline__ void plan_counts(const uint64_t* offsets, uint64_t b, uint64_t b1,
                                            uint32_t C, uint32_t pmin, const batch_skip_t& sk,
                                            uint32_t& kb, uint32_t& mflag, uint32_t& pflag) {
  kb = 0;
  pflag = 0;
  if (b < b1 && skipped(sk, b)) {
    mflag = 0;
    return;
  }
  if (b < b1) {
    const uint64_t nb = offsets[b + 1] - offsets[b];
    pflag = nb >= pmin ? 1u : 0u;   // Pippenger batch: no chunks, no combine
    kb = pflag ? 0u : (uint32_t)((nb + C - 1) / C);
  }
  mflag = (b < b1 && !pflag && kb != 1) ? 1u : 0u;
}

// Inclusive Hillis-Steele scan of three counters over a 1024-thread block.
__device__ __forceinline__ void block_scan3(uint32_t v[3], uint32_t (*s)[1024]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k][t] = v[k];
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    uint32_t x[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) x[k] = t >= d ? s[k][t - d] : 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 3; ++k) s[k][t] += x[k];
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = s[k][t];
}

__global__ __launch_bounds__(1024) void k_bv_plan_local(const uint64_t* __restrict__ offsets,
                                                        uint64_t b0, uint64_t b1, uint32_t C,
                                                        uint32_t pmin, batch_skip_t sk,
                                                        uint32_t* __restrict__ tot) {
  __shared__ uint32_t s[3][1024];
  uint32_t v[3];
  plan_counts(offsets, b0 + (uint64_t)blockIdx.x * 1024 + threadIdx.x, b1, C, pmin, sk, v[0],
              v[1], v[2]);
  block_scan3(v, s);
  if (threadIdx.x == 1023) {
#pragma unroll
    for (int k = 0; k < 3; ++k) tot[3 * blockIdx.x + k] = v[k];
  }
}

// nblk <= 4096 (a slice has at most 4M batches): 4 blocks per thread.
__global__ __launch_bounds__(1024) void k_bv_plan_top(uint32_t nblk, uint64_t nb,
                                                      uint32_t* __restrict__ tot,
                                                      uint32_t* __restrict__ chunk_start) {
  __shared__ uint32_t s[3][1024];
  const uint32_t t = threadIdx.x;
  uint32_t loc[4][3], v[3] = {0, 0, 0};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t blk = 4 * t + j;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      loc[j][k] = blk < nblk ? tot[3 * blk + k] : 0u;
      v[k] += loc[j][k];
    }
  }
  uint32_t inc[3] = {v[0], v[1], v[2]};
  block_scan3(inc, s);
  uint32_t run[3] = {inc[0] - v[0], inc[1] - v[1], inc[2] - v[2]};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t blk = 4 * t + j;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (blk < nblk) tot[3 * blk + k] = run[k];
      run[k] += loc[j][k];
    }
  }
  if (t == 1023) {
    chunk_start[nb] = run[0];
#pragma unroll
    for (int k = 0; k < 3; ++k) tot[3 * nblk + k] = run[k];   // device totals
  }
}

__global__ __launch_bounds__(1024) void k_bv_plan_apply(const uint64_t* __restrict__ offsets,
                                                        uint64_t b0, uint64_t b1, uint32_t C,
                                                        uint32_t pmin, batch_skip_t sk,
                                                        const uint32_t* __restrict__ tot,
                                                        uint32_t* __restrict__ chunk_start,
                                                        uint32_t* __restrict__ multi,
                                                        uint32_t* __restrict__ multi_first,
                                                        uint32_t* __restrict__ pip_list,
                                                        int32_t* __restrict__ status,
                                                        uint64_t* __restrict__ fail_index) {
  __shared__ uint32_t s[3][1024];
  const uint64_t b = b0 + (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  uint32_t kb, mflag, pflag;
  plan_counts(offsets, b, b1, C, pmin, sk, kb, mflag, pflag);
  uint32_t v[3] = {kb, mflag, pflag};
  block_scan3(v, s);
  if (b >= b1) return;
  if (skipped(sk, b)) {
    status[b] = NW_OK;
    if (fail_index) fail_index[b] = offsets[b + 1] - offsets[b];
  }
  const uint32_t ca = tot[3 * blockIdx.x] + v[0] - kb, cb = tot[3 * blockIdx.x + 1] + v[1] - mflag,
                 cc = tot[3 * blockIdx.x + 2] + v[2] - pflag;
  chunk_start[b - b0] = ca;
  if (mflag) {
    multi[cb] = (uint32_t)(b - b0);
    multi_first[cb] = ca;
  }
  if (pflag) pip_list[cc] = (uint32_t)(b - b0);
}

__global__ __launch_bounds__(256) void k_bv_expand(const uint64_t* __restrict__ offsets,
                                                   uint64_t b0, uint64_t nb, uint32_t nchunks,
                                                   const uint32_t* __restrict__ chunk_start,
                                                   bv_chunk* __restrict__ chunks) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks || c >= chunk_start[nb]) return;   // host bound, device total
  // batch: largest lb with chunk_start[lb] <= c (empty batches share a start; the last
  // of them is the one that owns chunk c)
  uint64_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (chunk_start[mid] <= c) lo = mid; else hi = mid;
  }
  const uint64_t ob = offsets[b0 + lo], n = offsets[b0 + lo + 1] - ob;
  const uint32_t kb = chunk_start[lo + 1] - chunk_start[lo], k = c - chunk_start[lo];
  const uint64_t l = n * k / kb, h = n * (k + 1) / kb;
  bv_chunk ch;
  ch.start = ob + l;
  ch.batch = (uint32_t)lo;
  ch.count = (uint32_t)(h - l);
  chunks[c] = ch;
}

// ------------------------------------------------------------------------------ items
// Item gi (slot li = gi - i0) of batch lo: flags, scalars and the R (and A) tables.
__device__ __forceinline__ void bv_item_build(
    uint64_t gi, uint64_t li, uint64_t lo, const uint32_t* __restrict__ digests,
    const uint32_t* __restrict__ pks, const uint32_t* __restrict__ sigs,
    const uint32_t* __restrict__ z16, const z_key_t& zkey, bv_item* __restrict__ items,
    ge_cached* __restrict__ tabs, const key_tables_t& keys) {
  const curve_consts& K = g_bc.k;
  uint32_t Aw[8], Rw[8], Sw[8], Mw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    Aw[j] = pks[8 * gi + j];
    Rw[j] = sigs[16 * gi + j];
    Sw[j] = sigs[16 * gi + 8 + j];
    Mw[j] = digests[8 * lo + j];
  }
  uint32_t flags = 0;
  if ((Sw[7] >> 29) != 0) flags |= BF_S_HIGH;
  sc s;
#pragma unroll
  for (int j = 0; j < 8; ++j) s.w[j] = Sw[j];
  if (!sc_is_canonical(s)) flags |= BF_S_NONCANON;
  uint32_t hx[16];
  hram96(hx, Rw, Aw, Mw);
  sc k;
  sc_reduce512(k, hx);
  uint32_t zw[4];
  if (z16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) zw[j] = z16[4 * gi + j];
  } else {
    chacha20_z(zw, zkey.key, zkey.nonce, gi);
  }
  sc z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z.w[j] = j < 4 ? zw[j] : 0u;
  sc c, b;
  sc_mul(c, z, k);
  if (flags & (BF_S_HIGH | BF_S_NONCANON)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s.w[j] = 0;   // verdict is decided by the flags
  }
  sc_mul(b, z, s);
  const uint32_t kk = keys.vote_key ? keys.vote_key[gi] : kNoKey;
  bv_item it;
  sc_recode(it.c, c, kk != kNoKey ? 0x80808080u : 0x88888888u);
  it.key = kk;
  it.pad = 0;
  uint32_t zr[8];
  sc_recode(zr, z, 0x88888888u);
#pragma unroll
  for (int j = 0; j < 5; ++j) it.z[j] = zr[j];
#pragma unroll
  for (int j = 0; j < 8; ++j) it.b[j] = b.w[j];

  ge P;
  ge_cached* tA = tabs + 16 * li;
  // A: the caller's pre-decompressed key tables when this vote's key has them (read by
  // k_bv_chunks directly), else decompressed and tabulated here
  if (kk != kNoKey) {
    if (!(keys.ok[kk] & 1u)) flags |= BF_A_DECODE;
  } else if (!ge_frombytes(P, Aw, K)) {
    flags |= BF_A_DECODE;
  }
  it.flags = flags;   // (R decode flag added below)
  // tables j*P, j = 1..8 (cached form): A (unless keyed), then R
#pragma unroll 1
  for (int which = kk != kNoKey ? 1 : 0; which < 2; ++which) {
    if (which == 1) {
      if (!ge_frombytes(P, Rw, K)) flags |= BF_R_DECODE;
      tA = tabs + 16 * li + 8;
    }
    ge_cached c1;
    ge_to_cached(c1, P, K.d2);
    tA[0] = c1;
    ge acc;
    ge_dbl(acc, P, true);
    ge_cached cj;
    ge_to_cached(cj, acc, K.d2);
    tA[1] = cj;
#pragma unroll 1
    for (int j = 3; j <= 8; ++j) {
      ge_add_cached(acc, acc, c1, true);
      ge_to_cached(cj, acc, K.d2);
      tA[j - 1] = cj;
    }
  }
  it.flags = flags;
  items[li] = it;
}

__global__ __launch_bounds__(256) void k_bv_items(
    const uint32_t* __restrict__ digests, const uint64_t* __restrict__ offsets, uint64_t b0,
    uint64_t b1, uint64_t i0, uint64_t i1, uint32_t pmin, const uint32_t* __restrict__ pks,
    const uint32_t* __restrict__ sigs, const uint32_t* __restrict__ z16, z_key_t zkey,
    bv_item* __restrict__ items, ge_cached* __restrict__ tabs, key_tables_t keys,
    batch_skip_t sk) {
  const uint64_t gi = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= i1) return;
  // batch of this item: largest b in [b0, b1) with offsets[b] <= gi
  uint64_t lo = b0, hi = b1;
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= gi) lo = mid; else hi = mid;
  }
  if (offsets[lo + 1] - offsets[lo] >= pmin) return;   // k_pip_points
  if (skipped(sk, lo)) return;
  bv_item_build(gi, gi - i0, lo, digests, pks, sigs, z16, zkey, items, tabs, keys);
}

// The same items driven by the chunk list (k_bv_expand): lane = chunk * C + j. When a skip
// list leaves only a few scattered batches to run (launch_votes_keyed's failed
// certificates), a lane per vote would leave most waves with one or two live lanes each
// paying a whole decompression and table build; here the live items are dense.
__global__ __launch_bounds__(256) void k_bv_items_chunked(
    const bv_chunk* __restrict__ chunks, uint32_t nchunks, const uint32_t* __restrict__ ctotal,
    uint32_t C, const uint32_t* __restrict__ digests, uint64_t b0, uint64_t i0,
    const uint32_t* __restrict__ pks, const uint32_t* __restrict__ sigs,
    const uint32_t* __restrict__ z16, z_key_t zkey, bv_item* __restrict__ items,
    ge_cached* __restrict__ tabs, key_tables_t keys) {
  const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t ci = l / C, j = l % C;
  if (ci >= nchunks || ci >= *ctotal) return;   // host bound, device total
  const bv_chunk ch = chunks[ci];
  if (j >= ch.count) return;
  const uint64_t gi = ch.start + j;
  bv_item_build(gi, gi - i0, b0 + ch.batch, digests, pks, sigs, z16, zkey, items, tabs, keys);
}

// ------------------------------------------------------------------------------ chunks
__device__ __forceinline__ int digit4(uint32_t word, int j) {
  return (int)((word >> ((j & 7) * 4)) & 15u) - 8;
}

__device__ __forceinline__ void add_entry(ge& acc, const ge_cached* tab, int d) {
  if (d != 0) {
    const int ad = d < 0 ? -d : d;
    ge_cached e = tab[ad - 1];
    ge_cached_cneg(e, d < 0);
    ge_add_cached(acc, acc, e, true);
  }
}

// Status of a batch from its first failures (reference order, crypto/src/lib.rs:214-218
// then dalek: parse / decompress A (fail fast), check_scalar, decompress R) or the sum.
__device__ __forceinline__ int batch_status(const uint32_t first[3], uint32_t flags0,
                                            bool identity, uint64_t n, uint64_t* idx) {
  if (first[0] != kNone) {
    *idx = first[0];
    return (flags0 & BF_S_HIGH) ? NW_ERR_S_HIGH_BITS : NW_ERR_A_DECODE;
  }
  if (first[1] != kNone) { *idx = first[1]; return NW_ERR_S_NONCANONICAL; }
  if (first[2] != kNone) { *idx = first[2]; return NW_ERR_R_DECODE; }
  *idx = n;
  return identity ? NW_OK : NW_ERR_EQUATION;
}

__device__ __forceinline__ int wave_max_int(int w) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int x = __shfl_xor(w, o);
    w = x > w ? x : w;
  }
  return __builtin_amdgcn_readfirstlane(w);
}

// Signed 8-bit digit m (0..31) of a 256-bit value recoded with + 0x80..80.
__device__ __forceinline__ int digit8(const uint32_t* w, int m) {
  return (int)((sel8(w, m >> 2) >> ((m & 3) * 8)) & 255u) - 128;
}

// Keyed vote: A's digit from its key table (129 entries j*A or j*2^128 A, affine niels:
// a mixed addition).
__device__ __forceinline__ void add_key_entry(ge& acc, const ge_niels_pad* tab129, int d) {
  if (d != 0) {
    ge_niels nb = tab129[d < 0 ? -d : d].n;
    ge_niels_cneg(nb, d < 0);
    ge_add_niels(acc, acc, nb, true);
  }
}

// One lane per chunk: the Straus ladder shared by the chunk's votes and B.
//   unkeyed chunk: 64 windows of 4 bits (252 doublings); c_i by 4-bit digits over the vote's
//     own j*A_i table, z_i by 4-bit digits over j*R_i, -sum b by 8-bit digits over j*B;
//   keyed chunk (every A_i has caller key tables j*A, j*2^128 A): 33 windows (128
//     doublings); c_i = c_lo + 2^128 c_hi by 8-bit digits over the two key tables, z_i as
//     before, -sum b = b_lo + 2^128 b_hi by 8-bit digits over j*B and j*2^128 B.
// A lane whose chunk is keyed simply has no digits above window 32 when the wave runs the
// long ladder for another lane (the identity doubles to itself).
__global__ __launch_bounds__(256) void k_bv_chunks(
    const bv_chunk* __restrict__ chunks, uint32_t nchunks, const uint64_t* __restrict__ offsets,
    uint64_t b0, uint64_t i0, const bv_item* __restrict__ items,
    const ge_cached* __restrict__ tabs, const ge_niels_pad* __restrict__ ktabs, keyspec ks,
    bv_chunk_out* __restrict__ out, int32_t* __restrict__ status,
    uint64_t* __restrict__ fail_index, const uint32_t* __restrict__ ctotal) {
  __shared__ ge_niels s_btab[129];
  __shared__ ge_niels s_b128[129];
  const uint32_t ci = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nch = min(nchunks, *ctotal);   // host bound, device total
  // a workgroup with no live chunk leaves before filling its 31 KB of LDS tables (the
  // certificate path launches for every certificate and runs only the failed ones)
  if (blockIdx.x * blockDim.x >= nch) return;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&g_bc.btab[0]);
    const uint32_t* src2 = reinterpret_cast<const uint32_t*>(&g_bc.b128[0]);
    uint32_t* dst = reinterpret_cast<uint32_t*>(s_btab);
    uint32_t* dst2 = reinterpret_cast<uint32_t*>(s_b128);
    for (int i = threadIdx.x; i < BT_WORDS; i += blockDim.x) {
      dst[i] = src[i];
      dst2[i] = src2[i];
    }
  }
  __syncthreads();
  const bool live = ci < nch;
  const bv_chunk ch = chunks[live ? ci : nch - 1];
  const uint64_t bidx = b0 + ch.batch;
  const uint64_t bstart = offsets[bidx];
  const uint64_t bn = offsets[bidx + 1] - bstart;
  const uint64_t l0 = ch.start - i0;
  // first failures, sum of b_i over the chunk, and whether every vote is keyed
  uint32_t first[3] = {kNone, kNone, kNone};
  uint32_t flags0 = 0;
  bool keyed = ktabs != nullptr;
  sc bsum;
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum.w[j] = 0;
  for (uint32_t t = 0; t < ch.count; ++t) {
    const bv_item* it = items + l0 + t;
    const uint32_t f = it->flags;
    const uint32_t rel = (uint32_t)(ch.start + t - bstart);
    if ((f & (BF_S_HIGH | BF_A_DECODE)) && first[0] == kNone) { first[0] = rel; flags0 = f; }
    if ((f & BF_S_NONCANON) && first[1] == kNone) first[1] = rel;
    if ((f & BF_R_DECODE) && first[2] == kNone) first[2] = rel;
    keyed &= it->key != kNone;
    sc bi;
#pragma unroll
    for (int j = 0; j < 8; ++j) bi.w[j] = it->b[j];
    sc_add(bsum, bsum, bi);
  }
  sc nb;
  sc_neg(nb, bsum);
  uint32_t bb[8];
  sc_recode(bb, nb, 0x80808080u);
  // an unkeyed chunk among keyed ones cannot read key tables; a keyed one needs no
  // 4-bit A digits (its c words hold 8-bit digits)
  const int W = wave_max_int(live ? (keyed ? 33 : 64) : 0);

  ge acc;
  ge_identity(acc);
#pragma unroll 1
  for (int j = W - 1; j >= 0; --j) {
    if (j != W - 1) {
#pragma unroll 1
      for (int t = 0; t < 3; ++t) ge_dbl(acc, acc, false);
      ge_dbl(acc, acc, true);
    }
    if (!live) continue;
#pragma unroll 1
    for (uint32_t t = 0; t < ch.count; ++t) {
      const bv_item* it = items + l0 + t;
      const ge_cached* tab = tabs + 16 * (l0 + t);
      if (keyed) {
        if ((j & 1) == 0 && j < 32) {
          const ge_niels_pad* kt = ktabs + ks.tab * (uint64_t)it->key;
          add_key_entry(acc, kt, digit8(it->c, j >> 1));
          add_key_entry(acc, kt + ks.half, digit8(it->c, 16 + (j >> 1)));
        }
      } else {
        add_entry(acc, tab, digit4(it->c[j >> 3], j));
      }
      if (j <= 32) add_entry(acc, tab + 8, digit4(it->z[j >> 3], j));
    }
    if ((j & 1) == 0) {
      if (keyed) {
        if (j < 32) {
          add_digit_niels(acc, s_btab, digit8(bb, j >> 1), true);
          add_digit_niels(acc, s_b128, digit8(bb, 16 + (j >> 1)), true);
        }
      } else {
        add_digit_niels(acc, s_btab, digit8(bb, j >> 1), true);
      }
    }
  }
  if (!live) return;
  if (ch.count == bn) {   // the batch is this one chunk: finish it here
    uint64_t idx;
    const int st = batch_status(first, flags0, ge_is_identity(acc), bn, &idx);
    status[bidx] = st;
    if (fail_index) fail_index[bidx] = idx;
  } else {
    bv_chunk_out o;
    o.P = acc;
    o.first[0] = first[0];
    o.first[1] = first[1];
    o.first[2] = first[2];
    o.pad = flags0;
    out[ci] = o;
  }
}

// ------------------------------------------------------------------------------ combine
// One 256-thread workgroup per listed batch (k_b == 0 or >= 2): threads sum a strided
// subset of the chunk points, then a tree through LDS. The grid is bounded
// (kCombineMaxBlocks) and strides over the device's count of listed batches: the host only
// knows an upper bound (every certificate of a group, 10^6 at N = 4), and a workgroup per
// bound that exits at once cost 0.24 ms per config-2 call.
constexpr uint32_t kCombineMaxBlocks = 2048;
__global__ __launch_bounds__(256) void k_bv_combine(const uint32_t* __restrict__ multi,
                                                    const uint32_t* __restrict__ multi_first,
                                                    uint32_t nmulti, const uint64_t* __restrict__ offsets,
                                                    uint64_t b0, uint32_t C,
                                                    const bv_chunk_out* __restrict__ out,
                                                    int32_t* __restrict__ status,
                                                    uint64_t* __restrict__ fail_index,
                                                    const uint32_t* __restrict__ mtotal) {
  __shared__ ge s_p[256];
  __shared__ uint32_t s_f[256][4];
  const uint32_t mt = *mtotal, mend = mt < nmulti ? mt : nmulti;   // device total, host bound
  const int tid = threadIdx.x;
  for (uint32_t m = blockIdx.x; m < mend; m += gridDim.x) {
    const uint64_t bidx = b0 + multi[m];
    const uint64_t bn = offsets[bidx + 1] - offsets[bidx];
    const uint32_t kb = (uint32_t)((bn + C - 1) / C);
    const uint32_t c0 = multi_first[m];
    const curve_consts& K = g_bc.k;
    ge acc;
    ge_identity(acc);
    uint32_t f[3] = {kNone, kNone, kNone};
    uint32_t flags0 = 0;
    for (uint32_t k = tid; k < kb; k += 256) {
      const bv_chunk_out& o = out[c0 + k];
      ge_cached c;
      ge_to_cached(c, o.P, K.d2);
      ge_add_cached(acc, acc, c, true);
      if (o.first[0] < f[0]) { f[0] = o.first[0]; flags0 = o.pad; }
      f[1] = min(f[1], o.first[1]);
      f[2] = min(f[2], o.first[2]);
    }
    s_p[tid] = acc;
    s_f[tid][0] = f[0]; s_f[tid][1] = f[1]; s_f[tid][2] = f[2]; s_f[tid][3] = flags0;
    __syncthreads();
    for (int stride = 128; stride > 0; stride >>= 1) {
      if (tid < stride && (uint32_t)(tid + stride) < kb) {
        ge_cached c;
        ge_to_cached(c, s_p[tid + stride], K.d2);
        ge t;
        ge_add_cached(t, s_p[tid], c, true);
        s_p[tid] = t;
        if (s_f[tid + stride][0] < s_f[tid][0]) {
          s_f[tid][0] = s_f[tid + stride][0];
          s_f[tid][3] = s_f[tid + stride][3];
        }
        s_f[tid][1] = min(s_f[tid][1], s_f[tid + stride][1]);
        s_f[tid][2] = min(s_f[tid][2], s_f[tid + stride][2]);
      }
      __syncthreads();
    }
    if (tid == 0) {
      uint64_t idx = 0;
      int st = NW_OK;
      if (bn > 0) {
        const uint32_t ff[3] = {s_f[0][0], s_f[0][1], s_f[0][2]};
        st = batch_status(ff, s_f[0][3], ge_is_identity(s_p[0]), bn, &idx);
      }
      status[bidx] = st;
      if (fail_index) fail_index[bidx] = idx;
    }
    __syncthreads();   // slot 0 read before the next batch's sums overwrite it
  }
}

// ------------------------------------------------------------------------------ Pippenger
// Large batches (n >= NW_BATCH_PIPPENGER_MIN votes, default kPipMin): a bucket
// multi-scalar multiplication over all 2n points of the batch, spread over the whole chip
// instead of one Straus ladder per chunk lane.
//
//   sum_i z_i R_i + sum_i c_i A_i = sum_{w<32} 2^(8w) sum_{b=1..128} b S_{w,b}
//
// with signed 8-bit digits (c_i: 32 windows, z_i: 17) and S_{w,b} = the sum of the points
// whose window-w digit is +-b (sign applied to the point). A vote costs two decompressions
// and <= 49 bucket additions; the per-batch tail (bucket sums, window sums, 248-doubling
// Horner over the windows with -sum b_i folded in by 8-bit windows over the LDS B table) is
// shared by the whole batch.
//
//   k_pip_points   one lane per point (A lanes also do the vote's scalars and flags),
//                  decompressed points written in affine niels form
//   k_pip_sort     one workgroup per (batch, window): counting sort of the window's digits
//                  into its buckets with LDS histograms and cursors ((point index | sign)
//                  entries; the order inside a bucket does not matter, addition commutes);
//                  one more workgroup per batch: sum b_i and the first failures
//   k_pip_buckets  G lanes per bucket: partial sums, combined by a lane-shuffle tree
//   k_pip_windows  one wave per window: sum_b b S_b by a suffix scan + tree over lanes;
//                  one more wave per batch: [-sum b_i]B from the comb tables (no doublings)
//   k_pip_final    one wave per batch: the 248-doubling Horner over the window sums,
//                  limb-parallel (nw_lp.hpp), identity test, status
//
// Each batch's scratch lives in the per-item table slots of its own items (16 cached
// entries = 2560 B per item, unused by this path): pip_region() lays it out.
constexpr uint32_t kPipMin = 512;
constexpr uint32_t kPipFloor = 400;     // smallest n whose item slots hold the region
constexpr int kPipWin = 32;             // 8-bit windows of c_i (< 2^253)
constexpr int kPipZWin = 17;            // 8-bit windows of z_i (< 2^128, recoded)
// Bins: window w, |digit| b -> w * 128 + b - 1, except the two windows whose digits are
// structurally skewed, which are spread over sub-bins so no bucket is much longer than the
// mean (bucket sums are sequential chains):
//   c_i window 31: c < l gives digit (c >> 248) + carry in [0, 17]; digit d of vote t goes
//     to 31 * 128 + (d - 1) + 17 (t % 7) (weight (j % 17) + 1 for bucket j of window 31);
//   z_i window 16: the recoding carry, digit 0 or 1 for every vote (about n/2 ones); vote t
//     goes to kPipWin * 128 + (t % 64), weight 1 at window 16.
constexpr int kPipWinCap = 2 * kPipWin;   // entry slots per vote: 2 per window
constexpr int kPipTopSub = 7, kPipTopStride = 17, kPipCarryBins = 64;
constexpr int kPipBins = kPipWin * 128 + kPipCarryBins;

struct pip_region {
  ge_niels_pad* pts; // 2n: A_t at 2t, R_t at 2t + 1 (one 128-byte line each: a bucket
                     // lane's gather of a 120-byte entry at a 120-byte stride fetched two)
  uint32_t* ent;     // window w: entries [2n w, 2n w + 2n), point index | sign << 31
  uint8_t* cd;       // 32 x n, window-major: byte w of recoded c_t at cd[w n + t]
  uint8_t* zd;       // 17 x n (+ pad): byte w of recoded z_t at zd[w n + t]
  uint32_t* cnt;     // kPipBins: entries per bucket
  uint32_t* off;     // kPipBins: first entry of each bucket
  ge* S;             // kPipBins bucket sums
  ge_cached* W;      // kPipWin window sums (cached form, for the Horner)
  uint32_t* hdr;     // first failures (3) and their flags (k_pip_sort's extra block)
  uint32_t* bb;      // -sum b_i, recoded to signed 8-bit digits (k_pip_sort's extra block)
  ge_cached* Bc;     // [-sum b_i]B (k_pip_windows' extra block), added after the Horner
};

constexpr size_t pip_region_bytes(uint64_t n) {
  return 2 * n * sizeof(ge_niels_pad) + 4 * kPipWinCap * n + 52 * n + 8 * kPipBins +
         sizeof(ge) * kPipBins + sizeof(ge_cached) * kPipWin + 16 + 32 + sizeof(ge_cached);
}
// per-vote bytes grow slower than the item slots (2560 B), so the floor is the binding n
static_assert(pip_region_bytes(kPipFloor) <= 16 * sizeof(ge_cached) * kPipFloor,
              "Pippenger region does not fit its items' table slots");
// certificate groups: >= kPipMin votes plus up to 256 committee keys
static_assert(pip_region_bytes(kPipMin + 256) <= 16 * sizeof(ge_cached) * kPipMin,
              "certificate-group region does not fit its votes' table slots");

// Certificate-group mode (launch_cert_groups): a "batch" is a group of whole certificates;
// each vote hashes its own certificate's digest, votes of certificates that already failed
// (pre-checks, header) contribute nothing, and the A terms are not bucketed per vote: every
// vote's A is a committee key, so c_i is summed per key (k_grp_keys) and the nkeys keys
// enter as extra "votes" t = n + j with the digits of their sums only.
struct pip_group_t {
  const uint64_t* cert_vote_offsets;   // ncert + 1 (device); null: plain batches
  uint64_t ncert, certs_per_group;
  const int32_t* pre1;
  const int32_t* pre2;
  const int32_t* hdr_st;
  const uint32_t* vote_key;
  const uint32_t* key_ok;
  const ge* key_base;                  // key j decompressed at key_base[2 j] (Z = 1)
  uint32_t nkeys;
  uint32_t* group_ok;                  // 1: the group's merged equation holds, no flags
};

__device__ __forceinline__ pip_region pip_at(ge_cached* tabs, uint64_t li0, uint64_t n) {
  char* p = reinterpret_cast<char*>(tabs + 16 * li0);
  pip_region r;
  r.pts = reinterpret_cast<ge_niels_pad*>(p); p += 2 * n * sizeof(ge_niels_pad);
  r.ent = reinterpret_cast<uint32_t*>(p); p += 4 * kPipWinCap * n;
  r.cd = reinterpret_cast<uint8_t*>(p); p += 32 * n;
  r.zd = reinterpret_cast<uint8_t*>(p); p += 20 * n;
  r.cnt = reinterpret_cast<uint32_t*>(p); p += 4 * kPipBins;
  r.off = reinterpret_cast<uint32_t*>(p); p += 4 * kPipBins;
  r.S = reinterpret_cast<ge*>(p); p += sizeof(ge) * kPipBins;
  r.W = reinterpret_cast<ge_cached*>(p); p += sizeof(ge_cached) * kPipWin;
  r.Bc = reinterpret_cast<ge_cached*>(p); p += sizeof(ge_cached);
  r.hdr = reinterpret_cast<uint32_t*>(p); p += 16;
  r.bb = reinterpret_cast<uint32_t*>(p);
  return r;
}

__device__ __forceinline__ uint64_t batch_of(const uint64_t* offsets, uint64_t b0, uint64_t b1,
                                             uint64_t gi) {
  uint64_t lo = b0, hi = b1;
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= gi) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void ge_to_niels_z1(ge_niels& q, const ge& P, const fe& d2) {
  fe_add(q.ypx, P.Y, P.X); fe_carry(q.ypx);
  fe_sub(q.ymx, P.Y, P.X);
  fe_mul(q.xy2d, P.T, d2);
}

// r = p + q for two extended points (q converted to cached form), with T.
__device__ __forceinline__ void ge_add_ge(ge& r, const ge& p, const ge& q, const fe& d2) {
  ge_cached c;
  ge_to_cached(c, q, d2);
  ge_add_cached(r, p, c, true);
}

__device__ __forceinline__ void ge_shfl(ge& r, const ge& p, int src) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.X.v[i] = (uint32_t)__shfl((int)p.X.v[i], src);
    r.Y.v[i] = (uint32_t)__shfl((int)p.Y.v[i], src);
    r.Z.v[i] = (uint32_t)__shfl((int)p.Z.v[i], src);
    r.T.v[i] = (uint32_t)__shfl((int)p.T.v[i], src);
  }
}

// Lane -> (item, role): consecutive waves take the roles of 64 votes in turn, so a wave
// never mixes two: role 0 = the vote's scalars (SHA-512 k, z, c, b, digits, parse flags;
// in group mode also the committee-key lookup), role 1 = decompress R, role 2 (plain
// batches only: in group mode A is a committee key) = decompress A. Three short chains
// instead of one lane doing the scalars and A's decompression in series (the one-call
// latency of config 1 is this kernel's longest lane).
__device__ __forceinline__ void pip_point_do(
    int which, uint64_t li, const uint32_t* __restrict__ digests,
    const uint64_t* __restrict__ offsets, uint64_t b0, uint64_t b1, uint64_t i0, uint64_t i1,
    uint32_t pmin, const uint32_t* __restrict__ pks, const uint32_t* __restrict__ sigs,
    const uint32_t* __restrict__ z16, const z_key_t& zkey, bv_item* __restrict__ items,
    ge_cached* __restrict__ tabs, const pip_group_t& grp) {
  const uint64_t gi = i0 + li;
  if (gi >= i1) return;
  const uint64_t lo = batch_of(offsets, b0, b1, gi);
  const uint64_t bs = offsets[lo], n = offsets[lo + 1] - bs;
  if (n < pmin) return;
  const uint64_t t = gi - bs;
  const bool group = grp.cert_vote_offsets != nullptr;
  const uint64_t nreg = n + (group ? grp.nkeys : 0);   // + key sums
  const pip_region reg = pip_at(tabs, bs - i0, nreg);
  const curve_consts& K = g_bc.k;
  bv_item* it = items + li;
  uint64_t dig = lo;   // digest index: the batch, or in group mode the vote's certificate
  if (group) {
    const uint64_t c0 = lo * grp.certs_per_group;
    const uint64_t c1 = c0 + grp.certs_per_group < grp.ncert ? c0 + grp.certs_per_group : grp.ncert;
    dig = batch_of(grp.cert_vote_offsets, c0, c1, gi);
    if (grp.pre1[dig] != 0 || grp.hdr_st[dig] != 0 || grp.pre2[dig] != 0) {
      // decided before the votes: contributes nothing
      if (which == 1) {
        it->pad = 0;
      } else if (which == 0) {
        it->z[0] = 0;
#pragma unroll
        for (int w = 0; w < kPipWin; ++w) reg.cd[w * nreg + t] = 0x80;
#pragma unroll
        for (int w = 0; w < kPipZWin; ++w) reg.zd[w * nreg + t] = 0x80;
#pragma unroll
        for (int j = 0; j < 8; ++j) it->b[j] = 0;
        it->flags = 0;
        it->key = kNone;
      }
      return;
    }
  }
  if (which != 0) {   // decompress R (role 1) or A (role 2) into the region
    uint32_t w8[8];
    const uint32_t* src = which == 1 ? sigs + 16 * gi : pks + 8 * gi;
#pragma unroll
    for (int j = 0; j < 8; ++j) w8[j] = src[j];
    ge P;
    ge_niels q;
    const bool ok = ge_frombytes(P, w8, K);
    ge_to_niels_z1(q, P, K.d2);
    if (which == 1) {
      it->pad = ok ? 0u : (uint32_t)BF_R_DECODE;
      reg.pts[2 * t + 1].n = q;
    } else {
      it->z[0] = ok ? 0u : (uint32_t)BF_A_DECODE;   // Pippenger batches: z[] is unused
      reg.pts[2 * t].n = q;
    }
    return;
  }
  uint32_t Aw[8], Rw[8], Sw[8], Mw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    Aw[j] = pks[8 * gi + j];
    Rw[j] = sigs[16 * gi + j];
    Sw[j] = sigs[16 * gi + 8 + j];
    Mw[j] = digests[8 * dig + j];
  }
  uint32_t flags = 0;
  if ((Sw[7] >> 29) != 0) flags |= BF_S_HIGH;
  sc s;
#pragma unroll
  for (int j = 0; j < 8; ++j) s.w[j] = Sw[j];
  if (!sc_is_canonical(s)) flags |= BF_S_NONCANON;
  uint32_t hx[16];
  hram96(hx, Rw, Aw, Mw);
  sc k;
  sc_reduce512(k, hx);
  uint32_t zw[4];
  if (z16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) zw[j] = z16[4 * gi + j];
  } else {
    chacha20_z(zw, zkey.key, zkey.nonce, gi);
  }
  sc z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z.w[j] = j < 4 ? zw[j] : 0u;
  sc c, b;
  sc_mul(c, z, k);
  if (flags & (BF_S_HIGH | BF_S_NONCANON)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s.w[j] = 0;   // verdict is decided by the flags
  }
  sc_mul(b, z, s);
  uint32_t cr[8], zr[8];
  sc_recode(cr, c, 0x80808080u);
  sc_recode(zr, z, 0x80808080u);
  uint32_t key = kNone;
  if (group) {
    // A = committee key: c_i goes to the key's sum (k_grp_keys), no per-vote A digits
    key = grp.vote_key[gi];
    if (key == kNone || !(grp.key_ok[key] & 1u)) {
      flags |= BF_A_DECODE;
      key = kNone;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      it->c[j] = c.w[j];
      cr[j] = 0x80808080u;
    }
    it->z[0] = 0;   // no A lane in group mode
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) it->b[j] = b.w[j];
#pragma unroll
  for (int w = 0; w < kPipWin; ++w) reg.cd[w * nreg + t] = (uint8_t)(cr[w >> 2] >> ((w & 3) * 8));
#pragma unroll
  for (int w = 0; w < kPipZWin; ++w) reg.zd[w * nreg + t] = (uint8_t)(zr[w >> 2] >> ((w & 3) * 8));
  it->flags = flags;
  it->key = key;
}

__global__ __launch_bounds__(256, 3) void k_pip_points(
    const uint32_t* __restrict__ digests, const uint64_t* __restrict__ offsets, uint64_t b0,
    uint64_t b1, uint64_t i0, uint64_t i1, uint32_t pmin, const uint32_t* __restrict__ pks,
    const uint32_t* __restrict__ sigs, const uint32_t* __restrict__ z16, z_key_t zkey,
    bv_item* __restrict__ items, ge_cached* __restrict__ tabs, pip_group_t grp,
    uint32_t roles, uint32_t role0) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, wave = g >> 6;
  pip_point_do((int)(role0 + wave % roles), (wave / roles) * 64 + (g & 63), digests, offsets, b0,
               b1, i0, i1, pmin, pks, sigs, z16, zkey, items, tabs, grp);
}

// Group mode: per group, sum_i c_i per committee key (LDS, 64-bit limb sums), reduced mod l,
// as the digits of the key "votes" t = n + j, whose A point is the decompressed key.
__global__ __launch_bounds__(1024) void k_grp_keys(const uint64_t* __restrict__ offsets,
                                                   uint64_t b0, uint64_t i0, uint32_t pmin,
                                                   const bv_item* __restrict__ items,
                                                   ge_cached* __restrict__ tabs, pip_group_t grp) {
  __shared__ unsigned long long s_acc[256][8];
  const uint64_t bidx = b0 + blockIdx.x;
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  if (n < pmin) return;
  const uint32_t N = grp.nkeys;
  const uint64_t nreg = n + N;   // votes, key sums
  const pip_region reg = pip_at(tabs, bs - i0, nreg);
  const int tid = threadIdx.x;
  for (int k = tid; k < 256 * 8; k += 1024) s_acc[k >> 3][k & 7] = 0;
  __syncthreads();
  const bv_item* its = items + (bs - i0);
  for (uint64_t t = tid; t < n; t += 1024) {
    const uint32_t key = its[t].key;
    if (key != kNone) {
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(&s_acc[key][j], (unsigned long long)its[t].c[j]);
    }
  }
  __syncthreads();
  for (uint32_t j = tid; j < N; j += 1024) {
    uint32_t x[16];
    unsigned long long carry = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      carry += s_acc[j][w];
      x[w] = (uint32_t)carry;
      carry >>= 32;
    }
    x[8] = (uint32_t)carry;
    x[9] = (uint32_t)(carry >> 32);
#pragma unroll
    for (int w = 10; w < 16; ++w) x[w] = 0;
    sc C;
    sc_reduce512(C, x);
    uint32_t cr[8];
    sc_recode(cr, C, 0x80808080u);
    const uint64_t t = n + j;
#pragma unroll
    for (int w = 0; w < kPipWin; ++w) reg.cd[w * nreg + t] = (uint8_t)(cr[w >> 2] >> ((w & 3) * 8));
#pragma unroll
    for (int w = 0; w < kPipZWin; ++w) reg.zd[w * nreg + t] = 0x80;
    ge_niels q;
    ge_to_niels_z1(q, grp.key_base[2 * j], g_bc.k.d2);
    reg.pts[2 * t].n = q;
  }
}

// The extra block of k_pip_sort (1024 threads): sum_i b_i and the first failures (in the
// reference's order) over the batch's votes; -sum b_i recoded into reg.bb for the comb in
// k_pip_windows' extra block (off the Horner's critical path).
// Scalar sum a += b mod l and first-failure merge across lanes (xor shuffles).
__device__ __forceinline__ void bsum_merge(sc& a, uint32_t f[4], int o) {
  sc b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b.w[j] = (uint32_t)__shfl_xor((int)a.w[j], o);
  sc_add(a, a, b);
  const uint32_t g0 = (uint32_t)__shfl_xor((int)f[0], o), g3 = (uint32_t)__shfl_xor((int)f[3], o);
  const uint32_t g1 = (uint32_t)__shfl_xor((int)f[1], o), g2 = (uint32_t)__shfl_xor((int)f[2], o);
  if (g0 < f[0]) { f[0] = g0; f[3] = g3; }
  f[1] = min(f[1], g1);
  f[2] = min(f[2], g2);
}

template <int NT>
__device__ __forceinline__ void pip_bsum_block(const pip_region& reg, uint64_t n,
                                               const bv_item* __restrict__ its,
                                               uint32_t (*s_b)[8], uint32_t (*s_f)[4]) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  sc bsum;
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum.w[j] = 0;
  uint32_t f[4] = {kNone, kNone, kNone, 0};
  for (uint64_t t = tid; t < n; t += NT) {
    const uint32_t fl = its[t].flags | its[t].pad | its[t].z[0];   // scalar, R and A lanes
    if ((fl & (BF_S_HIGH | BF_A_DECODE)) && f[0] == kNone) { f[0] = (uint32_t)t; f[3] = fl; }
    if ((fl & BF_S_NONCANON) && f[1] == kNone) f[1] = (uint32_t)t;
    if ((fl & BF_R_DECODE) && f[2] == kNone) f[2] = (uint32_t)t;
    sc bi;
#pragma unroll
    for (int j = 0; j < 8; ++j) bi.w[j] = its[t].b[j];
    sc_add(bsum, bsum, bi);
  }
#pragma unroll 1
  for (int o = 32; o > 0; o >>= 1) bsum_merge(bsum, f, o);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s_b[wv][j] = bsum.w[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) s_f[wv][j] = f[j];
  }
  __syncthreads();
  if (wv != 0) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum.w[j] = lane < NW ? s_b[lane][j] : 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) f[j] = lane < NW ? s_f[lane][j] : (j < 3 ? kNone : 0u);
#pragma unroll 1
  for (int o = NW / 2; o > 0; o >>= 1) bsum_merge(bsum, f, o);
  if (lane != 0) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) reg.hdr[j] = f[j];
  sc nb;
  sc_neg(nb, bsum);
  uint32_t bb[8];
  sc_recode(bb, nb, 0x80808080u);
#pragma unroll
  for (int j = 0; j < 8; ++j) reg.bb[j] = bb[j];
}

// The nonzero digits of every vote t < n in window w (c_i and, for w <= 16, z_i) as
// f(local bin, point index, negative), on a workgroup of NT threads; local bins 0..127 are
// buckets w * 128 + j, and in window 16 local bins 128..191 are the z-carry sub-bins. The
// digit bytes of 8 votes are loaded before their callbacks (the LDS atomics would otherwise
// wait out each load's latency in turn).
template <int NT, typename F>
__device__ __forceinline__ void pip_digits_pass(const pip_region& reg, uint64_t n, int w, F&& f) {
  constexpr int U = 8;
  for (uint64_t t0 = threadIdx.x; t0 < n; t0 += (uint64_t)NT * U) {
    int dc[U], dz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t t = t0 + (uint64_t)u * NT;
      dc[u] = t < n ? (int)reg.cd[w * n + t] - 128 : 0;
      dz[u] = (w < kPipZWin && t < n) ? (int)reg.zd[w * n + t] - 128 : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t t = t0 + (uint64_t)u * NT;
      if (dc[u] != 0) {
        const uint32_t ad = (uint32_t)(dc[u] < 0 ? -dc[u] : dc[u]);
        const uint32_t lb = w == kPipWin - 1 ? (uint32_t)(kPipTopStride * (t % kPipTopSub)) + ad - 1
                                             : ad - 1;
        f(lb, (uint32_t)(2 * t), dc[u] < 0);
      }
      if (dz[u] != 0) {
        const uint32_t ad = (uint32_t)(dz[u] < 0 ? -dz[u] : dz[u]);
        const uint32_t lb = w == kPipZWin - 1 ? (uint32_t)(128 + (t % kPipCarryBins)) : ad - 1;
        f(lb, (uint32_t)(2 * t + 1), dz[u] < 0);
      }
    }
  }
}

// Window w's counting sort on one workgroup of NT threads: histogram of the window's digits
// in LDS, scan, then scatter with LDS cursors into the window's entry range (capacity 2n).
constexpr int kPipSortBins = 128 + kPipCarryBins;
template <int NT>
__device__ __forceinline__ void pip_sort_window(const pip_region& reg, uint64_t n, int w,
                                                uint32_t* s_h, uint32_t* s_c) {
  constexpr int NL = kPipSortBins;
  static_assert(NT >= NL, "one thread per local bin");
  const int tid = threadIdx.x;
  if (tid < NL) s_h[tid] = 0;
  __syncthreads();
  pip_digits_pass<NT>(reg, n, w, [&](uint32_t lb, uint32_t, bool) { atomicAdd(&s_h[lb], 1u); });
  __syncthreads();
  // inclusive Hillis-Steele scan over the NL local bins (threads < NL)
  uint32_t v = tid < NL ? s_h[tid] : 0u;
  if (tid < NL) s_c[tid] = v;
  __syncthreads();
  for (int d = 1; d < NL; d <<= 1) {
    const uint32_t x = (tid < NL && tid >= d) ? s_c[tid - d] : 0u;
    __syncthreads();
    if (tid < NL) s_c[tid] += x;
    __syncthreads();
  }
  const uint32_t base = (uint32_t)(2 * n * (uint64_t)w);
  if (tid < NL) {
    const uint32_t ex = s_c[tid] - v;
    const bool carry = tid >= 128;
    if (!carry || w == kPipZWin - 1) {
      const uint32_t bin = carry ? (uint32_t)(kPipWin * 128 + tid - 128) : (uint32_t)(w * 128 + tid);
      reg.off[bin] = base + ex;
      reg.cnt[bin] = v;
    }
  }
  __syncthreads();
  if (tid < NL) s_c[tid] -= v;   // exclusive: cursors
  __syncthreads();
  pip_digits_pass<NT>(reg, n, w, [&](uint32_t lb, uint32_t pt, bool neg) {
    const uint32_t pos = atomicAdd(&s_c[lb], 1u);
    reg.ent[base + pos] = pt | (neg ? 0x80000000u : 0u);
  });
}

// Part k of K of window w's sort on one workgroup of NT threads: the workgroup owns local
// bins [lo, hi) (a 1/K slice of the window's 128 bins, or 192 with window 16's z-carry
// sub-bins), reads every digit of the window, histograms and scatters only its own bins, and
// places them after the window's entries in lower bins, which it counts itself (no workgroup
// waits for another). The K parts of a window write disjoint bins and entry ranges.
template <int NT>
__device__ __forceinline__ void pip_sort_window_part(const pip_region& reg, uint64_t n, int w,
                                                     int k, int K, uint32_t* s_h,
                                                     uint32_t* s_c, uint32_t* s_red) {
  const int tid = threadIdx.x;
  const int nl = w == kPipZWin - 1 ? kPipSortBins : 128;
  const uint32_t lo = (uint32_t)(k * nl / K), hi = (uint32_t)((k + 1) * nl / K), m = hi - lo;
  if (tid < (int)m) s_h[tid] = 0;
  __syncthreads();
  uint32_t below = 0;
  pip_digits_pass<NT>(reg, n, w, [&](uint32_t lb, uint32_t, bool) {
    if (lb >= lo && lb < hi) atomicAdd(&s_h[lb - lo], 1u);
    else if (lb < lo) ++below;
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) below += (uint32_t)__shfl_xor((int)below, o);
  if ((tid & 63) == 0) s_red[tid >> 6] = below;
  __syncthreads();
  uint32_t base_below = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) base_below += s_red[i];
  // inclusive Hillis-Steele scan over the m bins (threads < m)
  uint32_t v = tid < (int)m ? s_h[tid] : 0u;
  if (tid < (int)m) s_c[tid] = v;
  __syncthreads();
  for (uint32_t d = 1; d < m; d <<= 1) {
    const uint32_t x = (tid < (int)m && (uint32_t)tid >= d) ? s_c[tid - d] : 0u;
    __syncthreads();
    if (tid < (int)m) s_c[tid] += x;
    __syncthreads();
  }
  const uint32_t base = (uint32_t)(2 * n * (uint64_t)w) + base_below;
  if (tid < (int)m) {
    const uint32_t lb = lo + (uint32_t)tid;
    const uint32_t ex = s_c[tid] - v;
    const uint32_t bin = lb >= 128 ? (uint32_t)(kPipWin * 128 + lb - 128) : (uint32_t)(w * 128) + lb;
    reg.off[bin] = base + ex;
    reg.cnt[bin] = v;
  }
  __syncthreads();
  if (tid < (int)m) s_c[tid] -= v;   // exclusive: cursors
  __syncthreads();
  pip_digits_pass<NT>(reg, n, w, [&](uint32_t lb, uint32_t pt, bool neg) {
    if (lb >= lo && lb < hi) {
      const uint32_t pos = atomicAdd(&s_c[lb - lo], 1u);
      reg.ent[base + pos] = pt | (neg ? 0x80000000u : 0u);
    }
  });
}

// grid (kPipWin, npip), 1024 threads: window blockIdx.x + wbase's sort; window kPipWin is the
// batch's b sum and first failures.
__global__ __launch_bounds__(1024) void k_pip_sort(const uint32_t* __restrict__ pip_list,
                                                   const uint64_t* __restrict__ offsets,
                                                   uint64_t b0, uint64_t i0, uint32_t extra,
                                                   uint32_t pmin, ge_cached* __restrict__ tabs,
                                                   const bv_item* __restrict__ items,
                                                   uint32_t wbase) {
  __shared__ uint32_t s_h[kPipSortBins], s_c[kPipSortBins];
  __shared__ uint32_t s_b[16][8];
  __shared__ uint32_t s_f[16][4];
  const uint64_t bidx = b0 + pip_list[blockIdx.y];
  const uint64_t bs = offsets[bidx], n0 = offsets[bidx + 1] - bs;
  if (n0 < pmin) return;
  const uint64_t n = n0 + extra;   // votes + (group mode) key sums
  const pip_region reg = pip_at(tabs, bs - i0, n);
  const int w = (int)(blockIdx.x + wbase);
  if (w == kPipWin) {     // the batch's b sum and first failures
    pip_bsum_block<1024>(reg, n0, items + (bs - i0), s_b, s_f);
    return;
  }
  pip_sort_window<1024>(reg, n, w, s_h, s_c);
}

// Lanes [G bin, G bin + G) of the batch's bucket pass share bucket bin (gl: the lane's index
// in the pass, G = 2^lg): partial sums of the bin's entries, combined by a lane-shuffle tree.
// Entry k + 2's index and entry k + 1's point (whose index is already here) are fetched while
// entry k is added, so the dependent index -> point loads never stall the chain (a deeper
// ring of 2 or 3 points in flight measured slower: 0.375 vs 0.364 ms for config 1's call,
// profiles/r04g/pip_prefetch_ab.txt).
__device__ __forceinline__ void pip_bucket_lanes(const pip_region& reg, uint32_t gl,
                                                 uint32_t lg) {
  const uint32_t bin = gl >> lg, G = 1u << lg, g = gl & (G - 1);
  if (bin >= (uint32_t)kPipBins) return;   // whole G-groups (kPipBins is a multiple of 64)
  const uint32_t e0 = reg.off[bin], ne = reg.cnt[bin];
  const uint32_t a = e0 + (uint32_t)((uint64_t)ne * g >> lg),
                 e = e0 + (uint32_t)((uint64_t)ne * (g + 1) >> lg);
  ge acc;
  ge_identity(acc);
  uint32_t x = a < e ? reg.ent[a] : 0u;
  uint32_t x2 = a + 1 < e ? reg.ent[a + 1] : 0u;
  ge_niels nx;
  if (a < e) nx = reg.pts[x & 0x7fffffffu].n;
#pragma unroll 1
  for (uint32_t k = a; k < e; ++k) {
    ge_niels q = nx;
    const bool neg = (x >> 31) != 0;
    if (k + 1 < e) {
      x = x2;
      nx = reg.pts[x & 0x7fffffffu].n;
    }
    if (k + 2 < e) x2 = reg.ent[k + 2];
    ge_niels_cneg(q, neg);
    ge_add_niels(acc, acc, q, true);
  }
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll 1
  for (uint32_t o = 1; o < G; o <<= 1) {
    ge other;
    ge_shfl(other, acc, lane ^ (int)o);
    ge_add_ge(acc, acc, other, g_bc.k.d2);
  }
  if (g == 0) reg.S[bin] = acc;
}

// grid (bpb = kPipBins * G / 256 blocks per batch, npip). xcd: 1-D grid of
// 8 * bpb * ceil(npip / 8) blocks, remapped so that every block of a batch runs on one XCD
// (workgroups are dealt round-robin over the 8 XCDs) and each XCD walks its batches one after
// another: the batch's points (2n x 120 B, gathered at random by its buckets) then stay in
// that XCD's L2 instead of in all eight.
__global__ __launch_bounds__(256) void k_pip_buckets(const uint32_t* __restrict__ pip_list,
                                                     const uint64_t* __restrict__ offsets,
                                                     uint64_t b0, uint64_t i0, uint32_t lg,
                                                     uint32_t npip, uint32_t bpb, int xcd,
                                                     uint32_t extra, uint32_t pmin,
                                                     ge_cached* __restrict__ tabs) {
  uint32_t jb = blockIdx.y, xb = blockIdx.x;
  if (xcd) {
    const uint32_t k = blockIdx.x >> 3;
    jb = (blockIdx.x & 7) + 8 * (k / bpb);
    xb = k % bpb;
    if (jb >= npip) return;
  }
  const uint64_t bidx = b0 + pip_list[jb];
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  if (n < pmin) return;
  const pip_region reg = pip_at(tabs, bs - i0, n + extra);
  pip_bucket_lanes(reg, xb * blockDim.x + threadIdx.x, lg);
}

// grid (kPipWin, npip), one wave per window: sum_b b S_b as a suffix scan over lanes.
//   windows 0..30: lane l holds buckets 2l+1 and 2l+2, Q_l = S0 + S1, Suf_l = sum_{m>=l} Q_m:
//     sum_l (2l+1) S0 + (2l+2) S1 = Suf_0 + 2 sum_{l>=1} Suf_l + sum_l S1;
//     window 16 also adds the z-carry sub-bins (weight 1, lane l holds sub-bin l);
//   window 31: lane l < 17 folds the kPipTopSub sub-bins of digit l+1 into Q_l, and
//     sum_l (l+1) Q_l = sum_l Suf_l.
// Then a tree over lanes.
__global__ __launch_bounds__(64) void k_pip_windows(const uint32_t* __restrict__ pip_list,
                                                    const uint64_t* __restrict__ offsets,
                                                    uint64_t b0, uint64_t i0, uint32_t extra,
                                                    uint32_t pmin, ge_cached* __restrict__ tabs) {
  const uint64_t bidx = b0 + pip_list[blockIdx.y];
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  if (n < pmin) return;
  const pip_region reg = pip_at(tabs, bs - i0, n + extra);
  const int w = blockIdx.x, l = threadIdx.x;
  const fe& d2 = g_bc.k.d2;
  if (w == kPipWin) {
    // [-sum b_i]B = sum_w comb[w][digit w] (32 additions, no doublings), limb-parallel,
    // stored in cached form for the last addition of k_pip_final's Horner
    const lp_ctx L = lp_init((uint32_t)l);
    uint32_t bb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bb[j] = reg.bb[j];
    uint32_t v = lp_identity(L);
#pragma unroll 1
    for (int m = 0; m < kPipWin; ++m) {
      const int e = digit8(bb, m);
      v = lp_add(L, v, lp_niels_component(L, g_comb[129 * m + (e < 0 ? -e : e)], e < 0));
    }
    const uint32_t c = lp_to_cached(L, v, L.k < 10 ? d2.v[L.k] : 0u);
    const uint32_t field = L.row == 0 ? 1u : L.row == 1 ? 0u : L.row == 2 ? 3u : 2u;
    if (L.k < 10) reinterpret_cast<uint32_t*>(reg.Bc)[10 * field + L.k] = c;
    return;
  }
  const bool top = w == kPipWin - 1;
  ge suf, t;
  if (top) {
    ge_identity(suf);
    if (l < kPipTopStride) {
#pragma unroll 1
      for (int k = 0; k < kPipTopSub; ++k)
        ge_add_ge(suf, suf, reg.S[w * 128 + kPipTopStride * k + l], d2);
    }
  } else {
    ge_add_ge(suf, reg.S[w * 128 + 2 * l], reg.S[w * 128 + 2 * l + 1], d2);
  }
#pragma unroll 1
  for (int d = 1; d < 64; d <<= 1) {
    ge_shfl(t, suf, l + d < 64 ? l + d : l);
    if (l + d < 64) ge_add_ge(suf, suf, t, d2);
  }
  ge y;
  if (top) {
    y = suf;
  } else {
    if (l >= 1) ge_dbl(y, suf, true);
    else y = suf;
    ge_add_ge(y, y, reg.S[w * 128 + 2 * l + 1], d2);
    if (w == kPipZWin - 1) ge_add_ge(y, y, reg.S[kPipWin * 128 + l], d2);
  }
#pragma unroll 1
  for (int o = 32; o > 0; o >>= 1) {
    ge_shfl(t, y, l ^ o);
    ge_add_ge(y, y, t, d2);
  }
  if (l == 0) {
    ge_cached c;
    ge_to_cached(c, y, d2);
    reg.W[w] = c;
  }
}

// Latency form of k_pip_windows for few batches (npip <= kPipWinLpMax; config 1's one-call
// path): sum_d d S_{d-1} = sum_j 2^j T_j with T_j = sum of the buckets whose digit has bit j,
// every point operation limb-parallel (nw_lp.hpp), one wave per (window, part) on its own
// SIMD. k_pip_windows_lp, grid (kPipWin + 1, kPipWinLpParts, npip), 64 threads; part
// q = 2 j + h sums half h (entries 32 h .. 32 h + 31) of list j:
//   j < 8: T_j (windows 0..30: digits 1..128, 64 buckets for j < 7 and bucket 127 for
//     j = 7; window 31: digits 1..17 with their kPipTopSub sub-bins, j < 5);
//   j = 8: the z-carry sub-bins of window 16 (weight 1);
// and stores it (cached, lp layout) over the batch's point and entry arrays (contiguous,
// dead after k_pip_buckets).
// k_pip_wsum, grid (kPipWin, npip), one wave: the 7-doubling Horner over the parts.
// A wave's chain is <= 32 additions of ~0.4 us instead of the one-wave form's 15
// single-lane operations of ~5 us; in total instructions it is ~13x the one-wave form,
// hence only for few batches. Block kPipWin: [-sum b_i]B as in k_pip_windows (part 0).
constexpr uint32_t kPipWinLpMax = 8;
constexpr int kPipWinLpParts = 18;
uint32_t pip_win_lp_max() {   // NW_PIP_WIN_LP_MAX=0: always the one-wave form
  static const uint32_t v = (uint32_t)env_u64_zero("NW_PIP_WIN_LP_MAX", kPipWinLpMax);
  return v;
}
// the parts live in the dead point + entry arrays (contiguous in pip_at)
static_assert(2 * kPipFloor * sizeof(ge_niels_pad) + 4 * kPipWinCap * kPipFloor >=
                  4 * kPipWin * kPipWinLpParts * 64,
              "window parts do not fit the point array");

__device__ __forceinline__ uint32_t pip_lp_bucket(int w, int j, uint32_t i) {
  // i-th bucket of list j of window w, or ~0u
  if (j == 8) return (w == kPipZWin - 1 && i < (uint32_t)kPipCarryBins) ? kPipWin * 128 + i : ~0u;
  if (w != kPipWin - 1) {
    if (j == 7) return i == 0 ? (uint32_t)w * 128 + 127 : ~0u;
    if (i >= 64) return ~0u;
    const uint32_t d = ((i >> j) << (j + 1)) | (1u << j) | (i & ((1u << j) - 1));
    return (uint32_t)w * 128 + d - 1;
  }
  // top window: digits d in 1..17 with bit j, each over kPipTopSub sub-bins
  const uint32_t dd = i / kPipTopSub, k = i % kPipTopSub;
  uint32_t seen = 0;
  for (uint32_t d = 1; d <= (uint32_t)kPipTopStride; ++d) {
    if (!((d >> j) & 1)) continue;
    if (seen++ == dd) return (uint32_t)w * 128 + kPipTopStride * k + d - 1;
  }
  return ~0u;
}

// Extended point in lp layout (row r = coordinate r of X, Y, Z, T), identity for ~0u;
// branch-free, so the prefetched loads stay in flight across the additions.
__device__ __forceinline__ uint32_t pip_lp_load(const lp_ctx& L, const ge* S, uint32_t b) {
  const uint32_t x = reinterpret_cast<const uint32_t*>(S + (b == ~0u ? 0u : b))
      [10 * L.row + (L.k < 10 ? L.k : 9u)];
  return b == ~0u ? lp_identity(L) : L.k < 10 ? x : 0u;
}

// [-sum b_i]B = sum_w comb[w][digit w] (32 additions, no doublings), limb-parallel, stored
// in cached form for the last addition of the Horner (one wave).
__device__ __forceinline__ void pip_lp_bsum_point(const pip_region& reg, const lp_ctx& L,
                                                  uint32_t d2l) {
  uint32_t bb[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) bb[m] = reg.bb[m];
  uint32_t v = lp_identity(L);
#pragma unroll 1
  for (int m = 0; m < kPipWin; ++m) {
    const int e = digit8(bb, m);
    v = lp_add(L, v, lp_niels_component(L, g_comb[129 * m + (e < 0 ? -e : e)], e < 0));
  }
  const uint32_t c = lp_to_cached(L, v, d2l);
  if (L.k < 10) reinterpret_cast<uint32_t*>(reg.Bc)[10 * (L.row ^ 1u) + L.k] = c;
}

// Part q of window w (see above), half `half2` of its 32 entries on this wave: wave 1's sum
// is added by wave 0 through LDS (s_other, 64 words; both waves reach the barrier). Two chains
// of <= 16 additions side by side instead of one of <= 32 (config 1's one call: the window
// pass 29 -> 25 us). The part goes to parts[(w * kPipWinLpParts + q) * 64 + lane].
__device__ __forceinline__ void pip_lp_part(const pip_region& reg, const lp_ctx& L,
                                            uint32_t d2l, int w, int q, int half2, int lane,
                                            uint32_t* s_other, uint32_t* parts) {
  const int j = q >> 1;
  const uint32_t mine =
      lane < 16 ? pip_lp_bucket(w, j, 32u * (uint32_t)(q & 1) + 16u * (uint32_t)half2 + lane)
                : ~0u;
  const uint32_t cnt = (uint32_t)__builtin_popcountll(__ballot(mine != ~0u));
  uint32_t v = lp_identity(L);
  if (cnt) {
    uint32_t buf[8];   // point i + 8 is loaded while point i is added
#pragma unroll
    for (int u = 0; u < 8; ++u)
      buf[u] = pip_lp_load(L, reg.S, (uint32_t)__builtin_amdgcn_readlane((int)mine, u));
#pragma unroll 1
    for (uint32_t i = 0; i < cnt; i += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t x = buf[u];
        const uint32_t nx = i + 8 + u;
        buf[u] = pip_lp_load(
            L, reg.S, nx < 16 ? (uint32_t)__builtin_amdgcn_readlane((int)mine, (int)nx) : ~0u);
        v = lp_add(L, v, lp_to_cached(L, x, d2l));
      }
    }
  }
  if (half2 == 1) s_other[lane] = lp_to_cached(L, v, d2l);
  __syncthreads();
  if (half2 == 1) return;
  v = lp_add(L, v, s_other[lane]);
  parts[(w * kPipWinLpParts + q) * 64 + lane] = lp_to_cached(L, v, d2l);
}

// Part q of the top window on all four waves of the workgroup (8 entries each; waves 1-3's
// sums added by wave 0 through LDS, s_other4: 3 x 64 words): chains of <= 8 additions, the
// top window's parts being on the critical path of the fused tail.
__device__ __forceinline__ void pip_lp_part4(const pip_region& reg, const lp_ctx& L,
                                             uint32_t d2l, int q, int wave, int lane,
                                             uint32_t* s_other4, uint32_t* parts) {
  const int w = kPipWin - 1, j = q >> 1;
  const uint32_t mine =
      lane < 8 ? pip_lp_bucket(w, j, 32u * (uint32_t)(q & 1) + 8u * (uint32_t)wave + lane) : ~0u;
  const uint32_t cnt = (uint32_t)__builtin_popcountll(__ballot(mine != ~0u));
  uint32_t v = lp_identity(L);
  if (cnt) {
    uint32_t buf[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      buf[u] = pip_lp_load(L, reg.S, (uint32_t)__builtin_amdgcn_readlane((int)mine, u));
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if ((uint32_t)u < cnt) v = lp_add(L, v, lp_to_cached(L, buf[u], d2l));
  }
  if (wave != 0) s_other4[64 * (wave - 1) + lane] = lp_to_cached(L, v, d2l);
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) v = lp_add(L, v, s_other4[64 * k + lane]);
  parts[(w * kPipWinLpParts + q) * 64 + lane] = lp_to_cached(L, v, d2l);
}

// W_w = sum_j 2^j T_j: the 7-doubling Horner over window w's parts (one wave).
__device__ __forceinline__ void pip_lp_wsum(const pip_region& reg, const lp_ctx& L, int w,
                                            int lane, const uint32_t* parts) {
  const uint32_t* part = parts + (size_t)w * kPipWinLpParts * 64 + lane;
  uint32_t t[kPipWinLpParts];
#pragma unroll
  for (int q = 0; q < kPipWinLpParts; ++q) t[q] = part[64 * q];
  uint32_t r = lp_add(L, lp_identity(L), t[14]);
  r = lp_add(L, r, t[15]);
#pragma unroll 1
  for (int j = 6; j >= 0; --j) {
    r = lp_dbl(L, r);
    // 2 j and 2 j + 1 by a runtime index would put t in scratch: select instead
    uint32_t a = t[0], b = t[1];
#pragma unroll
    for (int k = 1; k < 7; ++k)
      if (j == k) a = t[2 * k], b = t[2 * k + 1];
    r = lp_add(L, r, a);
    r = lp_add(L, r, b);
  }
  if (w == kPipZWin - 1) {
    r = lp_add(L, r, t[16]);
    r = lp_add(L, r, t[17]);
  }
  const fe& d2 = g_bc.k.d2;
  const uint32_t c = lp_to_cached(L, r, L.k < 10 ? d2.v[L.k] : 0u);
  if (L.k < 10) reinterpret_cast<uint32_t*>(reg.W + w)[10 * (L.row ^ 1u) + L.k] = c;
}

// The batch's verdict from the Horner's result (lane 0 writes).
__device__ __forceinline__ void pip_verdict(const pip_region& reg, const lp_ctx& L, uint32_t v,
                                            uint32_t* s_tmp, uint64_t bidx, uint64_t n,
                                            int32_t* status, uint64_t* fail_index,
                                            uint32_t* group_ok) {
  const bool ident = lp_is_identity(L, v, s_tmp);
  if (threadIdx.x != 0) return;
  const uint32_t ff[3] = {reg.hdr[0], reg.hdr[1], reg.hdr[2]};
  if (group_ok) {   // group mode: any flag or a nonzero sum sends the group to the fallback
    group_ok[bidx] = (ff[0] == kNone && ff[1] == kNone && ff[2] == kNone && ident) ? 1u : 0u;
    return;
  }
  uint64_t idx;
  const int st = batch_status(ff, reg.hdr[3], ident, n, &idx);
  status[bidx] = st;
  if (fail_index) fail_index[bidx] = idx;
}

__global__ __launch_bounds__(128) void k_pip_windows_lp(const uint32_t* __restrict__ pip_list,
                                                       const uint64_t* __restrict__ offsets,
                                                       uint64_t b0, uint64_t i0, uint32_t extra,
                                                       uint32_t pmin,
                                                       ge_cached* __restrict__ tabs) {
  const uint64_t bidx = b0 + pip_list[blockIdx.z];
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  if (n < pmin) return;
  const pip_region reg = pip_at(tabs, bs - i0, n + extra);
  const int w = blockIdx.x, q = blockIdx.y, lane = (int)(threadIdx.x & 63);
  const int half2 = (int)(threadIdx.x >> 6);   // which 16 of the part's 32 entries
  const lp_ctx L = lp_init((uint32_t)lane);
  const fe& d2 = g_bc.k.d2;
  const uint32_t d2l = L.k < 10 ? d2.v[L.k] : 0u;
  if (w == kPipWin) {
    if (q == 0 && half2 == 0) pip_lp_bsum_point(reg, L, d2l);
    return;
  }
  __shared__ uint32_t s_other[64];
  pip_lp_part(reg, L, d2l, w, q, half2, lane, s_other, reinterpret_cast<uint32_t*>(reg.pts));
}

__global__ __launch_bounds__(64) void k_pip_wsum(const uint32_t* __restrict__ pip_list,
                                                 const uint64_t* __restrict__ offsets,
                                                 uint64_t b0, uint64_t i0, uint32_t extra,
                                                 uint32_t pmin, ge_cached* __restrict__ tabs) {
  const uint64_t bidx = b0 + pip_list[blockIdx.y];
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  if (n < pmin) return;
  const pip_region reg = pip_at(tabs, bs - i0, n + extra);
  const int lane = (int)threadIdx.x;
  pip_lp_wsum(reg, lp_init((uint32_t)lane), blockIdx.x, lane,
              reinterpret_cast<const uint32_t*>(reg.pts));
}

__global__ __launch_bounds__(64) void k_pip_final(const uint32_t* __restrict__ pip_list,
                                                  const uint64_t* __restrict__ offsets,
                                                  uint64_t b0, uint64_t i0,
                                                  ge_cached* __restrict__ tabs,
                                                  int32_t* __restrict__ status,
                                                  uint64_t* __restrict__ fail_index,
                                                  uint32_t extra, uint32_t pmin,
                                                  uint32_t* __restrict__ group_ok) {
  __shared__ uint32_t s_tmp[40];
  const uint64_t bidx = b0 + pip_list[blockIdx.x];
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  if (n < pmin) return;
  const pip_region reg = pip_at(tabs, bs - i0, n + extra);
  const int tid = threadIdx.x;
  // Horner over the windows, the point spread limb-parallel over the wave (nw_lp.hpp)
  const lp_ctx L = lp_init((uint32_t)tid);
  uint32_t v = lp_identity(L);
#pragma unroll 1
  for (int w = kPipWin - 1; w >= 0; --w) {
    if (w != kPipWin - 1) {
#pragma unroll 1
      for (int k = 0; k < 8; ++k) v = lp_dbl(L, v);
    }
    v = lp_add(L, v, lp_cached_component(L, reg.W[w]));
  }
  v = lp_add(L, v, lp_cached_component(L, *reg.Bc));   // + [-sum b_i]B
  pip_verdict(reg, L, v, s_tmp, bidx, n, status, fail_index, group_ok);
}

// ---- config 1's one-call tail: buckets, window parts, window sums and the Horner in ONE
// launch, ordered by completion counters instead of kernel boundaries ----------------------
// The bucket pass is chain-bound and uneven: windows 16..31 hold only the c_i digits (half
// the entries per bucket of windows 0..15, which also hold z_i's), so their buckets are done
// at about half the pass. Here their window parts and sums start as soon as their own buckets
// are summed, and the Horner (the 248-doubling chain) starts on W_31 while windows 0..15 are
// still in their buckets; it needs W_w only 3.4 us x (31 - w) later, by which time the
// lower windows are summed.
//
// Roles by ticket (a per-launch counter taken by each workgroup as it starts, so a workgroup
// only ever waits for workgroups with smaller tickets, which are already running: no
// deadlock, whatever the residency):
//   [0, nbk)                 bucket workgroups (the bucket pass's blocks), each adding one to
//                            the completion count of every window its bins touch
//   nbk                      [-sum b_i]B
//   nbk + 1 + q              window 31's part q < 10 (its digits are <= 17: lists j <= 4
//                            only) on all four waves, after its buckets
//   nbk + 11                 the Horner (wave 0): W_31 from window 31's ten parts itself
//                            (4 doublings), then W_30 .. W_0 as their sums land, the verdict
//   nbk + 12 + 9 (30 - w) + i  window w's parts 2 i and 2 i + 1 (waves 0-1, 2-3), i < 9,
//                            after its buckets (window 16 also after the z-carry bins); the
//                            ninth workgroup of the window to finish sums it (wave 0)
// Every workgroup but the Horner waits only for smaller tickets; the Horner holds one
// workgroup slot, so the others always progress. The launch reserves kFuseLds of LDS per
// workgroup: one workgroup per CU, one wave per SIMD, so the Horner's chain issues alone on
// its SIMD as in k_pip_final (at 3 waves per SIMD it shared one with bucket and part waves:
// the tail took 224 vs 209 us as four launches).
// Waits spin on relaxed loads with s_sleep, bounded by kFuseSpinTicks of the 100 MHz
// real-time counter: on expiry the workgroup stops and the batch reports NW_E_DEVICE (never
// expected; a guard against a wedged launch).
constexpr int kFuseParts = kPipWinLpParts / 2;   // part workgroups per window (w < 31)
constexpr int kFuseTopParts = 10;                 // window 31: lists j <= 4, one part each
constexpr uint32_t kFuseCtr = 4 * 33 + 4;        // counter words: zero before the head
                                                 // (k_iota in w.chunk_start, or a job's own
                                                 // counters), and zero again after the tail:
                                                 // its last workgroup clears them (fz_exit)
constexpr uint64_t kFuseSpinTicks = 200000000;   // 2 s
constexpr uint32_t kFuseLds = 96 * 1024;         // > 160 KiB / 2: one workgroup per CU
enum : uint32_t { kFzTicket = 0, kFzError = 1, kFzTicket2 = 2, kFzBuckets = 4, kFzParts = 4 + 33,
                  kFzWsum = 4 + 66, kFzRole0 = 4 + 99, kFzPoints = 4 + 100, kFzExit = 4 + 101 };
static_assert(kFzExit < kFuseCtr, "counters within the zeroed words");
constexpr size_t kFusePartBytes = 4ull * (kPipWin + 1) * kPipWinLpParts * 64;
// the parts live in the batch's digit arrays (cd, zd: dead after k_pip_sort)
constexpr uint64_t kFuseMinN = (kFusePartBytes + 51) / 52;
// ... and the fused launches are for latency: one round of one workgroup per CU. Above
// 16,384 votes the head's digit + point + sort workgroups exceed 256 and the separate
// kernels (3 waves per SIMD) take the batch.
constexpr uint64_t kFuseMaxN = 16384;
constexpr uint32_t kFuseMaxLg = 4;   // bucket lanes per bin in the fused tail (260 workgroups)

// Polls are relaxed (an acquire per poll would invalidate the XCD's L2 under the bucket
// lanes' gathers every few hundred cycles); the waiter takes ONE agent-scope acquire fence
// once the count is reached (fz_acquire), and a producer workgroup ONE release (fz_add after
// its barrier: the release is cumulative over the workgroup's stores ordered before it).
bool pip_fuse_on() {   // NW_PIP_FUSE=0: the tail as four launches (A/B hook)
  static const bool v = env_u64_zero("NW_PIP_FUSE", 1) != 0;
  return v;
}
bool pip_fuse_head_on() {   // NW_PIP_FUSE_HEAD=0: the points and sort kernels (A/B hook)
  static const bool v = env_u64_zero("NW_PIP_FUSE_HEAD", 1) != 0;
  return v;
}

// NW_PIP_FUSE_STAMPS=1 (diagnostic, one caller at a time): a host-mapped stamp buffer for
// k_pip_tail_fused; each launch first prints the previous launch's timeline (that call has
// returned): per role the first start and last end, W_31's arrival at the Horner, the
// Horner's W_15 and end, in us from the launch's first workgroup start.
// The same for k_pip_points_sorted: decompression and digit waves' last ends, the sorts'
// start (digits ready) and last end, in us from the launch's first workgroup start.
uint64_t* head_stamps(uint32_t nblk) {
  static const bool on = env_u64_zero("NW_PIP_FUSE_STAMPS", 0) != 0;
  static uint64_t* buf = nullptr;
  static uint32_t prev = 0;
  if (!on) return nullptr;
  if (buf && prev) {
    uint64_t t0 = ~0ull;
    for (uint32_t i = 0; i < prev; ++i) t0 = std::min(t0, buf[4 * i]);
    double dec = 0, dig = 0, s0 = 1e30, s1 = 0;
    for (uint32_t i = 0; i < prev; ++i) {
      const uint64_t* s = buf + 4 * i;
      const uint32_t role = (uint32_t)(s[2] >> 8);
      if (role == 6) {
        if (s[1]) dec = std::max(dec, (s[1] - t0) / 100.0);
        if (s[3]) dig = std::max(dig, (s[3] - t0) / 100.0);
      } else if (role == 7) {
        s0 = std::min(s0, (s[3] - t0) / 100.0);
        s1 = std::max(s1, (s[1] - t0) / 100.0);
      }
    }
    fprintf(stderr, "[head] digits done %.1f decompressions done %.1f sorts %.1f-%.1f\n", dig,
            dec, s0, s1);
  }
  if (!buf || nblk > prev) {
    if (buf) (void)hipHostFree(buf);
    buf = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&buf), 32ull * nblk,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return nullptr;
  }
  memset(buf, 0, 32ull * nblk);
  prev = nblk;
  void* dp = nullptr;
  return hipHostGetDevicePointer(&dp, buf, 0) == hipSuccess ? static_cast<uint64_t*>(dp)
                                                            : nullptr;
}

uint64_t* fuse_stamps(uint32_t nblk) {
  static const bool on = env_u64_zero("NW_PIP_FUSE_STAMPS", 0) != 0;
  static uint64_t* buf = nullptr;
  static uint32_t prev = 0;
  if (!on) return nullptr;
  if (buf && prev) {
    uint64_t t0 = ~0ull;
    for (uint32_t i = 0; i < prev; ++i) t0 = std::min(t0, buf[4 * i]);
    double rs[8][2];
    for (auto& r : rs) r[0] = 1e30, r[1] = 0;
    double w31 = 0, w15 = 0, hend = 0, wsum_end[33] = {0};
    for (uint32_t i = 0; i < prev; ++i) {
      const uint64_t* s = buf + 4 * i;
      const uint32_t role = (uint32_t)(s[2] >> 8);
      const double a = (s[0] - t0) / 100.0, e = (s[1] - t0) / 100.0;
      if (role < 8) rs[role][0] = std::min(rs[role][0], a), rs[role][1] = std::max(rs[role][1], e);
      if (role == 4) wsum_end[s[2] & 63] = e;
      if (role == 5) w31 = (s[3] - t0) / 100.0, hend = e;
    }
    double b31 = 0, b30 = 0, r31a = 1e30, r31b = 0, p31 = 0;
    for (uint32_t i = 0; i < prev; ++i) {
      const uint64_t* s = buf + 4 * i;
      const uint32_t role = (uint32_t)(s[2] >> 8), wv = (uint32_t)(s[2] & 0xff);
      if ((buf[4 * i + 2] >> 8) == 5) w15 = (s[1] - t0) / 100.0;
      if (role == 1 && wv == 31) b31 = std::max(b31, (s[1] - t0) / 100.0);
      if (role == 1 && wv == 30) b30 = std::max(b30, (s[1] - t0) / 100.0);
      if (role == 3 && wv == 31) {
        r31a = std::min(r31a, (s[3] - t0) / 100.0);
        r31b = std::max(r31b, (s[3] - t0) / 100.0);
        p31 = std::max(p31, (s[1] - t0) / 100.0);
      }
    }
    fprintf(stderr, "[fuse31] w31 buckets done %.1f (w30 %.1f); w31 parts saw them %.1f-%.1f, "
            "done %.1f\n", b31, b30, r31a, r31b, p31);
    fprintf(stderr,
            "[fuse] buckets %.1f-%.1f bsum %.1f-%.1f parts %.1f-%.1f wsum -%.1f horner %.1f-%.1f "
            "(W_31 at %.1f) | W ready: w31 %.1f w24 %.1f w16 %.1f w15 %.1f w8 %.1f w0 %.1f\n",
            rs[1][0], rs[1][1], rs[2][0], rs[2][1], rs[3][0], rs[3][1], rs[4][1], rs[5][0],
            hend, w31, wsum_end[31], wsum_end[24], wsum_end[16], wsum_end[15], wsum_end[8],
            wsum_end[0]);
    (void)w15;
  }
  if (!buf || nblk > prev) {
    if (buf) (void)hipHostFree(buf);
    buf = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&buf), 32ull * nblk,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return nullptr;
  }
  memset(buf, 0, 32ull * nblk);
  prev = nblk;
  void* dp = nullptr;
  return hipHostGetDevicePointer(&dp, buf, 0) == hipSuccess ? static_cast<uint64_t*>(dp)
                                                            : nullptr;
}

__device__ __forceinline__ uint32_t fz_poll(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fz_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }
__device__ __forceinline__ void fz_add(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// Lane 0 spins until *p >= want (or the budget is spent: false, error flagged).
__device__ __forceinline__ bool fz_wait(uint32_t* ctr, uint32_t idx, uint32_t want) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (fz_poll(ctr + idx) < want) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kFuseSpinTicks) {
      __hip_atomic_store(ctr + kFzError, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}
// A workgroup of k_pip_tail_fused is done with the counters: its one thread that made the
// workgroup's last counter access counts it out, and the last of the launch's workgroups
// clears every counter word (the head's too: it has finished), so the next call on the same
// counters starts from zero with no zeroing kernel or copy. Every role calls this exactly
// once per workgroup, on every return path, after its last wait / add.
__device__ __forceinline__ void fz_exit(uint32_t* ctr) {
  const uint32_t prev = __hip_atomic_fetch_add(ctr + kFzExit, 1u, __ATOMIC_ACQ_REL,
                                               __HIP_MEMORY_SCOPE_AGENT);
  if (prev + 1 == gridDim.x)
    for (uint32_t i = 0; i < kFuseCtr; ++i)
      __hip_atomic_store(ctr + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Bucket workgroups whose bins touch window w (w = kPipWin: the z-carry bins).
__device__ __forceinline__ uint32_t fz_bucket_blocks(int w, uint32_t lg) {
  const uint32_t b0 = (uint32_t)w * 128, b1 = w == kPipWin ? b0 + kPipCarryBins : b0 + 128;
  return (((b1 - 1) << lg) >> 8) - ((b0 << lg) >> 8) + 1;
}

__global__ __launch_bounds__(256) void k_pip_tail_fused(const uint64_t* __restrict__ offsets,
                                                        uint64_t bidx, uint64_t i0,
                                                        uint32_t lg, uint32_t nbk,
                                                        ge_cached* __restrict__ tabs,
                                                        uint32_t* __restrict__ ctr,
                                                        int32_t* __restrict__ status,
                                                        uint64_t* __restrict__ fail_index,
                                                        uint64_t* __restrict__ stamps,
                                                        const bv_item* __restrict__ items,
                                                        int bsum_here, uint32_t* done,
                                                        uint32_t done_seq) {
  __shared__ uint32_t s_ticket, s_ok;
  __shared__ uint32_t s_other[3][64];
  __shared__ uint32_t s_tmp[40];
  const int tid = (int)threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    s_ticket = __hip_atomic_fetch_add(ctr + kFzTicket, 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    s_ok = 1u;
  }
  __syncthreads();
  const uint32_t t = s_ticket;
  // NW_PIP_FUSE_STAMPS: per workgroup (by ticket) start, end, role / window (diagnostic)
  const auto stamp = [&](int slot, uint64_t v) {
    if (stamps && tid == 0) stamps[4 * t + slot] = v;
  };
  stamp(0, __builtin_amdgcn_s_memrealtime());
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  const pip_region reg = pip_at(tabs, bs - i0, n);
  uint32_t* parts = reinterpret_cast<uint32_t*>(reg.cd);
  const lp_ctx L = lp_init((uint32_t)lane);
  const uint32_t d2l = L.k < 10 ? g_bc.k.d2.v[L.k] : 0u;
  if (t < nbk) {   // ---- buckets
    pip_bucket_lanes(reg, t * 256 + (uint32_t)tid, lg);
    __syncthreads();
    if (tid == 0) {
      const uint32_t bin0 = (t * 256) >> lg, bin1 = ((t + 1) * 256 - 1) >> lg;
      for (uint32_t wv = bin0 >> 7; wv <= ((bin1 < (uint32_t)kPipBins ? bin1 : kPipBins - 1) >> 7);
           ++wv)
        if (bin0 < (uint32_t)kPipBins) fz_add(ctr + kFzBuckets + wv, 1u);
      stamp(1, __builtin_amdgcn_s_memrealtime());
      stamp(2, 0x100u | ((t * 256) >> lg >> 7));
      fz_exit(ctr);
    }
    return;
  }
  if (t == nbk) {   // ---- (fused head: sum b_i and the first failures, then) [-sum b_i]B
    if (bsum_here) {
      __shared__ uint32_t s_b[4][8];
      __shared__ uint32_t s_f[4][4];
      pip_bsum_block<256>(reg, n, items + (bs - i0), s_b, s_f);
      __syncthreads();
      fz_acquire();   // lane 0 of wave 0 wrote hdr / bb
    }
    if (wave == 0) {
      pip_lp_bsum_point(reg, L, d2l);
      if (lane == 0) fz_add(ctr + kFzWsum + kPipWin, 1u);
      stamp(1, __builtin_amdgcn_s_memrealtime());
      stamp(2, 0x200u);
      if (lane == 0) fz_exit(ctr);
    }
    return;
  }
  const uint32_t pt = t - nbk - 1;
  if (pt < (uint32_t)kFuseTopParts) {   // ---- window 31's parts
    if (tid == 0) s_ok = fz_wait(ctr, kFzBuckets + kPipWin - 1, fz_bucket_blocks(kPipWin - 1, lg))
                             ? 1u : 0u;
    __syncthreads();
    if (!s_ok) {
      if (tid == 0) fz_exit(ctr);
      return;
    }
    fz_acquire();
    stamp(3, __builtin_amdgcn_s_memrealtime());
    pip_lp_part4(reg, L, d2l, (int)pt, wave, lane, &s_other[0][0] + 0, parts);
    if (wave == 0 && lane == 0) fz_add(ctr + kFzParts + kPipWin - 1, 1u);
    stamp(1, __builtin_amdgcn_s_memrealtime());
    stamp(2, 0x300u | (uint32_t)(kPipWin - 1));
    if (wave == 0 && lane == 0) fz_exit(ctr);
    return;
  }
  if (pt > (uint32_t)kFuseTopParts) {   // ---- window parts (+ the window's sum)
    const uint32_t pg = pt - kFuseTopParts - 1;
    const int w = kPipWin - 2 - (int)(pg / kFuseParts), i = (int)(pg % kFuseParts);
    if (tid == 0) {
      bool ok = fz_wait(ctr, kFzBuckets + w, fz_bucket_blocks(w, lg));
      if (ok && w == kPipZWin - 1) ok = fz_wait(ctr, kFzBuckets + kPipWin, fz_bucket_blocks(kPipWin, lg));
      s_ok = ok ? 1u : 0u;
    }
    __syncthreads();
    if (!s_ok) {
      if (tid == 0) fz_exit(ctr);
      return;
    }
    fz_acquire();
    stamp(3, __builtin_amdgcn_s_memrealtime());   // its buckets were ready
    const int q = 2 * i + (wave >> 1), half2 = wave & 1;
    pip_lp_part(reg, L, d2l, w, q, half2, lane, s_other[wave >> 1], parts);
    __syncthreads();   // wave 2's part before wave 0 counts the workgroup (waves 1 and 3
                       // returned from pip_lp_part after its barrier)
    if (wave != 0) return;
    uint32_t last = 0;
    if (lane == 0)
      last = __hip_atomic_fetch_add(ctr + kFzParts + w, 1u, __ATOMIC_ACQ_REL,
                                    __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)kFuseParts - 1;
    stamp(1, __builtin_amdgcn_s_memrealtime());
    stamp(2, 0x300u | (uint32_t)w);
    if (!__builtin_amdgcn_readfirstlane(last)) {
      if (lane == 0) fz_exit(ctr);
      return;
    }
    fz_acquire();
    pip_lp_wsum(reg, L, w, lane, parts);
    if (lane == 0) fz_add(ctr + kFzWsum + w, 1u);
    stamp(1, __builtin_amdgcn_s_memrealtime());
    stamp(2, 0x400u | (uint32_t)w);   // this workgroup also summed the window
    if (lane == 0) fz_exit(ctr);
    return;
  }
  // ---- the Horner (wave 0)
  if (wave != 0) return;
  // W_31 = sum_{j <= 4} 2^j T_j straight from window 31's parts (2 j, 2 j + 1 = T_j)
  uint32_t got0 = 1;
  if (lane == 0)
    got0 = fz_wait(ctr, kFzParts + kPipWin - 1, (uint32_t)kFuseTopParts) ? 1u : 0u;
  bool ok = __builtin_amdgcn_readfirstlane(got0) != 0;
  fz_acquire();
  stamp(3, __builtin_amdgcn_s_memrealtime());
  const uint32_t* top = parts + (size_t)(kPipWin - 1) * kPipWinLpParts * 64 + lane;
  uint32_t tp[kFuseTopParts];
#pragma unroll
  for (int q = 0; q < kFuseTopParts; ++q) tp[q] = top[64 * q];
  uint32_t v = lp_add(L, lp_identity(L), tp[8]);
  v = lp_add(L, v, tp[9]);
#pragma unroll
  for (int j = 3; j >= 0; --j) {
    v = lp_dbl(L, v);
    v = lp_add(L, v, tp[2 * j]);
    v = lp_add(L, v, tp[2 * j + 1]);
  }
#pragma unroll 1
  for (int w = kPipWin - 2; w >= 0 && ok; --w) {
#pragma unroll 1
    for (int k = 0; k < 8; ++k) v = lp_dbl(L, v);
    uint32_t got = 1;
    if (lane == 0) got = fz_wait(ctr, kFzWsum + w, 1u) ? 1u : 0u;
    ok = __builtin_amdgcn_readfirstlane(got) != 0;
    fz_acquire();
    if (w == kPipZWin - 2) stamp(1, __builtin_amdgcn_s_memrealtime());   // reached W_15
    v = lp_add(L, v, lp_cached_component(L, reg.W[w]));
  }
  uint32_t got = ok ? 1u : 0u;
  if (ok && lane == 0) got = fz_wait(ctr, kFzWsum + kPipWin, 1u) ? 1u : 0u;
  ok = __builtin_amdgcn_readfirstlane(got) != 0;
  fz_acquire();
  if (lane == 0 && fz_poll(ctr + kFzError)) ok = false;
  ok = __builtin_amdgcn_readfirstlane(ok ? 1u : 0u) != 0;
  if (!ok) {
    if (lane == 0) {
      status[bidx] = NW_E_DEVICE;
      if (fail_index) fail_index[bidx] = 0;
      __threadfence_system();
      if (done) __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      fz_exit(ctr);
    }
    return;
  }
  if (lane == 0) fz_exit(ctr);   // the Horner's counter accesses are over
  v = lp_add(L, v, lp_cached_component(L, *reg.Bc));   // + [-sum b_i]B
  pip_verdict(reg, L, v, s_tmp, bidx, n, status, fail_index, nullptr);
  stamp(1, __builtin_amdgcn_s_memrealtime());
  stamp(2, 0x500u);
  if (lane == 0) __threadfence_system();   // outputs may be host-mapped (direct outputs)
  // the verdict is out: tell a host spinning on `done` (NW_BATCH_SPIN), ahead of the
  // kernel's completion signal (the other workgroups are counting out)
  if (lane == 0 && done)
    __hip_atomic_store(done, done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

struct bv_ws {
  bv_item* items;
  ge_cached* tabs;
  bv_chunk* chunks;
  bv_chunk_out* outs;
  uint32_t* multi;
  uint32_t* multi_first;
  uint32_t* chunk_start;
  uint32_t* pip_list;
  uint32_t* plan_tot;   // 3 per 1024-batch plan block
};

size_t bv_layout(uint64_t units, char* base, bv_ws* w) {
  const uint64_t u = units ? units : 1;
  const size_t s_items = a256(sizeof(bv_item) * u), s_tabs = a256(sizeof(ge_cached) * 16 * u),
               s_ch = a256(sizeof(bv_chunk) * u), s_out = a256(sizeof(bv_chunk_out) * u),
               s_m = a256(4 * u);
  if (w) {
    char* p = base;
    w->items = reinterpret_cast<bv_item*>(p); p += s_items;
    w->tabs = reinterpret_cast<ge_cached*>(p); p += s_tabs;
    w->chunks = reinterpret_cast<bv_chunk*>(p); p += s_ch;
    w->outs = reinterpret_cast<bv_chunk_out*>(p); p += s_out;
    w->multi = reinterpret_cast<uint32_t*>(p); p += s_m;
    w->multi_first = reinterpret_cast<uint32_t*>(p); p += s_m;
    w->pip_list = reinterpret_cast<uint32_t*>(p); p += s_m;
    w->plan_tot = reinterpret_cast<uint32_t*>(p); p += a256(12 * (u / 1024 + 2));
    w->chunk_start = reinterpret_cast<uint32_t*>(p);
  }
  return s_items + s_tabs + s_ch + s_out + 3 * s_m + a256(12 * (u / 1024 + 2)) + a256(4 * (u + 1));
}

}  // namespace

hipError_t upload_batch_consts() {
  static batch_consts host;
  static std::once_flag once;
  std::call_once(once, [] {
    compute_consts(host.k, host.btab);
    strict_consts sk;
    compute_strict_consts(sk, host.b128);
    compute_torsion(host.tor);
    for (int i = 0; i < 8; ++i) host.l[i] = L_W[i];
  });
  static std::vector<ge_niels> comb(32 * 129);
  static std::once_flag once_comb;
  std::call_once(once_comb, [] { compute_comb(comb.data()); });
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_bc), &host, sizeof(host), 0, hipMemcpyHostToDevice);
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_comb), comb.data(), sizeof(ge_niels) * comb.size(), 0,
                           hipMemcpyHostToDevice);
}

size_t batch_workspace_bytes(uint64_t nbatches, uint64_t nitems) {
  return bv_layout(std::min<uint64_t>(nitems + nbatches, slice_units()), nullptr, nullptr);
}

// Committee key tables (a committee's keys, tabulated once while the committee is
// unchanged): per key the comb tables j * 2^(W t) A with the runtime keyspec (nw_kernels.h
// keyspec_for: W = 20 up to 64 keys, else 16; t < ntab = ceil(253 / W), j = 0..2^(W-1),
// affine niels), plus a j * 2^128 A table when W does not divide 128. Keyed strict checks (headers, votes) take
// [k]A from them with no doublings; keyed vote chunks use the j * A and j * 2^128 A tables.
//   k_key_cmp   one block: flag = force or (pks != saved); then saved = pks when they differ.
//   k_key_base  one lane per key: decompress (dalek semantics), the comb bases 2^(W t) A by
//               W doublings each; base[2 key] = A, base[2 key + 1] = 2^128 A for the group
//               path, comb[kKeyTables key + t] for k_key_tabs.
//   k_key_tabs  one lane per run of kKeyRun consecutive entries of one (key, t): j0 * P by
//               double-and-add, then j * P for the run by additions of P, each point parked
//               in its own output slot (X, Y, Z and the product of the run's earlier Z's,
//               packed 32 bytes each), ONE inversion per run (Montgomery's trick) and a
//               backward pass that rewrites every slot as its affine niels form: about 15
//               multiplications per entry instead of an inversion per entry (16-bit tables:
//               524,304 entries per key).
__global__ __launch_bounds__(256) void k_key_cmp(const uint32_t* __restrict__ pks,
                                                 uint32_t* __restrict__ saved, uint64_t nkeys,
                                                 uint32_t force, uint32_t* __restrict__ flag) {
  int diff = force ? 1 : 0;
  for (uint64_t i = threadIdx.x; i < 8 * nkeys && !diff; i += blockDim.x)
    diff = pks[i] != saved[i];
  diff = __syncthreads_or(diff);
  if (diff)
    for (uint64_t i = threadIdx.x; i < 8 * nkeys; i += blockDim.x) saved[i] = pks[i];
  if (threadIdx.x == 0) *flag = diff ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_key_base(const uint32_t* __restrict__ pks,
                                                  uint64_t nkeys, keyspec ks,
                                                  ge* __restrict__ base,
                                                  ge* __restrict__ comb,
                                                  uint32_t* __restrict__ ok,
                                                  const uint32_t* __restrict__ flag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nkeys || (flag && *flag == 0)) return;   // same committee: tables kept
  uint32_t Aw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) Aw[j] = pks[8 * i + j];
  ge P;
  const bool dec = ge_frombytes(P, Aw, g_bc.k);
  // lambda: [l] A == [lambda] T8 (l A lies in E[8] for every curve point), by
  // double-and-add over the 253 bits of l — once per key per committee
  uint32_t lam = 0;
  if (dec) {
    ge_cached Pc;
    ge_to_cached(Pc, P, g_bc.k.d2);
    ge acc;
    ge_identity(acc);
#pragma unroll 1
    for (int bit = 252; bit >= 0; --bit) {
      ge_dbl(acc, acc, true);
      if ((g_bc.l[bit >> 5] >> (bit & 31)) & 1u) ge_add_cached(acc, acc, Pc, true);
    }
    const int j = torsion_index(acc, g_bc.tor);
    lam = j > 0 ? (uint32_t)j : 0u;
  }
  ok[i] = (dec ? kKeyDecoded : 0u) | (dec && ge_is_small_order(P) ? kKeySmall : 0u) |
          (lam << kKeyLambdaShift);
  base[2 * i] = P;
  const uint32_t W = ks.W, nt = keyspec_tables(ks);
  ge H;   // 2^(W floor(128 / W)) A, doubled up to 2^128 A when W does not divide 128
#pragma unroll 1
  for (int t = 0; t < (int)ks.ntab; ++t) {
    if (t) {
#pragma unroll 1
      for (int d = 0; d < (int)W; ++d) ge_dbl(P, P, d == (int)W - 1);
    }
    comb[nt * i + t] = P;
    if (t == (int)(128 / W)) H = P;
  }
  if (128 % W) {
#pragma unroll 1
    for (int d = 0; d < (int)(128 % W); ++d) ge_dbl(H, H, true);
    comb[nt * i + ks.ntab] = H;
  }
  base[2 * i + 1] = H;
}

constexpr uint32_t kKeyRun = 64;

NW_HD void put_fe32(uint32_t* w, const fe& f) {
  uint32_t b[8];
  fe_tobytes(b, f);
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = b[i];
}

__global__ __launch_bounds__(256) void k_key_tabs(uint64_t nkeys, keyspec ks,
                                                  const ge* __restrict__ comb,
                                                  ge_niels_pad* __restrict__ tabs,
                                                  const uint32_t* __restrict__ flag) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t N = ks.nent, runs = (N + kKeyRun - 1) / kKeyRun;   // runs per table
  if (g >= nkeys * keyspec_tables(ks) * runs || (flag && *flag == 0)) return;
  const uint64_t pt = g / runs;   // tables * key + t
  const uint32_t j0 = (uint32_t)(g % runs) * kKeyRun;
  const uint32_t cnt = N - j0 < kKeyRun ? N - j0 : kKeyRun;
  const ge P = comb[pt];
  ge_cached Pc;
  ge_to_cached(Pc, P, g_bc.k.d2);
  ge acc;
  ge_identity(acc);
  if (j0) {
#pragma unroll 1
    for (int bit = 31 - __builtin_clz(j0); bit >= 0; --bit) {
      ge_dbl(acc, acc, true);
      if ((j0 >> bit) & 1) ge_add_cached(acc, acc, Pc, true);
    }
  }
  uint32_t* slot = reinterpret_cast<uint32_t*>(tabs + pt * N + j0);
  static_assert(sizeof(ge_niels_pad) == 128, "slot = 32 words");
  fe prefix;   // product of the Z's of the run's earlier entries
  fe_1(prefix);
#pragma unroll 1
  for (uint32_t e = 0; e < cnt; ++e) {
    uint32_t* w = slot + 32 * e;
    put_fe32(w, acc.X);
    put_fe32(w + 8, acc.Y);
    put_fe32(w + 16, acc.Z);
    put_fe32(w + 24, prefix);
    fe_mul(prefix, prefix, acc.Z);
    if (e + 1 < cnt) ge_add_cached(acc, acc, Pc, true);
  }
  fe inv;   // 1 / (Z_0 ... Z_e) while walking back
  fe_invert(inv, prefix);
#pragma unroll 1
  for (int e = (int)cnt - 1; e >= 0; --e) {
    uint32_t* w = slot + 32 * e;
    fe X, Y, Z, pre, zi, x, y;
    fe_frombytes(X, w);
    fe_frombytes(Y, w + 8);
    fe_frombytes(Z, w + 16);
    fe_frombytes(pre, w + 24);
    fe_mul(zi, inv, pre);   // 1 / Z_e
    fe_mul(inv, inv, Z);
    fe_mul(x, X, zi);
    fe_mul(y, Y, zi);
    ge_niels_pad out;
    fe_add(out.n.ypx, y, x);
    fe_carry(out.n.ypx);
    fe_sub(out.n.ymx, y, x);
    fe_mul(out.n.xy2d, x, y);
    fe_mul(out.n.xy2d, out.n.xy2d, g_bc.k.d2);
    out.pad[0] = out.pad[1] = 0;
    tabs[pt * N + j0 + (uint32_t)e] = out;
  }
}

size_t key_tables_bytes(uint64_t nkeys, const keyspec& ks) {
  const uint64_t n = nkeys ? nkeys : 1;
  return sizeof(ge_niels_pad) * (uint64_t)ks.tab * n + sizeof(ge) * (2 + keyspec_tables(ks)) * n;
}

hipError_t launch_key_tables(const uint32_t* pks, uint64_t nkeys, const keyspec& ks,
                             ge_niels_pad* tabs, uint32_t* ok, hipStream_t stream,
                             uint32_t* saved, uint32_t* flag, bool force) {
  if (nkeys == 0) return hipSuccess;
  if (ks.W < 16 || ks.W > kKeyWMax || ks.ntab > 16) return hipErrorInvalidValue;
  ge* base = reinterpret_cast<ge*>(tabs + (uint64_t)ks.tab * nkeys);
  ge* comb = base + 2 * nkeys;
  const uint32_t* fl = saved && flag ? flag : nullptr;
  if (fl)
    hipLaunchKernelGGL(k_key_cmp, dim3(1), dim3(256), 0, stream, pks, saved, nkeys,
                       force ? 1u : 0u, flag);
  hipLaunchKernelGGL(k_key_base, dim3((unsigned)((nkeys + 63) / 64)), dim3(64), 0, stream, pks,
                     nkeys, ks, base, comb, ok, fl);
  const uint64_t runs = (ks.nent + kKeyRun - 1) / kKeyRun;
  hipLaunchKernelGGL(k_key_tabs,
                     dim3((unsigned)((nkeys * keyspec_tables(ks) * runs + 255) / 256)),
                     dim3(256), 0, stream, nkeys, ks, comb, tabs, fl);
  return hipGetLastError();
}

namespace {

// ---- config 1's one-call head: the points and the window sorts in ONE launch ------------
// The sorts read only the digits (role-0 lanes: hash, scalars, recoding), which are done
// long before the R / A decompressions (the 252-squaring chains); here each window's sort
// starts when every role-0 wave has counted itself, beside the decompressions, instead of
// after the whole points kernel (one 10k batch: ~24 us off the chain). Roles by ticket:
// [0, nb0) digit workgroups (role 0: hash, scalars, recoding; 4 waves of 64 votes each,
// counted once per workgroup on kFzRole0), [nb0, npb) decompression workgroups (waves
// alternate R, A), then K workgroups per window's sort (each its own slice of the window's
// bins, NW_PIP_SORT_SPLIT, 2: with one release per wave K = 1 / 2 / 4 / 8 measured
// 0.330-0.336 / 0.334-0.335 / 0.336-0.339 / 0.365-0.369 ms, profiles/r04g/sort_split_ab.txt;
// with grouped digit workgroups 0.318-0.320 for K = 1, 2 and 4, head_ab.txt). The b sum and
// first failures (k_pip_sort's extra block) move to k_pip_tail_fused's [-sum b_i]B
// workgroup: they are needed only at the Horner's end. 256 threads, kFuseLds of LDS: one
// workgroup per CU (waits are only on smaller tickets).
__global__ __launch_bounds__(256) void k_pip_points_sorted(
    const uint32_t* __restrict__ digests, const uint64_t* __restrict__ offsets, uint64_t bidx,
    uint64_t i0, uint64_t i1, const uint32_t* __restrict__ pks,
    const uint32_t* __restrict__ sigs, const uint32_t* __restrict__ z16, z_key_t zkey,
    bv_item* __restrict__ items, ge_cached* __restrict__ tabs, uint32_t npb, uint32_t wv,
    uint32_t ksort, uint32_t* __restrict__ ctr, uint64_t* __restrict__ stamps,
    input_gate_t gate) {
  __shared__ uint32_t s_ticket, s_ok;
  __shared__ uint32_t s_h[kPipSortBins], s_c[kPipSortBins];
  const int tid = (int)threadIdx.x;
  if (tid == 0)
    s_ticket = __hip_atomic_fetch_add(ctr + kFzTicket2, 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const uint32_t t = s_ticket;
  const auto stamp = [&](int slot, uint64_t v) {   // NW_PIP_FUSE_STAMPS (diagnostic)
    if (stamps && (tid & 63) == 0) stamps[4 * t + slot] = v;
  };
  stamp(0, __builtin_amdgcn_s_memrealtime());
  const uint32_t nb0 = (wv + 3) / 4;   // role-0 workgroups (4 digit waves each)
  if (t < npb) {
    const pip_group_t nogrp{};
    const uint64_t wi = (uint64_t)(t < nb0 ? t : t - nb0) * 4 + (uint64_t)(tid >> 6);
    const int which = t < nb0 ? 0 : 1 + (int)(wi & 1);
    const uint64_t grp64 = t < nb0 ? wi : wi >> 1;   // 64-vote group of the wave
    if (gate.flags && grp64 < wv) {
      // the CPU may still be writing this wave's votes (input_gate_t): lane 0 waits for
      // their chunk's flag, then the whole wave acquires at system scope
      if ((tid & 63) == 0) {
        const uint32_t* f = gate.flags + (grp64 * 64) / gate.chunk;
        const uint64_t g0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != gate.seq) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - g0 > kFuseSpinTicks) {
            __hip_atomic_store(ctr + kFzError, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    if (grp64 < wv)
      pip_point_do(which, grp64 * 64 + (uint64_t)(tid & 63), digests, offsets, bidx, bidx + 1,
                   i0, i1, 0, pks, sigs, z16, zkey, items, tabs, nogrp);
    if (t < nb0) {
      // the workgroup's digits, then ONE count (a release per wave is an L2 write-back
      // each: 628 of them slowed the decompressions 73 -> 114 us); the decompressions signal
      // nothing, the launch boundary publishes their points
      __syncthreads();
      if (tid == 0) fz_add(ctr + kFzRole0, 1u);
      stamp(3, __builtin_amdgcn_s_memrealtime());
    } else {
      stamp(1, __builtin_amdgcn_s_memrealtime());
    }
    stamp(2, 0x600u);
    return;
  }
  const int w = (int)((t - npb) / ksort), k = (int)((t - npb) % ksort);   // window, part
  if (tid == 0) s_ok = fz_wait(ctr, kFzRole0, nb0) ? 1u : 0u;
  __syncthreads();
  if (!s_ok) return;   // kFzError is set: the tail reports NW_E_DEVICE
  fz_acquire();
  stamp(3, __builtin_amdgcn_s_memrealtime());
  const uint64_t bs = offsets[bidx], n = offsets[bidx + 1] - bs;
  __shared__ uint32_t s_red[4];
  pip_sort_window_part<256>(pip_at(tabs, bs - i0, n), n, w, k, (int)ksort, s_h, s_c, s_red);
  if (tid == 0) {
    stamp(1, __builtin_amdgcn_s_memrealtime());
    stamp(2, 0x700u | (uint32_t)w);
  }
}

// The Pippenger kernels over the pip_list batches of one slice (plain batches or, with
// grp.cert_vote_offsets set, certificate groups).
hipError_t launch_pip(const uint32_t* digests, const uint64_t* offsets, uint64_t b, uint64_t e,
                uint64_t i0, uint64_t i1, uint32_t pmin, uint64_t npip, uint64_t pmax,
                const uint32_t* pks, const uint32_t* sigs, const uint32_t* z16,
                const z_key_t& zkey, const bv_ws& w, int32_t* status, uint64_t* fail_index,
                const pip_group_t& grp, hipStream_t stream,
                uint32_t* fctr, const input_gate_t* gate = nullptr, uint32_t* done = nullptr,
                uint32_t done_seq = 0) {
  const bool group = grp.cert_vote_offsets != nullptr;
  const uint32_t extra = group ? grp.nkeys : 0;   // key sums
  const uint32_t roles = group ? 2 : 3;
  const uint64_t wv = (i1 - i0 + 63) / 64;   // waves per role
  // one large batch alone in its slice (config 1's call): the fused head and tail
  const bool fused = pip_fuse_on() && !group && npip == 1 && e - b == 1 && pmax >= kFuseMinN &&
                     pmax <= kFuseMaxN && npip <= pip_win_lp_max();
  const bool fuse_head = fused && pip_fuse_head_on();
  if (fuse_head) {
    // one large batch alone (config 1's call): points and sorts in one launch
    const uint32_t npb = (uint32_t)((wv + 3) / 4 + (2 * wv + 3) / 4);   // digit + point WGs
    static const uint32_t lds = (uint32_t)env_u64_zero("NW_PIP_FUSE_LDS", kFuseLds);
    // K workgroups per window's sort (each its own slice of the bins): NW_PIP_SORT_SPLIT
    static const uint32_t ks =
        (uint32_t)std::min<uint64_t>(8, std::max<uint64_t>(1, env_u64("NW_PIP_SORT_SPLIT", 2)));
    hipLaunchKernelGGL(k_pip_points_sorted, dim3(npb + kPipWin * ks), dim3(256), lds, stream,
                       digests, offsets, b, i0, i1, pks, sigs, z16, zkey, w.items, w.tabs, npb,
                       (uint32_t)wv, ks, fctr, head_stamps(npb + kPipWin * ks),
                       gate ? *gate : input_gate_t{nullptr, 0u, 64u});
  } else {
    hipLaunchKernelGGL(k_pip_points, dim3((unsigned)((wv * roles * 64 + 255) / 256)), dim3(256),
                       0, stream, digests, offsets, b, e, i0, i1, pmin, pks, sigs, z16, zkey,
                       w.items, w.tabs, grp, roles, 0u);
    if (group)
      hipLaunchKernelGGL(k_grp_keys, dim3((unsigned)npip), dim3(1024), 0, stream, offsets, b,
                         i0, pmin, w.items, w.tabs, grp);
    hipLaunchKernelGGL(k_pip_sort, dim3(kPipWin + 1, (unsigned)npip), dim3(1024), 0, stream,
                       w.pip_list, offsets, b, i0, extra, pmin, w.tabs, w.items, 0u);
  }
  // G lanes per bucket: about 8 additions each at the largest batch's mean bucket size
  // (<= 49 digits per vote over kPipBins buckets); more lanes measured slower (the shuffle
  // tree's full additions cost more than the niels additions they replace: 10k batch,
  // G = 64 122 us vs G = 16 68 us)
  uint32_t lg = 0;
  while (lg < 6 && (49 * (pmax + extra)) / kPipBins > 8ull << lg) ++lg;
  // ... but no more lanes than the chip runs at once (the shuffle tree is overhead)
  while (lg > 0 && ((npip * kPipBins) << lg) > (1ull << 21)) --lg;
  static const uint64_t lg_env = env_u64("NW_PIP_LG", 99);   // A/B hook
  if (lg_env <= 6) lg = (uint32_t)lg_env;
  if (fused && lg > kFuseMaxLg) lg = kFuseMaxLg;
  const uint32_t bpb = ((kPipBins << lg) + 255) / 256;
  // One large batch alone in its slice (config 1's call): the fused tail (NW_PIP_FUSE=0: the
  // four kernels below; fctr: zeroed counters, the caller's or w.chunk_start by k_iota)
  if (fused) {
    const uint32_t nbk = bpb;
    static const uint32_t lds = (uint32_t)env_u64_zero("NW_PIP_FUSE_LDS", kFuseLds);   // A/B
    const uint32_t nblk = nbk + 2 + kFuseTopParts + (kPipWin - 1) * kFuseParts;
    hipLaunchKernelGGL(k_pip_tail_fused, dim3(nblk), dim3(256), lds, stream, offsets, b, i0, lg,
                       nbk, w.tabs, fctr, status, fail_index, fuse_stamps(nblk), w.items,
                       fuse_head ? 1 : 0, done, done_seq);
    return hipGetLastError();
  }
  const int xcd = npip >= 8;
  const dim3 gb = xcd ? dim3((unsigned)(8 * bpb * ((npip + 7) / 8))) : dim3(bpb, (unsigned)npip);
  hipLaunchKernelGGL(k_pip_buckets, gb, dim3(256), 0, stream, w.pip_list, offsets, b, i0, lg,
                     (uint32_t)npip, bpb, xcd, extra, pmin, w.tabs);
  if (npip <= pip_win_lp_max()) {
    hipLaunchKernelGGL(k_pip_windows_lp, dim3(kPipWin + 1, kPipWinLpParts, (unsigned)npip),
                       dim3(128), 0, stream, w.pip_list, offsets, b, i0, extra, pmin, w.tabs);
    hipLaunchKernelGGL(k_pip_wsum, dim3(kPipWin, (unsigned)npip), dim3(64), 0, stream,
                       w.pip_list, offsets, b, i0, extra, pmin, w.tabs);
  } else
    hipLaunchKernelGGL(k_pip_windows, dim3(kPipWin + 1, (unsigned)npip), dim3(64), 0, stream,
                       w.pip_list, offsets, b, i0, extra, pmin, w.tabs);
  hipLaunchKernelGGL(k_pip_final, dim3((unsigned)npip), dim3(64), 0, stream, w.pip_list,
                     offsets, b, i0, w.tabs, status, fail_index, extra, pmin, grp.group_ok);
  return hipGetLastError();
}

uint32_t pip_min() {
  return (uint32_t)std::max<uint64_t>(
      kPipFloor, std::min<uint64_t>(0xffffffffu, env_u64("NW_BATCH_PIPPENGER_MIN", kPipMin)));
}

__global__ __launch_bounds__(256) void k_iota(uint32_t* __restrict__ list, uint32_t n,
                                              uint32_t* __restrict__ zero, uint32_t nz) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) list[i] = i;
  if (i < nz) zero[i] = 0;   // k_pip_tail_fused's counters
}

// Group g = certificates [g K, min(g K + K, ncert)): gofs[g] = its first vote; identity list.
__global__ __launch_bounds__(256) void k_grp_setup(const uint64_t* __restrict__ cvo,
                                                   uint64_t ncert, uint64_t K, uint64_t ngroups,
                                                   uint64_t* __restrict__ gofs,
                                                   uint32_t* __restrict__ ident,
                                                   uint32_t* __restrict__ group_ok) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g > ngroups) return;
  const uint64_t c = g * K < ncert ? g * K : ncert;
  gofs[g] = cvo[c];
  if (g < ngroups) {
    ident[g] = (uint32_t)g;
    group_ok[g] = 0;
  }
}

}  // namespace

hipError_t launch_verify_batch(const uint32_t* digests, const uint64_t* offsets,
                               const uint64_t* host_offsets, uint64_t nbatches,
                               const uint32_t* pks, const uint32_t* sigs, uint64_t nitems,
                               const uint32_t* z16, const z_key_t& zkey, void* workspace,
                               int32_t* status, uint64_t* fail_index, hipStream_t stream,
                               const key_tables_t* keys, const uint32_t* skip_group_ok,
                               uint64_t skip_per_group, double active_frac,
                               uint32_t* fuse_ctr, const input_gate_t* gate,
                               uint32_t* done, uint32_t done_seq) {
  // a gate is honoured by the fused head only: refuse it anywhere else (its waves would
  // read bytes the CPU has not written yet)
  if (gate && !verify_batch_gate_ok(nbatches, nitems)) return hipErrorInvalidValue;
  if (gate && (gate->chunk == 0 || gate->chunk % 64 != 0)) return hipErrorInvalidValue;
  if (done && !verify_batch_outputs_direct(nbatches, nitems)) return hipErrorInvalidValue;
  const key_tables_t kt = keys ? *keys : key_tables_t{nullptr, nullptr, nullptr, {}};
  const batch_skip_t sk{skip_group_ok, skip_per_group ? skip_per_group : 1};
  if (nbatches == 0) return hipSuccess;
  const uint64_t cap = std::min<uint64_t>(nitems + nbatches, slice_units());
  bv_ws w;
  bv_layout(cap, static_cast<char*>(workspace), &w);
  // Chunk size: fill the chip (~2 waves per SIMD of chunk lanes) but share the 252
  // doublings over as many votes as possible.
  // With a skip list only a fraction active_frac of the votes runs (the caller's estimate):
  // chunks are then cut small enough that those votes alone fill the chip — a 67-vote
  // certificate in one chunk is one lane's 2,300 serial additions. At 1 % failed
  // certificates that is one vote per chunk: each slice's latency is then one vote's
  // 128-doubling ladder (config 2 at 1 % invalid, N = 10 / 50 / 100: 0.82 / 0.79 / 0.80 of
  // the all-valid rate with chunks of >= 4 votes, 0.88 / 0.88 / 0.87 with 1).
  const uint64_t target_lanes = 256ull * 4 * 2 * 64;
  const double frac = skip_group_ok ? std::min(1.0, std::max(1e-6, active_frac)) : 1.0;
  const uint64_t run_votes = (uint64_t)(frac * (double)std::min(nitems, cap));
  uint32_t C = (uint32_t)std::min<uint64_t>(
      kMaxChunk, std::max<uint64_t>(1, run_votes / target_lanes));
  C = (uint32_t)std::min<uint64_t>(kMaxChunk, env_u64("NW_BATCH_CHUNK", C));
  const bool compact = skip_group_ok && frac < 1.0;   // items from the chunk list
  // Batches of at least pmin votes take the Pippenger path (NW_BATCH_PIPPENGER_MIN test
  // hook; never below kPipFloor, whose item slots are the smallest that hold the region).
  // With a skip list no batch may (launch_cert_groups only skips below pmin).
  const uint32_t pmin = skip_group_ok ? 0xffffffffu : pip_min();
  const pip_group_t nogrp{};
  uint64_t b = 0;
  while (b < nbatches) {
    // slice [b, e): items + batches <= cap
    uint64_t e = b, items = 0, chunks = 0, multi = 0, npip = 0, pmax = 0;
    while (e < nbatches) {
      const uint64_t n = host_offsets[e + 1] - host_offsets[e];
      if (e > b && items + n + (e - b + 1) > cap) break;
      if (n + 1 > cap) return hipErrorInvalidValue;   // one batch larger than a slice
      items += n;
      if (n >= pmin) {
        ++npip;
        pmax = std::max(pmax, n);
      } else {
        const uint64_t kb = (n + C - 1) / C;
        chunks += kb;
        multi += kb != 1;
      }
      ++e;
    }
    const uint64_t i0 = host_offsets[b], i1 = host_offsets[e];
    const unsigned nblk = (unsigned)((e - b + 1023) / 1024);
    // the caller's zeroed counters (fused path only, verify_batch_outputs_direct)
    const bool own_ctr = fuse_ctr && nbatches == 1 && pip_fuse_head_on() &&
                         verify_batch_outputs_direct(nbatches, nitems);
    if (npip == e - b && own_ctr) {
      // the fused head and tail read neither the Pippenger list nor zeroed workspace
    } else if (npip == e - b) {
      // every batch of the slice takes the Pippenger path (config 1's one 10k batch): no
      // chunk plan, the Pippenger list is the slice's batches in order
      hipLaunchKernelGGL(k_iota, dim3((unsigned)((npip + 255) / 256)), dim3(256), 0, stream,
                         w.pip_list, (uint32_t)npip, w.chunk_start, kFuseCtr);
    } else {
      hipLaunchKernelGGL(k_bv_plan_local, dim3(nblk), dim3(1024), 0, stream, offsets, b, e, C,
                         pmin, sk, w.plan_tot);
      hipLaunchKernelGGL(k_bv_plan_top, dim3(1), dim3(1024), 0, stream, nblk, e - b, w.plan_tot,
                         w.chunk_start);
      hipLaunchKernelGGL(k_bv_plan_apply, dim3(nblk), dim3(1024), 0, stream, offsets, b, e, C,
                         pmin, sk, w.plan_tot, w.chunk_start, w.multi, w.multi_first, w.pip_list,
                         status, fail_index);
    }
    if (chunks)
      hipLaunchKernelGGL(k_bv_expand, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                         stream, offsets, b, e - b, (uint32_t)chunks, w.chunk_start, w.chunks);
    if (compact && chunks)
      hipLaunchKernelGGL(k_bv_items_chunked, dim3((unsigned)((chunks * C + 255) / 256)),
                         dim3(256), 0, stream, w.chunks, (uint32_t)chunks,
                         w.chunk_start + (e - b), C, digests, b, i0, pks, sigs, z16, zkey,
                         w.items, w.tabs, kt);
    else if (i1 > i0 && npip != e - b && !compact)
      hipLaunchKernelGGL(k_bv_items, dim3((unsigned)((i1 - i0 + 255) / 256)), dim3(256), 0,
                         stream, digests, offsets, b, e, i0, i1, pmin, pks, sigs, z16, zkey,
                         w.items, w.tabs, kt, sk);
    if (npip) {
      const hipError_t pe = launch_pip(digests, offsets, b, e, i0, i1, pmin, npip, pmax, pks,
                                       sigs, z16, zkey, w, status, fail_index, nogrp, stream,
                                       own_ctr ? fuse_ctr : w.chunk_start, gate, done,
                                       done_seq);
      if (pe != hipSuccess) return pe;
    }
    if (chunks)
      hipLaunchKernelGGL(k_bv_chunks, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                         stream, w.chunks, (uint32_t)chunks, offsets, b, i0, w.items, w.tabs,
                         kt.tabs, kt.ks, w.outs, status, fail_index, w.chunk_start + (e - b));
    if (multi)
      hipLaunchKernelGGL(k_bv_combine,
                         dim3((unsigned)std::min<uint64_t>(multi, kCombineMaxBlocks)), dim3(256),
                         0, stream, w.multi, w.multi_first, (uint32_t)multi, offsets, b, C,
                         w.outs, status, fail_index, w.plan_tot + 3 * nblk + 1);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    b = e;
  }
  return hipSuccess;
}

size_t verify_batch_fuse_ctr_bytes() { return 4ull * kFuseCtr; }

bool verify_batch_gate_ok(uint64_t nbatches, uint64_t nitems) {
  return verify_batch_outputs_direct(nbatches, nitems) && pip_fuse_head_on();
}

bool verify_batch_outputs_direct(uint64_t nbatches, uint64_t nitems) {
  return nbatches == 1 && pip_fuse_on() && pip_win_lp_max() >= 1 &&
         nitems >= std::max<uint64_t>(kFuseMinN, pip_min()) && nitems <= kFuseMaxN &&
         nitems + 1 <= slice_units();
}

const ge* key_tables_base(const ge_niels_pad* tabs, uint64_t nkeys, const keyspec& ks) {
  return reinterpret_cast<const ge*>(tabs + (uint64_t)ks.tab * nkeys);
}

// Certificates per merged group, or 0 to verify every certificate's votes on its own:
// injected coefficients (deterministic tests want each certificate's own combination),
// NW_CERT_MERGE=0, committees above 256 keys, certificates with Pippenger-size vote sets,
// or too few votes to fill a group.
uint64_t cert_group_size(const uint64_t* host_cvo, uint64_t ncert, uint64_t nkeys,
                         bool injected_z, uint64_t target_votes) {
  const char* m = getenv("NW_CERT_MERGE");
  if (injected_z || (m && m[0] == '0') || nkeys == 0 || nkeys > 256 || ncert == 0 ||
      target_votes == 0)
    return 0;
  const uint64_t nvotes = host_cvo[ncert] - host_cvo[0];
  uint64_t qmax = 0;
  for (uint64_t c = 0; c < ncert; ++c) qmax = std::max(qmax, host_cvo[c + 1] - host_cvo[c]);
  if (qmax == 0 || qmax >= kPipMin) return 0;
  const uint64_t target =
      std::min<uint64_t>(env_u64("NW_CERT_GROUP_VOTES", target_votes), 1ull << 20);
  if (nvotes < std::max<uint64_t>(target, kPipMin)) return 0;
  // K from the mean votes per certificate, capped so that K certificates of the largest
  // vote count still fit one workspace slice (skewed counts never overflow a slice)
  const uint64_t K = std::max<uint64_t>(1, target * ncert / nvotes);
  return std::max<uint64_t>(1, std::min<uint64_t>(K, slice_units() / qmax));
}

bool cert_group_env_fixed() { return getenv("NW_CERT_GROUP_VOTES") != nullptr; }

// How many of the call's groups failed the merged check (group_ok == 0) and how many of its
// counted certificates (no pre-check or header failure) have a failing vote batch, for the
// host's adaptive grouping: k_grp_count sums into cnt (3 device words, zero between calls)
// over the whole grid, k_grp_publish copies the sums to host-mapped memory (read by a later
// call) and clears cnt. Launched after the per-certificate verify_batch (batch_st final).
__global__ __launch_bounds__(256) void k_grp_count(
    const uint32_t* __restrict__ group_ok, uint64_t ngroups, uint64_t ncert,
    const int32_t* __restrict__ batch_st, const int32_t* __restrict__ pre1,
    const int32_t* __restrict__ pre2, const int32_t* __restrict__ hdr_st,
    uint32_t* __restrict__ cnt) {
  uint32_t v[3] = {0, 0, 0};   // failed groups, counted certificates, failing ones
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t g = t0; g < ngroups; g += stride) v[0] += group_ok[g] == 0;
  for (uint64_t c = t0; c < ncert; c += stride) {
    if (pre1[c] != 0 || hdr_st[c] != 0 || pre2[c] != 0) continue;
    ++v[1];
    v[2] += batch_st[c] != 0;
  }
  // wave sums, then the workgroup's through LDS: three atomics per workgroup (one per wave
  // on one address serialised at the L2: 82 us for a 10^6-certificate call)
  __shared__ uint32_t s_v[4][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += (uint32_t)__shfl_xor((int)v[k], o);
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) s_v[threadIdx.x >> 6][k] = v[k];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    uint32_t t = 0;
    for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) t += s_v[wv][threadIdx.x];
    if (t) atomicAdd(&cnt[threadIdx.x], t);
  }
}

__global__ void k_grp_publish(uint32_t ngroups, uint32_t tag, uint32_t* __restrict__ cnt,
                              uint32_t* __restrict__ fb) {
  fb[1] = ngroups;
  fb[2] = cnt[0];
  fb[3] = tag;
  fb[4] = cnt[1];
  fb[5] = cnt[2];
  cnt[0] = cnt[1] = cnt[2] = 0;
  __threadfence_system();
  fb[0] = fb[0] + 1;   // sequence number, written last
}

hipError_t launch_group_feedback(const uint32_t* group_ok, uint64_t ncert, uint64_t K,
                                 uint32_t tag, const int32_t* batch_st, const int32_t* pre1,
                                 const int32_t* pre2, const int32_t* hdr_st, uint32_t* cnt,
                                 uint32_t* fb, hipStream_t stream) {
  const uint64_t ngroups = K && group_ok ? (ncert + K - 1) / K : 0;
  const uint64_t work = std::max(ngroups, ncert);
  const unsigned blocks = (unsigned)std::min<uint64_t>(256, std::max<uint64_t>(1, (work + 2047) / 2048));
  hipLaunchKernelGGL(k_grp_count, dim3(blocks), dim3(256), 0, stream, group_ok, ngroups, ncert,
                     batch_st, pre1, pre2, hdr_st, cnt);
  hipLaunchKernelGGL(k_grp_publish, dim3(1), dim3(1), 0, stream, (uint32_t)ngroups, tag, cnt, fb);
  return hipGetLastError();
}

size_t cert_groups_bytes(uint64_t ncert) {
  const uint64_t m = ncert ? ncert : 1;
  return a256(8 * (m + 1)) + a256(4 * m) + a256(4 * m);
}

// Certificate::verify's vote batches merged over groups of certificates:
// per group one Pippenger MSM of sum_i z_i R_i + sum_keys (sum c_i) A_key - (sum b_i) B over
// the votes of its certificates that passed every earlier check; group_ok[g] = 1 when it
// is the identity and no vote has a parse/decode flag. Returns with group_ok in scratch
// (the caller then runs launch_verify_batch with skip_group_ok for the per-certificate
// verdicts of the other groups). Random coefficients only.
hipError_t launch_cert_groups(const uint32_t* cert_digest, const uint64_t* cvo,
                              const uint64_t* host_cvo, uint64_t ncert, const uint32_t* pks,
                              const uint32_t* sigs, uint64_t nvotes, const z_key_t& zkey,
                              void* batch_ws, void* group_ws, const int32_t* pre1,
                              const int32_t* pre2, const int32_t* hdr_st,
                              const key_tables_t& keys, const ge* key_base, uint32_t nkeys,
                              uint64_t K, uint32_t** group_ok_out, hipStream_t stream) {
  if (ncert == 0 || nkeys > 256) return hipErrorInvalidValue;
  const uint64_t ngroups = (ncert + K - 1) / K;
  char* gp = static_cast<char*>(group_ws);
  uint64_t* gofs = reinterpret_cast<uint64_t*>(gp);
  uint32_t* ident = reinterpret_cast<uint32_t*>(gp + a256(8 * (ncert + 1)));
  uint32_t* group_ok = reinterpret_cast<uint32_t*>(gp + a256(8 * (ncert + 1)) + a256(4 * ncert));
  *group_ok_out = group_ok;
  hipLaunchKernelGGL(k_grp_setup, dim3((unsigned)((ngroups + 1 + 255) / 256)), dim3(256), 0,
                     stream, cvo, ncert, K, ngroups, gofs, ident, group_ok);
  const uint64_t cap = std::min<uint64_t>(nvotes + ncert, slice_units());
  bv_ws w;
  bv_layout(cap, static_cast<char*>(batch_ws), &w);
  w.pip_list = ident;   // every group of a slice, relative index = group - first group
  pip_group_t grp{cvo, ncert, K, pre1, pre2, hdr_st, keys.vote_key, keys.ok, key_base, nkeys,
                  group_ok};
  const uint32_t pmin = kPipMin;   // smaller groups stay with the per-certificate path
  auto gvotes = [&](uint64_t g) {
    return host_cvo[std::min((g + 1) * K, ncert)] - host_cvo[std::min(g * K, ncert)];
  };
  uint64_t g = 0;
  while (g < ngroups) {
    uint64_t e = g, votes = 0, pmax = 0;
    while (e < ngroups && (e == g || votes + gvotes(e) <= cap)) {
      votes += gvotes(e);
      pmax = std::max(pmax, gvotes(e));
      ++e;
    }
    if (votes > cap) return hipErrorInvalidValue;
    const uint64_t i0 = host_cvo[std::min(g * K, ncert)], i1 = host_cvo[std::min(e * K, ncert)];
    if (i1 > i0) {
      const hipError_t pe = launch_pip(cert_digest, gofs, g, e, i0, i1, pmin, e - g, pmax, pks,
                                       sigs, nullptr, zkey, w, nullptr, nullptr, grp, stream,
                                       w.chunk_start);
      if (pe != hipSuccess) return pe;
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    g = e;
  }
  return hipSuccess;
}


// ------------------------------------------------------------------ small certificate groups
// For streams whose big merged groups keep failing (invalid certificates spread through the
// stream: at 1 % every ~32k-vote group holds some), the adaptive policy (nw_api.cpp) checks
// the votes in groups of K certificates (a handful) with one keyed Straus MSM each and runs
// the per-certificate ladders only for the certificates of groups that fail — from the SAME
// per-vote items, so a failing group's fallback costs its ladders only:
//
//   sum_votes z_i R_i + sum_keys (sum c_i) A_key - (sum b_i) B == identity
//
// per slice of whole groups:
//   k_bv_items      (keyed) per vote: flags, k_i, z_i, c_i, b_i and the R table j*R_i
//   k_sgrp_keys     one wave per group: c_i summed per committee key (LDS), sum b_i, the
//                   group's flags; the used keys compacted into a list; counted votes marked
//   k_sgrp_ladder   one lane per (group, chunk): the 132-doubling keyed ladder over the
//                   chunk's counted votes (z_i by 4-bit windows over their R tables), its share
//                   of the key list (8-bit windows over the two key tables) and, chunk 0, -sum b
//   k_sgrp_combine  one lane per group: sum of its chunks, identity test -> group_ok
//   k_bv_plan_* / k_bv_expand / k_bv_chunks / k_bv_combine  the per-certificate verify_batch
//                   of every certificate in a failed group (settled ones get status Ok)
//
// A counted vote costs 33 additions here instead of 65 in its own certificate's ladder (the
// A term is paid per distinct key of the group, the doublings and B per group). Counted
// votes are those of certificates that passed every earlier check (as in
// launch_cert_groups); group_ok[g] = 1 when the sum is the identity and no counted vote has
// a flag. Every counted vote is keyed, so its A-table slots (0..7) are free: the key list
// lives in slot 0 of the group's votes 0..M-1 (M <= counted votes), the header in slot 1 of
// vote 0 (the fallback ladders read only R tables and the committee key tables).
namespace {

struct sgrp_hdr {
  uint32_t nkeys;    // M: distinct keys among the counted votes
  uint32_t flagged;  // OR of the counted votes' BF_* flags
  uint32_t bb[8];    // -sum b_i mod l, recoded to signed 8-bit digits
};
struct sgrp_key {
  uint32_t key;
  uint32_t c[8];     // sum of the key's c_i mod l, recoded to signed 8-bit digits
};
static_assert(sizeof(sgrp_hdr) <= sizeof(ge_cached) && sizeof(sgrp_key) <= sizeof(ge_cached),
              "small-group records must fit a table slot");

constexpr uint64_t kSgrpMaxCerts = 32;

__device__ __forceinline__ bool cert_decided(const int32_t* pre1, const int32_t* pre2,
                                             const int32_t* hdr_st, uint64_t c) {
  return pre1[c] != 0 || hdr_st[c] != 0 || pre2[c] != 0;
}

__global__ __launch_bounds__(64) void k_sgrp_keys(
    const uint64_t* __restrict__ cvo, uint64_t g0, uint64_t ncert, uint64_t K, uint64_t i0,
    uint32_t nkeys, const int32_t* __restrict__ pre1, const int32_t* __restrict__ pre2,
    const int32_t* __restrict__ hdr_st, bv_item* __restrict__ items,
    ge_cached* __restrict__ tabs) {
  __shared__ unsigned long long s_acc[256][8];
  __shared__ uint32_t s_cnt[256];
  const int tid = threadIdx.x;
  const uint64_t g = g0 + blockIdx.x;
  const uint64_t c0 = g * K, c1 = c0 + K < ncert ? c0 + K : ncert;
  const uint64_t v0 = cvo[c0], v1 = cvo[c1];
  if (v1 == v0) return;   // no votes: k_sgrp_combine settles the group
  for (uint32_t j = tid; j < nkeys; j += 64) {
    s_cnt[j] = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) s_acc[j][w] = 0;
  }
  __syncthreads();
  sc bsum;
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum.w[j] = 0;
  uint32_t flagged = 0;
  for (uint64_t v = v0 + tid; v < v1; v += 64) {
    const uint64_t c = batch_of(cvo, c0, c1, v);
    const bool counted = !cert_decided(pre1, pre2, hdr_st, c);
    items[v - i0].pad = counted ? 1u : 0u;   // k_sgrp_ladder adds counted votes only
    if (!counted) continue;
    const bv_item& it = items[v - i0];
    flagged |= it.flags;
    const uint32_t key = it.key;
    if (key == kNone || key >= nkeys) {   // cannot happen for a counted vote (k_cert_prepare)
      flagged |= BF_A_DECODE;
      continue;
    }
    // c_i from its signed-digit recoding (c + 0x80..80, no final carry since c < l)
    uint64_t borrow = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const uint64_t d = (uint64_t)it.c[w] - 0x80808080u - borrow;
      borrow = (d >> 63) & 1;
      atomicAdd(&s_acc[key][w], (unsigned long long)(uint32_t)d);
    }
    atomicAdd(&s_cnt[key], 1u);
    sc bi;
#pragma unroll
    for (int j = 0; j < 8; ++j) bi.w[j] = it.b[j];
    sc_add(bsum, bsum, bi);
  }
#pragma unroll 1
  for (int o = 32; o > 0; o >>= 1) {
    sc b;
#pragma unroll
    for (int j = 0; j < 8; ++j) b.w[j] = (uint32_t)__shfl_xor((int)bsum.w[j], o);
    sc_add(bsum, bsum, b);
    flagged |= (uint32_t)__shfl_xor((int)flagged, o);
  }
  __syncthreads();
  ge_cached* slots = tabs + 16 * (v0 - i0);
  uint32_t base = 0;
  for (uint32_t j0 = 0; j0 < nkeys; j0 += 64) {
    const uint32_t j = j0 + tid;
    const bool used = j < nkeys && s_cnt[j] != 0;
    const uint64_t mask = __ballot(used);
    if (used) {
      const uint32_t pos = base + (uint32_t)__popcll(mask & ((1ull << tid) - 1));
      uint32_t x[16];
      unsigned long long carry = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        carry += s_acc[j][w];
        x[w] = (uint32_t)carry;
        carry >>= 32;
      }
      x[8] = (uint32_t)carry;
      x[9] = (uint32_t)(carry >> 32);
#pragma unroll
      for (int w = 10; w < 16; ++w) x[w] = 0;
      sc s;
      sc_reduce512(s, x);
      sgrp_key e;
      e.key = j;
      sc_recode(e.c, s, 0x80808080u);
      *reinterpret_cast<sgrp_key*>(slots + 16 * (uint64_t)pos) = e;
    }
    base += (uint32_t)__popcll(mask);
  }
  if (tid == 0) {
    sgrp_hdr h;
    h.nkeys = base;
    h.flagged = flagged;
    sc nb;
    sc_neg(nb, bsum);
    sc_recode(h.bb, nb, 0x80808080u);
    *reinterpret_cast<sgrp_hdr*>(slots + 1) = h;
  }
}

// One lane per (group, chunk), nch chunks per group. Chunk k takes the group's votes
// [V k / nch, V (k + 1) / nch) (counted ones only), its keys m = k, k + nch, ... and (k = 0)
// the B term; its partial sum goes to out[(g - g0) nch + k] for k_sgrp_combine.
__global__ __launch_bounds__(256) void k_sgrp_ladder(
    const uint64_t* __restrict__ cvo, uint64_t g0, uint64_t g1, uint64_t ncert, uint64_t K,
    uint32_t nch, uint64_t i0, const bv_item* __restrict__ items,
    const ge_cached* __restrict__ tabs, const ge_niels_pad* __restrict__ ktabs, keyspec ks,
    bv_chunk_out* __restrict__ out) {
  __shared__ ge_niels s_btab[129];
  __shared__ ge_niels s_b128[129];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&g_bc.btab[0]);
    const uint32_t* src2 = reinterpret_cast<const uint32_t*>(&g_bc.b128[0]);
    uint32_t* dst = reinterpret_cast<uint32_t*>(s_btab);
    uint32_t* dst2 = reinterpret_cast<uint32_t*>(s_b128);
    for (int i = threadIdx.x; i < BT_WORDS; i += blockDim.x) {
      dst[i] = src[i];
      dst2[i] = src2[i];
    }
  }
  __syncthreads();
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nl = (g1 - g0) * nch;
  if ((uint64_t)blockIdx.x * blockDim.x >= nl) return;   // whole block past the end
  const bool inrange = lane < nl;
  const uint64_t gl = inrange ? lane : nl - 1;
  const uint64_t g = g0 + gl / nch;
  const uint32_t k = (uint32_t)(gl % nch);
  const uint64_t c0 = g * K, c1 = c0 + K < ncert ? c0 + K : ncert;
  const uint64_t v0 = cvo[c0], V = cvo[c1] - v0;
  const uint64_t t0 = v0 + V * k / nch, t1 = v0 + V * (k + 1) / nch;
  const bool live = inrange && V > 0;
  sgrp_hdr h{};
  if (live) h = *reinterpret_cast<const sgrp_hdr*>(tabs + 16 * (v0 - i0) + 1);
  const ge_cached* slots = tabs + 16 * (v0 - i0);
  ge acc;
  ge_identity(acc);
  const int W = wave_max_int(live ? 33 : 0);
#pragma unroll 1
  for (int j = W - 1; j >= 0; --j) {
    if (j != W - 1) {
#pragma unroll 1
      for (int t = 0; t < 3; ++t) ge_dbl(acc, acc, false);
      ge_dbl(acc, acc, true);
    }
    if (!live) continue;
#pragma unroll 1
    for (uint64_t t = t0; t < t1; ++t) {
      const bv_item* it = items + (t - i0);
      if (it->pad) add_entry(acc, tabs + 16 * (t - i0) + 8, digit4(it->z[j >> 3], j));
    }
    if ((j & 1) == 0 && j < 32) {
#pragma unroll 1
      for (uint32_t m = k; m < h.nkeys; m += nch) {
        const sgrp_key& e = *reinterpret_cast<const sgrp_key*>(slots + 16 * (uint64_t)m);
        const ge_niels_pad* kt = ktabs + ks.tab * (uint64_t)e.key;
        add_key_entry(acc, kt, digit8(e.c, j >> 1));
        add_key_entry(acc, kt + ks.half, digit8(e.c, 16 + (j >> 1)));
      }
      if (k == 0) {
        add_digit_niels(acc, s_btab, digit8(h.bb, j >> 1), true);
        add_digit_niels(acc, s_b128, digit8(h.bb, 16 + (j >> 1)), true);
      }
    }
  }
  if (!inrange) return;
  out[gl].P = acc;
}

// One lane per group: the sum of its chunks' points; group_ok = identity and no flags.
__global__ __launch_bounds__(256) void k_sgrp_combine(
    const uint64_t* __restrict__ cvo, uint64_t g0, uint64_t g1, uint64_t ncert, uint64_t K,
    uint32_t nch, uint64_t i0, const ge_cached* __restrict__ tabs,
    const bv_chunk_out* __restrict__ out, uint32_t* __restrict__ group_ok) {
  const uint64_t gl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g0 + gl >= g1) return;
  const uint64_t g = g0 + gl;
  const uint64_t c0 = g * K, c1 = c0 + K < ncert ? c0 + K : ncert;
  const uint64_t v0 = cvo[c0];
  if (cvo[c1] == v0) {   // no votes: nothing to check
    group_ok[g] = 1;
    return;
  }
  const sgrp_hdr& h = *reinterpret_cast<const sgrp_hdr*>(tabs + 16 * (v0 - i0) + 1);
  ge acc = out[gl * nch].P;
#pragma unroll 1
  for (uint32_t k = 1; k < nch; ++k) {
    ge_cached c;
    ge_to_cached(c, out[gl * nch + k].P, g_bc.k.d2);
    ge_add_cached(acc, acc, c, true);
  }
  group_ok[g] = (h.flagged == 0 && ge_is_identity(acc)) ? 1u : 0u;
}

}  // namespace

// Cost model (point additions per certificate), the per-vote items being
// common to both paths: a certificate's own keyed ladder costs q (33 + 32) + 151 (132
// doublings and 32 B additions); in a group of K it costs 33 per vote, its share of
// 32 per distinct key and 151 per group, plus, when the group fails (probability
// 1 - (1 - p)^K), its own ladder. K minimises that; *beats_per_cert says whether the best K
// is cheaper than the certificate's own ladder.
uint64_t cert_sgroup_size(const uint64_t* host_cvo, uint64_t ncert, uint64_t nkeys,
                          bool injected_z, double p_cert, bool* beats_per_cert) {
  if (beats_per_cert) *beats_per_cert = false;
  const char* m = getenv("NW_CERT_MERGE");
  if (injected_z || (m && m[0] == '0') || nkeys == 0 || nkeys > 256 || ncert == 0) return 0;
  const uint64_t nvotes = host_cvo[ncert] - host_cvo[0];
  uint64_t qmax = 0;
  for (uint64_t c = 0; c < ncert; ++c) qmax = std::max(qmax, host_cvo[c + 1] - host_cvo[c]);
  if (qmax == 0 || qmax >= kPipMin || nvotes == 0) return 0;
  const uint64_t kcap = std::max<uint64_t>(
      1, std::min<uint64_t>(kSgrpMaxCerts, slice_units() / (2 * (qmax + 1))));
  const uint64_t forced = env_u64("NW_CERT_SMALL_K", 0);
  if (forced) {
    if (beats_per_cert) *beats_per_cert = true;
    return std::min(forced, kcap);
  }
  const double q = (double)nvotes / (double)ncert;
  const double p = std::min(0.5, std::max(1e-5, p_cert));
  const double own = q * 65.0 + 151.0;
  uint64_t best = 1;
  double best_cost = 1e300;
  for (uint64_t K = 1; K <= kcap; ++K) {
    const double keys = std::min((double)nkeys, (double)K * q);
    const double fail = 1.0 - std::pow(1.0 - p, (double)K);
    const double cost = q * 33.0 + (32.0 * keys + 151.0) / (double)K + fail * own;
    if (cost < best_cost) { best_cost = cost; best = K; }
  }
  if (beats_per_cert) *beats_per_cert = best_cost < own;
  return best;
}

hipError_t launch_cert_sgroups(const uint32_t* cert_digest, const uint64_t* cvo,
                               const uint64_t* host_cvo, uint64_t ncert, const uint32_t* pks,
                               const uint32_t* sigs, uint64_t nvotes, const z_key_t& zkey,
                               void* batch_ws, void* group_ws, const int32_t* pre1,
                               const int32_t* pre2, const int32_t* hdr_st,
                               const key_tables_t& keys, uint32_t nkeys, uint64_t K,
                               double p_cert, int32_t* status, uint64_t* fail_index,
                               uint32_t** group_ok_out, hipStream_t stream) {
  if (ncert == 0 || nkeys > 256 || K == 0 || K > kSgrpMaxCerts || !keys.tabs || !keys.vote_key)
    return hipErrorInvalidValue;
  const uint64_t ngroups = (ncert + K - 1) / K;
  char* gp = static_cast<char*>(group_ws);
  uint32_t* group_ok = reinterpret_cast<uint32_t*>(gp + a256(8 * (ncert + 1)) + a256(4 * ncert));
  *group_ok_out = group_ok;
  const uint64_t cap = std::min<uint64_t>(nvotes + ncert, slice_units());
  bv_ws w;
  bv_layout(cap, static_cast<char*>(batch_ws), &w);
  const batch_skip_t nosk{nullptr, 1}, sk{group_ok, K};
  uint64_t qmax = 0;
  for (uint64_t c = 0; c < ncert; ++c) qmax = std::max(qmax, host_cvo[c + 1] - host_cvo[c]);
  // group chunks: about Cg votes each, so that they fill the chip (~2 waves per SIMD) while
  // the 132 doublings are shared by as many votes as possible (balanced split per group);
  // fallback chunks as in launch_verify_batch
  const uint64_t target_lanes = 256ull * 4 * 2 * 64;
  const uint64_t Cg = env_u64("NW_SGRP_CHUNK",
                              std::min<uint64_t>(32, std::max<uint64_t>(4, nvotes / target_lanes)));
  const uint64_t kq = std::min(K, ncert) * qmax;
  const uint32_t nch = (uint32_t)std::min<uint64_t>(cap, std::max<uint64_t>(1, (kq + Cg - 1) / Cg));
  // Fallback chunks: only the failed groups' certificates run (about a fraction
  // 1 - (1 - p)^K of a slice's votes), so they are cut small enough to fill the chip on
  // their own: a certificate of q votes split over several chunks costs a few more doublings,
  // one chunk per certificate leaves most SIMDs idle at N = 100 (67-vote ladders).
  const double fail = 1.0 - std::pow(1.0 - std::min(0.5, std::max(0.0, p_cert)), (double)K);
  const uint64_t fb_votes = (uint64_t)(fail * (double)std::min(nvotes, cap));
  uint32_t C = (uint32_t)std::min<uint64_t>(kMaxChunk, std::max<uint64_t>(4, fb_votes / target_lanes));
  C = (uint32_t)std::min<uint64_t>(kMaxChunk, env_u64("NW_BATCH_CHUNK", C));
  auto cert_at = [&](uint64_t g) { return std::min(g * K, ncert); };
  uint64_t g = 0;
  while (g < ngroups) {
    // slice [g, e) of whole groups: votes + certificates and the group chunks fit the workspace
    uint64_t e = g;
    while (e < ngroups) {
      const uint64_t b = cert_at(g), be = cert_at(e + 1);
      if (e > g && ((host_cvo[be] - host_cvo[b]) + (be - b) > cap || (e + 1 - g) * nch > cap))
        break;
      ++e;
    }
    const uint64_t b = cert_at(g), be = cert_at(e);
    const uint64_t i0 = host_cvo[b], i1 = host_cvo[be];
    if ((i1 - i0) + (be - b) > cap || (e - g) * nch > cap) return hipErrorInvalidValue;
    uint64_t chunks = 0, multi = 0;   // host upper bounds for the fallback (every certificate)
    for (uint64_t c = b; c < be; ++c) {
      const uint64_t kb = (host_cvo[c + 1] - host_cvo[c] + C - 1) / C;
      chunks += kb;
      multi += kb != 1;
    }
    if (i1 > i0)
      hipLaunchKernelGGL(k_bv_items, dim3((unsigned)((i1 - i0 + 255) / 256)), dim3(256), 0,
                         stream, cert_digest, cvo, b, be, i0, i1, kPipMin, pks, sigs, nullptr,
                         zkey, w.items, w.tabs, keys, nosk);
    hipLaunchKernelGGL(k_sgrp_keys, dim3((unsigned)(e - g)), dim3(64), 0, stream, cvo, g, ncert,
                       K, i0, nkeys, pre1, pre2, hdr_st, w.items, w.tabs);
    hipLaunchKernelGGL(k_sgrp_ladder, dim3((unsigned)(((e - g) * nch + 255) / 256)), dim3(256),
                       0, stream, cvo, g, e, ncert, K, nch, i0, w.items, w.tabs, keys.tabs,
                       keys.ks, w.outs);
    hipLaunchKernelGGL(k_sgrp_combine, dim3((unsigned)((e - g + 255) / 256)), dim3(256), 0,
                       stream, cvo, g, e, ncert, K, nch, i0, w.tabs, w.outs, group_ok);
    // the certificates of failed groups: their own verify_batch from the same items
    const unsigned nblk = (unsigned)((be - b + 1023) / 1024);
    hipLaunchKernelGGL(k_bv_plan_local, dim3(nblk), dim3(1024), 0, stream, cvo, b, be, C,
                       kPipMin, sk, w.plan_tot);
    hipLaunchKernelGGL(k_bv_plan_top, dim3(1), dim3(1024), 0, stream, nblk, be - b, w.plan_tot,
                       w.chunk_start);
    hipLaunchKernelGGL(k_bv_plan_apply, dim3(nblk), dim3(1024), 0, stream, cvo, b, be, C, kPipMin,
                       sk, w.plan_tot, w.chunk_start, w.multi, w.multi_first, w.pip_list, status,
                       fail_index);
    if (chunks) {
      hipLaunchKernelGGL(k_bv_expand, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                         stream, cvo, b, be - b, (uint32_t)chunks, w.chunk_start, w.chunks);
      hipLaunchKernelGGL(k_bv_chunks, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                         stream, w.chunks, (uint32_t)chunks, cvo, b, i0, w.items, w.tabs,
                         keys.tabs, keys.ks, w.outs, status, fail_index, w.chunk_start + (be - b));
    }
    if (multi)
      hipLaunchKernelGGL(k_bv_combine,
                         dim3((unsigned)std::min<uint64_t>(multi, kCombineMaxBlocks)), dim3(256),
                         0, stream, w.multi, w.multi_first, (uint32_t)multi, cvo, b, C, w.outs,
                         status, fail_index, w.plan_tot + 3 * nblk + 1);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    g = e;
  }
  return hipSuccess;
}

}  // namespace nw
