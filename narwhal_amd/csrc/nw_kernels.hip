// nw_kernels.hip — gfx950 kernels for Narwhal's crypto hot path.
//
//   k_sha512_digest32     Digest(Sha512(m)[..32]) for many messages, one lane per message
//                         (worker/src/processor.rs:38, primary/src/messages.rs:70-84 ...).
//   k_verify_strict       crypto::Signature::verify (crypto/src/lib.rs:200-204), one lane per
//                         signature: decompress A and R, small-order tests, k = H(R||A||M)
//                         mod l, [s]B + [k](-A) by a joint signed-window ladder (A table in
//                         per-lane scratch, 8-bit B table in LDS), projective compare with R.
//   (crypto::Signature::verify_batch lives in nw_batch.hip.)
//
// Everything here is integer VALU work; no MFMA (modular arithmetic is not a contraction).
#include "nw_kernels.h"
#include "nw_point.hpp"
#include "nw_scalar.hpp"
#include "nw_sha512.hpp"
#include "nw_ladder.hpp"
#include "nw_consts.hpp"

#include <mutex>

namespace nw {

struct dev_consts {
  curve_consts k;
  ge_niels btab[129];   // j * B, j = 0..128, affine niels (signed 8-bit windows)
};

__constant__ dev_consts g_consts;

static constexpr int BT_WORDS = 129 * 30;

// ---------------------------------------------------------------------------------------
// Small helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Copy the B table from constant memory into LDS (all threads of the block).
__device__ __forceinline__ void load_btab(ge_niels* s_btab) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&g_consts.btab[0]);
  uint32_t* dst = reinterpret_cast<uint32_t*>(s_btab);
  for (int i = threadIdx.x; i < BT_WORDS; i += blockDim.x) dst[i] = src[i];
}

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
// Loads 128 bytes starting at byte address p (any alignment) as 16 big-endian u64 words.
// Only dwords that contain message bytes are read (no over-read past the message).
__device__ __forceinline__ void load_block_full(uint64_t w[16], const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  uint32_t d[33];
#pragma unroll
  for (int i = 0; i < 32; ++i) d[i] = q[i];
  d[32] = sh ? q[32] : 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    // little-endian message dwords, realigned by the byte offset
    const uint32_t lo = __builtin_amdgcn_alignbit(d[2 * i + 1], d[2 * i], sh);
    const uint32_t hi = __builtin_amdgcn_alignbit(d[2 * i + 2], d[2 * i + 1], sh);
    w[i] = ((uint64_t)bswap32(lo) << 32) | bswap32(hi);
  }
}

// Tail block(s): message bytes [base, len) followed by 0x80, zeros, and (if last) the
// 128-bit big-endian bit length in the final 16 bytes.
__device__ __forceinline__ void load_block_tail(uint64_t w[16], const uint8_t* msg, uint64_t base,
                                                uint64_t len, bool last) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    uint64_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t pos = base + 8 * i + b;
      uint32_t byte = 0;
      if (pos < len) byte = msg[pos];
      else if (pos == len) byte = 0x80;
      v = (v << 8) | byte;
    }
    w[i] = v;
  }
  if (last) {
    w[14] = len >> 61;
    w[15] = len << 3;
  }
}

__global__ __launch_bounds__(256) void k_sha512_digest32(const uint8_t* __restrict__ data,
                                                         const uint64_t* __restrict__ offsets,
                                                         const uint64_t* __restrict__ lengths,
                                                         uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* msg = data + offsets[i];
  const uint64_t len = lengths ? lengths[i] : offsets[i + 1] - offsets[i];
  const uint64_t nblocks = (len + 17 + 127) / 128;
  const uint64_t nfull = len / 128;   // blocks entirely inside the message
  uint64_t st[8], w[16];
  sha512_init(st);
#pragma unroll 1
  for (uint64_t k = 0; k < nfull; ++k) {
    load_block_full(w, msg + 128 * k);
    sha512_compress(st, w);
  }
#pragma unroll 1
  for (uint64_t k = nfull; k < nblocks; ++k) {
    load_block_tail(w, msg, 128 * k, len, k + 1 == nblocks);
    sha512_compress(st, w);
  }
  uint32_t* o = out + 8 * i;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[2 * j] = bswap32((uint32_t)(st[j] >> 32));
    o[2 * j + 1] = bswap32((uint32_t)st[j]);
  }
}

// ---------------------------------------------------------------------------------------
// Strict verification
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int strict_status(bool s_high, bool okA, bool s_canon, bool okR,
                                             bool smallR, bool smallA, bool eq) {
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

__global__ __launch_bounds__(256) void k_verify_strict(const uint32_t* __restrict__ msgs,
                                                       uint32_t msg_stride_words,
                                                       const uint32_t* __restrict__ pks,
                                                       const uint32_t* __restrict__ sigs,
                                                       uint64_t n, int32_t* __restrict__ status,
                                                       uint64_t* __restrict__ bitmap) {
  __shared__ ge_niels s_btab[129];
  load_btab(s_btab);
  __syncthreads();
  const uint64_t gi = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = gi < n;
  const uint64_t i = active ? gi : n - 1;
  const curve_consts& K = g_consts.k;

  uint32_t Aw[8], Rw[8], Sw[8], Mw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    Aw[j] = pks[8 * i + j];
    Rw[j] = sigs[16 * i + j];
    Sw[j] = sigs[16 * i + 8 + j];
    Mw[j] = msgs[(uint64_t)msg_stride_words * i + j];
  }
  const bool s_high = (Sw[7] >> 29) != 0;
  sc s;
#pragma unroll
  for (int j = 0; j < 8; ++j) s.w[j] = Sw[j];
  const bool s_canon = sc_is_canonical(s);

  ge A, R;
  const bool okA = ge_frombytes(A, Aw, K);
  const bool okR = ge_frombytes(R, Rw, K);
  const bool smallA = ge_is_small_order(A);
  const bool smallR = ge_is_small_order(R);

  uint32_t hx[16];
  hram96(hx, Rw, Aw, Mw);
  sc k;
  sc_reduce512(k, hx);

  // [s]B + [k](-A)
  ge minusA;
  ge_neg(minusA, A);
  ge_cached tab[9];
  build_table9(tab, minusA, K.d2);
  sc s_use = s;
  if (!s_canon || s_high) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s_use.w[j] = 0;   // keep digits in range; verdict is Err anyway
  }
  ge acc;
  dsm_var_base(acc, tab, k, s_use, s_btab);
  const bool eq = ge_eq_affine(acc, R);

  const int st = strict_status(s_high, okA, s_canon, okR, smallR, smallA, eq);
  if (active) status[gi] = st;
  const uint64_t mask = __ballot(active && st == NW_OK);
  if ((threadIdx.x & 63) == 0 && gi < n) bitmap[gi >> 6] = mask;
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

// ---------------------------------------------------------------------------------------
// Host side: constants and launchers
// ---------------------------------------------------------------------------------------
namespace nw {

hipError_t upload_consts() {
  static dev_consts host;
  static std::once_flag once;
  std::call_once(once, [] { compute_consts(host.k, host.btab); });
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_consts), &host, sizeof(host), 0,
                                   hipMemcpyHostToDevice);
  return e != hipSuccess ? e : upload_batch_consts();
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

hipError_t launch_verify_strict(const uint32_t* msgs, uint32_t msg_stride_words,
                                const uint32_t* pks, const uint32_t* sigs, uint64_t n,
                                int32_t* status, uint64_t* bitmap, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_verify_strict, dim3(grid_for(n, 256)), dim3(256), 0, stream, msgs,
                     msg_stride_words, pks, sigs, n, status, bitmap);
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
