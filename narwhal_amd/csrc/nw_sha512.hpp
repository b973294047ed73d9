// nw_sha512.hpp — FIPS 180-4 SHA-512 compression for gfx950.
//
// 64-bit words live as 32-bit halves: a rotation is two v_alignbit_b32, Ch/Maj/xor3 are a
// single v_bitop3_b32 each, additions are v_lshl_add_u64. Round constants are uniform
// (wave-wide) and come from scalar loads.
#pragma once
#include "nw_field.hpp"

namespace nw {

// FIPS 180-4 round constants, shared by the device copy below and the host path (nw_host.cpp).
#define NW_SHA512_K_INIT {                                                                    \
  0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, \
  0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, \
  0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, \
  0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL, \
  0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL, \
  0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, \
  0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, \
  0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, \
  0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL, \
  0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL, \
  0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, \
  0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, \
  0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, \
  0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL, \
  0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL, \
  0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, \
  0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, \
  0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL, \
  0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL, \
  0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL \
}

__constant__ static const uint64_t SHA512_K[80] = NW_SHA512_K_INIT;

static constexpr uint64_t SHA512_H0[8] = {
  0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
  0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

// (lo, hi) -> u64 as a plain register pair (no shift/or: the compiler would otherwise turn
// `(hi << 32) | lo` into a half-rate v_lshl_add_u64).
typedef uint32_t nw_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) {
  return __builtin_bit_cast(uint64_t, nw_u32x2{lo, hi});
}

__device__ __forceinline__ uint64_t rotr64(uint64_t x, const int n) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rlo, rhi;
  if (n < 32) {
    rlo = __builtin_amdgcn_alignbit(hi, lo, n);
    rhi = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    rlo = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rhi = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return pack64(rlo, rhi);
}
__device__ __forceinline__ uint64_t shr64(uint64_t x, const int n) {   // n < 32
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack64(__builtin_amdgcn_alignbit(hi, lo, n), hi >> n);
}
__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// Three-input bitwise functions as one v_bitop3_b32 per 32-bit half (the compiler does not
// form them from ^/&/| on its own). LUT index = (x << 2) | (y << 1) | z.
template <int LUT>
__device__ __forceinline__ uint64_t bitop3_64(uint64_t x, uint64_t y, uint64_t z) {
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)x, (uint32_t)y, (uint32_t)z, LUT);
  const uint32_t hi = __builtin_amdgcn_bitop3_b32((uint32_t)(x >> 32), (uint32_t)(y >> 32),
                                                  (uint32_t)(z >> 32), LUT);
  return pack64(lo, hi);
}
__device__ __forceinline__ uint64_t xor3_64(uint64_t x, uint64_t y, uint64_t z) {
  return bitop3_64<0x96>(x, y, z);
}
__device__ __forceinline__ uint64_t maj64(uint64_t x, uint64_t y, uint64_t z) {
  return bitop3_64<0xE8>(x, y, z);
}
__device__ __forceinline__ uint64_t ch64(uint64_t x, uint64_t y, uint64_t z) {
  return bitop3_64<0xCA>(x, y, z);   // x ? y : z
}

// 16 rounds; FIRST = the block words themselves, else the schedule is advanced in place.
template <bool FIRST>
__device__ __forceinline__ void sha512_16rounds(uint64_t& a, uint64_t& b, uint64_t& c,
                                                uint64_t& d, uint64_t& e, uint64_t& f,
                                                uint64_t& g, uint64_t& h, uint64_t w[16],
                                                int r) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    uint64_t wj;
    if (FIRST) {
      wj = w[j];
    } else {
      const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
      const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
      wj = w[j] + s0 + w[(j + 9) & 15] + s1;
      w[j] = wj;
    }
    const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
    const uint64_t ch = ch64(e, f, g);
    const uint64_t t1 = h + S1 + ch + SHA512_K[r + j] + wj;
    const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
    const uint64_t maj = maj64(a, b, c);
    const uint64_t t2 = S0 + maj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
}

// One compression. w[16] = the block as big-endian 64-bit words (consumed as the
// message-schedule window).
__device__ __forceinline__ void sha512_compress(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
           h = st[7];
  sha512_16rounds<true>(a, b, c, d, e, f, g, h, w, 0);
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) sha512_16rounds<false>(a, b, c, d, e, f, g, h, w, r);
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g;
  st[7] += h;
}

__device__ __forceinline__ void sha512_init(uint64_t st[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = SHA512_H0[i];
}

// Tail block(s): message bytes [base, len) followed by 0x80, zeros, and (if last) the
// 128-bit big-endian bit length in the final 16 bytes. Reads only the aligned dwords that
// hold a message byte (such a dword never crosses a page, so nothing past the buffer can
// fault) and masks the bytes at or beyond len.
__device__ __forceinline__ void load_block_tail(uint64_t w[16], const uint8_t* msg, uint64_t base,
                                                uint64_t len, bool last) {
  const uintptr_t a0 = (uintptr_t)(msg + base);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a0 & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a0 & 3) * 8;
  // message bytes in this block; negative for a padding-only block after the 0x80 block
  const int64_t rem = (int64_t)len - (int64_t)base;
  // dword q[i] covers block bytes [4 i - sh/8, 4 i - sh/8 + 4). Every load is issued before
  // any is used: from pinned host memory (the small-job kernel) a load is a ~1-2 us round
  // trip, and 33 of them one after another cost a header's tail block ~40 us.
  uint32_t qd[33];
#pragma unroll
  for (int i = 0; i < 33; ++i) {
    const int64_t first = 4 * (int64_t)i - (int64_t)(sh >> 3);   // block byte of q[i]'s byte 0
    qd[i] = first < rem ? q[i] : 0u;
  }
  uint32_t prev = 0;
#pragma unroll
  for (int i = 0; i < 33; ++i) {
    const uint32_t cur = qd[i];
    if (i > 0) {
      // block dword i-1 = bytes [4(i-1), 4i): LE word realigned from q[i-1], q[i]
      uint32_t lo = __builtin_amdgcn_alignbit(cur, prev, sh);
      const int64_t k0 = 4 * (int64_t)(i - 1);                 // its first block byte
      // keep bytes < rem, put 0x80 at byte rem
      uint32_t keep = 0, pad = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t pos = k0 + b;
        keep |= (pos < rem ? 0xffu : 0u) << (8 * b);
        pad |= (pos == rem ? 0x80u : 0u) << (8 * b);
      }
      lo = (lo & keep) | pad;
      const int wi = (i - 1) >> 1;
      const uint64_t be = (uint64_t)__builtin_bswap32(lo);
      if ((i - 1) & 1) w[wi] = (w[wi] & 0xffffffff00000000ull) | be;
      else w[wi] = be << 32;
    }
    prev = cur;
  }
  if (last) {
    w[14] = len >> 61;
    w[15] = len << 3;
  }
}

// The 33 aligned dwords covering the 128-byte block at p (the 33rd only when p is not
// 4-byte aligned; only dwords that contain message bytes), and their realignment by the
// byte offset into 16 big-endian words — two halves, so the next block's loads can be issued
// before this block's compression.
__device__ __forceinline__ void load_block_raw(uint32_t d[33], const uint8_t* p) {
  // The integer round trip makes these flat_load_dwordx4; keeping the global address space
  // (global_load_dwordx4) measured 4 % slower (1,231 vs 1,279 GB/s, different schedule).
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
#pragma unroll
  for (int i = 0; i < 32; ++i) d[i] = q[i];
  d[32] = (a & 3) ? q[32] : 0u;
}
__device__ __forceinline__ void block_from_raw(uint64_t w[16], const uint32_t d[33], uint32_t sh) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t lo = __builtin_amdgcn_alignbit(d[2 * i + 1], d[2 * i], sh);
    const uint32_t hi = __builtin_amdgcn_alignbit(d[2 * i + 2], d[2 * i + 1], sh);
    w[i] = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
  }
}


// Digest(Sha512(msg[0..len))[..32]) on one lane into out[8] (LE words). Full blocks are
// double-buffered: block k + 1's loads are issued before block k's 80 rounds, so a lone
// wave per SIMD does not stall on each block's memory latency (HBM, or pinned host memory
// for the small-job kernel, nw_small.hip).
__device__ __forceinline__ void sha512_digest32_lane(const uint8_t* msg, uint64_t len,
                                                     uint32_t* out) {
  const uint64_t nblocks = (len + 17 + 127) / 128;
  const uint64_t nfull = len / 128;   // blocks entirely inside the message
  const uint32_t sh = (uint32_t)((uintptr_t)msg & 3) * 8;
  uint64_t st[8], w[16];
  sha512_init(st);
  uint32_t d[33];
  if (nfull) load_block_raw(d, msg);
#pragma unroll 1
  for (uint64_t k = 0; k < nfull; ++k) {
    block_from_raw(w, d, sh);
    if (k + 1 < nfull) load_block_raw(d, msg + 128 * (k + 1));
    sha512_compress(st, w);
  }
#pragma unroll 1
  for (uint64_t k = nfull; k < nblocks; ++k) {
    load_block_tail(w, msg, 128 * k, len, k + 1 == nblocks);
    sha512_compress(st, w);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    out[2 * j] = __builtin_bswap32((uint32_t)(st[j] >> 32));
    out[2 * j + 1] = __builtin_bswap32((uint32_t)st[j]);
  }
}

// SHA-512 of the 96-byte R || A || M (one block) -> 16 LE words of the digest.
__device__ __forceinline__ void sha512_hram96(uint32_t x[16], const uint32_t R[8],
                                              const uint32_t A[8], const uint32_t M[8]) {
  uint64_t w[16], st[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = ((uint64_t)__builtin_bswap32(R[2 * i]) << 32) | __builtin_bswap32(R[2 * i + 1]);
    w[4 + i] = ((uint64_t)__builtin_bswap32(A[2 * i]) << 32) | __builtin_bswap32(A[2 * i + 1]);
    w[8 + i] = ((uint64_t)__builtin_bswap32(M[2 * i]) << 32) | __builtin_bswap32(M[2 * i + 1]);
  }
  w[12] = 0x8000000000000000ULL;
  w[13] = 0;
  w[14] = 0;
  w[15] = 96 * 8;
  sha512_init(st);
  sha512_compress(st, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x[2 * i] = __builtin_bswap32((uint32_t)(st[i] >> 32));
    x[2 * i + 1] = __builtin_bswap32((uint32_t)st[i]);
  }
}

// Digest(Sha512(x32 || u64 LE || y32)[..32]): Vote::digest / Certificate::digest
// (primary/src/messages.rs:145-153, 226-234; 72 bytes, one block).
__device__ __forceinline__ void sha512_digest72(uint32_t out[8], const uint32_t x[8],
                                                uint64_t round, const uint32_t y[8]) {
  uint64_t w[16], st[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = ((uint64_t)__builtin_bswap32(x[2 * i]) << 32) | __builtin_bswap32(x[2 * i + 1]);
    w[5 + i] = ((uint64_t)__builtin_bswap32(y[2 * i]) << 32) | __builtin_bswap32(y[2 * i + 1]);
  }
  w[4] = __builtin_bswap64(round);
  w[9] = 0x8000000000000000ULL;
#pragma unroll
  for (int i = 10; i < 15; ++i) w[i] = 0;
  w[15] = 72 * 8;
  sha512_init(st);
  sha512_compress(st, w);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = __builtin_bswap32((uint32_t)(st[i] >> 32));
    out[2 * i + 1] = __builtin_bswap32((uint32_t)st[i]);
  }
}

}  // namespace nw
