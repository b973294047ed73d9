// nw_chacha.hpp — ChaCha20 keystream blocks for the batch coefficients z_i: rand 0.7's
// StdRng is ChaCha20, the reference draws z_i from thread_rng; here the key is
// 32 bytes from the OS CSPRNG per call (or the caller's), block i / 4 of the stream gives
// z_i for i, 4 .. 4 + 3.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace nw {

__device__ __forceinline__ uint32_t chacha_rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// z_i = ChaCha20(key, nonce, block i/4) bytes [16 (i%4), 16 (i%4) + 16) (DJB layout).
__device__ inline void chacha20_z(uint32_t z[4], const uint32_t key[8], uint64_t nonce, uint64_t i) {
  const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1],
                          key[2], key[3], key[4], key[5], key[6], key[7], (uint32_t)(i >> 2),
                          (uint32_t)(i >> 34), (uint32_t)nonce, (uint32_t)(nonce >> 32)};
  uint32_t x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = s[j];
#define NW_QR(a, b, c, d)                                                   \
  x[a] += x[b]; x[d] ^= x[a]; x[d] = chacha_rotl32(x[d], 16); x[c] += x[d];        \
  x[b] ^= x[c]; x[b] = chacha_rotl32(x[b], 12); x[a] += x[b]; x[d] ^= x[a];        \
  x[d] = chacha_rotl32(x[d], 8); x[c] += x[d]; x[b] ^= x[c]; x[b] = chacha_rotl32(x[b], 7);
#pragma unroll 1
  for (int r = 0; r < 10; ++r) {
    NW_QR(0, 4, 8, 12) NW_QR(1, 5, 9, 13) NW_QR(2, 6, 10, 14) NW_QR(3, 7, 11, 15)
    NW_QR(0, 5, 10, 15) NW_QR(1, 6, 11, 12) NW_QR(2, 7, 8, 13) NW_QR(3, 4, 9, 14)
  }
#undef NW_QR
  const int q = (int)(i & 3) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t v = x[0] + s[0];
#pragma unroll
    for (int t = 1; t < 16; ++t) v = (q + j == t) ? x[t] + s[t] : v;
    z[j] = v;
  }
}

}  // namespace nw
