// nw_committee.hpp — config::Committee lookups on the device (config/src/lib.rs:139-173):
// BTreeMap<PublicKey, Authority>::get as a binary search over the sorted 32-byte keys, stake,
// and the committee staged in LDS. Shared by the bulk message kernels (nw_cert.hip) and the
// small-job kernel (nw_small.hip).
#pragma once
#include "nw_kernels.h"

namespace nw {

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Committee lookup (BTreeMap<PublicKey, Authority>::get): binary search over the sorted
// 32-byte keys; -1 if absent. key = 8 little-endian words of the public key bytes.
__device__ inline int committee_find(const cert_committee_t& c, const uint32_t key[8]) {
  uint32_t kb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) kb[j] = __builtin_bswap32(key[j]);   // lexicographic order
  int lo = 0, hi = (int)c.nauth - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const uint32_t* m = c.pks + 8 * (size_t)mid;
    int cmp = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t mb = __builtin_bswap32(m[j]);
      if (cmp == 0 && mb != kb[j]) cmp = mb < kb[j] ? -1 : 1;
    }
    if (cmp == 0) return mid;
    if (cmp < 0) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

__device__ __forceinline__ uint32_t committee_stake(const cert_committee_t& c, int a) {
  return a < 0 ? 0u : c.stakes[a];
}

// The committee's sorted keys and stakes staged in LDS for committees of up to
// kLdsAuth members (8.5 KB): the per-vote binary searches then chain LDS reads instead of
// ~6 dependent global loads per vote (k_cert_prepare at N = 50: ~140 us per small job,
// a lane walks its certificate's 50 votes).
constexpr uint32_t kLdsAuth = 256;
__device__ __forceinline__ cert_committee_t committee_to_lds(const cert_committee_t& com,
                                                            uint32_t* s_pks,
                                                            uint32_t* s_stakes) {
  cert_committee_t c = com;
  if (com.nauth <= kLdsAuth) {
    for (uint32_t k = threadIdx.x; k < 8 * (uint32_t)com.nauth; k += blockDim.x)
      s_pks[k] = com.pks[k];
    for (uint32_t k = threadIdx.x; k < (uint32_t)com.nauth; k += blockDim.x)
      s_stakes[k] = com.stakes[k];
    c.pks = s_pks;
    c.stakes = s_stakes;
  }
  __syncthreads();
  return c;
}

}  // namespace nw
