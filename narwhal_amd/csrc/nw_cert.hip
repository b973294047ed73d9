// nw_cert.hip — primary message checks around the verification kernels.
//
//   k_cert_prepare    one lane per Header / Certificate (primary/src/messages.rs:48-67,
//                     189-215): header id == Sha512(header bytes)[..32] (the digest comes
//                     from k_sha512_digest32), committee checks (stake, worker ids, vote
//                     reuse / stake / quorum, config/src/lib.rs:148-173), genesis rule, and
//                     Certificate::digest = Sha512(id || round || origin)[..32] (226-234).
//   k_cert_finalize   first failure in the reference's order, combining those checks with
//                     the header's strict verdict (k_verify_strict) and the votes' batch
//                     verdict (k_batch_*).
//   k_vote_prepare    Vote::verify (131-153): stake(author) > 0, Vote::digest and the
//                     author's committee index (for the keyed comb).
//   k_vote_finalize
//
// These are byte/integer bookkeeping kernels (a few hundred bytes per item); the
// arithmetic lives in nw_kernels.hip.
#include "nw_kernels.h"
#include "nw_sha512.hpp"
#include "nw_committee.hpp"

namespace nw {

// One lane per vote: the committee index of the vote's key (vote_key, kNoKey when absent),
// so that k_cert_prepare's lanes, which walk their certificate's votes in order, read one
// word per vote instead of running a dependent binary search per vote (committees of up to
// kLdsAuth; larger ones keep the in-loop lookup). Every vote gets its index, also votes
// after a certificate's first failed check: those certificates are settled by that check
// (Certificate::verify returns at the first failure, messages.rs:199-215), so their votes'
// signature verdicts are never read.
__global__ __launch_bounds__(256) void k_vote_keys(cert_committee_t com_g, uint64_t nv,
                                                   const uint32_t* __restrict__ vote_pks,
                                                   uint32_t* __restrict__ vote_key) {
  __shared__ uint32_t s_pks[8 * kLdsAuth], s_stakes[kLdsAuth];
  const cert_committee_t com = committee_to_lds(com_g, s_pks, s_stakes);
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nv) return;
  uint32_t pk[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) pk[j] = vote_pks[8 * v + j];
  const int a = committee_find(com, pk);
  vote_key[v] = a >= 0 ? (uint32_t)a : kNoKey;
}

__global__ __launch_bounds__(256) void k_cert_prepare(cert_committee_t com_g, cert_stream_t cs,
                                                      int headers_only,
                                                      const uint32_t* __restrict__ hdr_digest,
                                                      uint32_t* __restrict__ authors,
                                                      uint32_t* __restrict__ cert_digest,
                                                      int32_t* __restrict__ pre1,
                                                      int32_t* __restrict__ pre2,
                                                      uint64_t* __restrict__ idx1,
                                                      uint64_t* __restrict__ idx2,
                                                      uint32_t* __restrict__ vote_key,
                                                      uint32_t* __restrict__ author_key,
                                                      uint32_t* __restrict__ vote_cert,
                                                      int keys_pre) {
  __shared__ uint32_t s_pks[8 * kLdsAuth], s_stakes[kLdsAuth];
  const cert_committee_t com = committee_to_lds(com_g, s_pks, s_stakes);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cs.n) return;
  const uint8_t* h = cs.header_bytes + cs.header_offsets[i];
  uint32_t author[8], id[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    author[j] = ld_le32(h + 4 * j);
    id[j] = cs.ids[8 * i + j];
  }
  const uint64_t round = (uint64_t)ld_le32(h + 32) | ((uint64_t)ld_le32(h + 36) << 32);
#pragma unroll
  for (int j = 0; j < 8; ++j) authors[8 * i + j] = author[j];

  const int a = committee_find(com, author);
  if (author_key) author_key[i] = a >= 0 ? (uint32_t)a : kNoKey;
  int32_t p1 = 0, p2 = 0;
  uint64_t x1 = 0, x2 = 0;
  // Certificate::verify: genesis(committee).contains(self) compares (header.id, round,
  // origin) with Certificate::genesis = (Digest::default(), 0, name) for every authority.
  uint32_t idor = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) idor |= id[j];
  const bool genesis = !headers_only && idor == 0 && round == 0 && a >= 0;
  // Header::verify, in order: id well formed, author stake, worker ids.
  bool id_ok = true;
#pragma unroll
  for (int j = 0; j < 8; ++j) id_ok &= hdr_digest[8 * i + j] == id[j];
  if (!id_ok) {
    p1 = NW_DAG_INVALID_HEADER_ID;
  } else if (committee_stake(com, a) == 0) {
    p1 = NW_DAG_UNKNOWN_AUTHORITY;
    x1 = ~0ULL;
  } else {
    const uint32_t np = cs.payload_counts[i];
    const uint64_t wb = com.worker_offsets[a], we = com.worker_offsets[a + 1];
    for (uint32_t e = 0; e < np && p1 == 0; ++e) {
      const uint32_t wid = ld_le32(h + 40 + 36 * (uint64_t)e + 32);
      bool found = false;
      for (uint64_t w = wb; w < we; ++w) found |= com.worker_ids[w] == wid;
      if (!found) { p1 = NW_DAG_MALFORMED_HEADER; x1 = e; }
    }
  }
  if (!headers_only) {
    // Quorum over the votes (messages.rs:199-211): reuse, then stake, per vote in order.
    // Committee::quorum_threshold and the vote weight are config::Stake = u32 sums (wrapping
    // as in a release build).
    uint32_t total = 0;
    for (uint64_t q = 0; q < com.nauth; ++q) total += com.stakes[q];
    const uint32_t quorum = 2u * total / 3u + 1u;
    const uint64_t vb = cs.vote_offsets[i], ve = cs.vote_offsets[i + 1];
    // committee index of each vote's key (for the batch's pre-decompressed key tables);
    // votes the loop below does not reach keep kNoKey (decompressed in the batch kernel)
    if (vote_key && !keys_pre)
      for (uint64_t v = vb; v < ve; ++v) vote_key[v] = kNoKey;
    if (vote_cert)   // each vote's certificate (the keyed vote checks run one lane per vote)
      for (uint64_t v = vb; v < ve; ++v) vote_cert[v] = (uint32_t)i;
    uint32_t weight = 0;
    // `used` only ever holds names that passed the stake check, i.e. committee members, so
    // AuthorityReuse is "this committee index was seen before" (a bitmap for committees of
    // up to 256; pairwise key comparison above that).
    uint32_t seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool small_com = com.nauth <= 256;
    // the votes' keys are fetched kVoteChunk at a time (one load latency per chunk instead of
    // one per vote: a lane walks all of its certificate's votes); the checks themselves run
    // vote by vote, in order, exactly as before
    constexpr int kVoteChunk = 4;
    uint32_t pkc[kVoteChunk][8];
    if (keys_pre) {   // k_vote_keys ran (small committee): one word per vote, 8 at a time
      uint32_t kc[8];
      for (uint64_t v = vb; v < ve && p2 == 0; ++v) {
        const int u = (int)((v - vb) % 8);
        if (u == 0) {
#pragma unroll
          for (int c = 0; c < 8; ++c) kc[c] = v + c < ve ? vote_key[v + c] : kNoKey;
        }
        uint32_t k = kc[0];
#pragma unroll
        for (int c = 1; c < 8; ++c) k = u == c ? kc[c] : k;
        const int av = k == kNoKey ? -1 : (int)k;
        bool reuse = false;
        if (av >= 0) {
          const uint32_t bit = 1u << (av & 31);
          uint32_t word = 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) word = (av >> 5) == q ? seen[q] : word;
          reuse = (word & bit) != 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) seen[q] |= (av >> 5) == q ? bit : 0u;
        }
        if (reuse) { p2 = NW_DAG_AUTHORITY_REUSE; x2 = v - vb; break; }
        const uint32_t st = committee_stake(com, av);
        if (st == 0) { p2 = NW_DAG_UNKNOWN_AUTHORITY; x2 = v - vb; break; }
        weight += st;
      }
    }
    for (uint64_t v = vb; !keys_pre && v < ve && p2 == 0; ++v) {
      const int u = (int)((v - vb) % kVoteChunk);
      if (u == 0) {
#pragma unroll
        for (int c = 0; c < kVoteChunk; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            pkc[c][j] = v + c < ve ? cs.vote_pks[8 * (v + c) + j] : 0u;
      }
      uint32_t pk[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint32_t x = pkc[0][j];
#pragma unroll
        for (int c = 1; c < kVoteChunk; ++c) x = u == c ? pkc[c][j] : x;
        pk[j] = x;
      }
      const int av = committee_find(com, pk);
      bool reuse = false;
      if (small_com) {
        if (av >= 0) {
          const uint32_t bit = 1u << (av & 31);
          uint32_t word = 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) word = (av >> 5) == q ? seen[q] : word;
          reuse = (word & bit) != 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) seen[q] |= (av >> 5) == q ? bit : 0u;
        }
      } else {
        for (uint64_t u = vb; u < v && !reuse; ++u) {
          bool eq = true;
#pragma unroll
          for (int j = 0; j < 8; ++j) eq &= cs.vote_pks[8 * u + j] == pk[j];
          reuse = eq;
        }
      }
      if (reuse) { p2 = NW_DAG_AUTHORITY_REUSE; x2 = v - vb; break; }
      if (vote_key && av >= 0) vote_key[v] = (uint32_t)av;
      const uint32_t st = committee_stake(com, av);
      if (st == 0) { p2 = NW_DAG_UNKNOWN_AUTHORITY; x2 = v - vb; break; }
      weight += st;
    }
    if (p2 == 0 && weight < quorum) p2 = NW_DAG_REQUIRES_QUORUM;
    uint32_t cd[8];
    sha512_digest72(cd, id, round, author);
#pragma unroll
    for (int j = 0; j < 8; ++j) cert_digest[8 * i + j] = cd[j];
  }
  pre1[i] = genesis ? -1 : p1;
  pre2[i] = p2;
  idx1[i] = x1;
  idx2[i] = x2;
}

__global__ __launch_bounds__(256) void k_cert_finalize(uint64_t n, int headers_only,
                                                       const int32_t* __restrict__ pre1,
                                                       const int32_t* __restrict__ pre2,
                                                       const uint64_t* __restrict__ idx1,
                                                       const uint64_t* __restrict__ idx2,
                                                       const int32_t* __restrict__ hdr_status,
                                                       const int32_t* __restrict__ batch_status,
                                                       const uint64_t* __restrict__ batch_index,
                                                       int32_t* __restrict__ status,
                                                       uint64_t* __restrict__ index) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t st = 0;
  uint64_t ix = 0;
  const int32_t p1 = pre1[i];
  if (p1 < 0) {
    st = 0;                                           // genesis certificate
  } else if (p1 > 0) {
    st = p1; ix = idx1[i];
  } else if (hdr_status[i] != 0) {
    st = NW_DAG_INVALID_SIGNATURE + hdr_status[i];
  } else if (!headers_only) {
    if (pre2[i] != 0) {
      st = pre2[i]; ix = idx2[i];
    } else if (batch_status[i] != 0) {
      st = NW_DAG_INVALID_VOTES + batch_status[i]; ix = batch_index[i];
    }
  }
  status[i] = st;
  if (index) index[i] = ix;
}

__global__ __launch_bounds__(256) void k_vote_prepare(cert_committee_t com_g, uint64_t n,
                                                      const uint32_t* __restrict__ ids,
                                                      const uint64_t* __restrict__ rounds,
                                                      const uint32_t* __restrict__ origins,
                                                      const uint32_t* __restrict__ authors,
                                                      uint32_t* __restrict__ digests,
                                                      int32_t* __restrict__ pre,
                                                      uint32_t* __restrict__ author_key) {
  __shared__ uint32_t s_pks[8 * kLdsAuth], s_stakes[kLdsAuth];
  const cert_committee_t com = committee_to_lds(com_g, s_pks, s_stakes);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t id[8], org[8], au[8], d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    id[j] = ids[8 * i + j];
    org[j] = origins[8 * i + j];
    au[j] = authors[8 * i + j];
  }
  sha512_digest72(d, id, rounds[i], org);
#pragma unroll
  for (int j = 0; j < 8; ++j) digests[8 * i + j] = d[j];
  const int a = committee_find(com, au);
  pre[i] = committee_stake(com, a) == 0 ? NW_DAG_UNKNOWN_AUTHORITY : 0;
  // a member's signature is checked against its pre-decompressed key tables (keyed comb)
  if (author_key) author_key[i] = a >= 0 ? (uint32_t)a : kNoKey;
}

__global__ __launch_bounds__(256) void k_vote_finalize(uint64_t n, const int32_t* __restrict__ pre,
                                                       const int32_t* __restrict__ sig_status,
                                                       int32_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  status[i] = pre[i] ? pre[i] : (sig_status[i] ? NW_DAG_INVALID_SIGNATURE + sig_status[i] : 0);
}

static inline unsigned blocks_for(uint64_t n) { return (unsigned)((n + 255) / 256); }

hipError_t launch_cert_prepare(const cert_committee_t& com, const cert_stream_t& cs,
                               int headers_only, const uint32_t* hdr_digest, uint32_t* authors,
                               uint32_t* cert_digest, int32_t* pre1, int32_t* pre2,
                               uint64_t* idx1, uint64_t* idx2, uint32_t* vote_key,
                               uint32_t* author_key, uint32_t* vote_cert, uint64_t nvotes,
                               hipStream_t stream) {
  if (cs.n == 0) return hipSuccess;
  const int keys_pre = !headers_only && vote_key && com.nauth <= kLdsAuth && nvotes;
  if (keys_pre)
    hipLaunchKernelGGL(k_vote_keys, dim3(blocks_for(nvotes)), dim3(256), 0, stream, com,
                       nvotes, cs.vote_pks, vote_key);
  hipLaunchKernelGGL(k_cert_prepare, dim3(blocks_for(cs.n)), dim3(256), 0, stream, com, cs,
                     headers_only, hdr_digest, authors, cert_digest, pre1, pre2, idx1, idx2,
                     vote_key, author_key, vote_cert, keys_pre);
  return hipGetLastError();
}

hipError_t launch_cert_finalize(uint64_t n, int headers_only, const int32_t* pre1,
                                const int32_t* pre2, const uint64_t* idx1, const uint64_t* idx2,
                                const int32_t* hdr_status, const int32_t* batch_status,
                                const uint64_t* batch_index, int32_t* status, uint64_t* index,
                                hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_cert_finalize, dim3(blocks_for(n)), dim3(256), 0, stream, n,
                     headers_only, pre1, pre2, idx1, idx2, hdr_status, batch_status,
                     batch_index, status, index);
  return hipGetLastError();
}

hipError_t launch_vote_prepare(const cert_committee_t& com, uint64_t n, const uint32_t* ids,
                               const uint64_t* rounds, const uint32_t* origins,
                               const uint32_t* authors, uint32_t* digests, int32_t* pre,
                               uint32_t* author_key, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_vote_prepare, dim3(blocks_for(n)), dim3(256), 0, stream, com, n, ids,
                     rounds, origins, authors, digests, pre, author_key);
  return hipGetLastError();
}

hipError_t launch_vote_finalize(uint64_t n, const int32_t* pre, const int32_t* sig_status,
                                int32_t* status, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_vote_finalize, dim3(blocks_for(n)), dim3(256), 0, stream, n, pre,
                     sig_status, status);
  return hipGetLastError();
}

}  // namespace nw
