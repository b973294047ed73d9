// nw_small.hip — Header::verify / Vote::verify / Certificate::verify of a SMALL job in one
// launch: the latency path of the aggregation service (nw_service.cpp).
//
// Narwhal's primary checks one message at a time on its Core task (primary/src/core.rs:
// 306-346: sanitize_header / sanitize_vote / sanitize_certificate call
// primary/src/messages.rs:48-67, 131-142, 189-215 inline), so the service's jobs are mostly a
// handful of messages. The bulk pipeline (nw_api.cpp cert_pipeline) spends a one-certificate
// job in ~20 launches whose work is single-lane chains (keyed checks, batched inversions,
// verify_batch planning): ~0.3 ms of device time, and every job serialises on the device
// lease. Here one launch does the whole check, each independent chain in its own wave:
//
//   slot   one signature: a certificate's header signature (j = 0) and its votes (j = 1..q),
//          a header's signature, a vote's signature. Slots are numbered in message order;
//          workgroup w takes slots [w S, w S + S), S = 4 .. 64 (the host picks S for the
//          job size: small S = short comb chains, large S = fewer workgroups).
//   wave 0 decompresses R of every slot (curve25519-dalek decompress, a lane per slot): the
//          ~255-squaring chain starts at once and runs beside everything else.
//   wave 1 the messages whose first slot is here: Sha512(header bytes) == id, author stake,
//          worker ids, genesis; then each certificate's vote quorum (reuse / stake / weight,
//          lanes over its votes); a vote's author stake.
//   wave 2 per slot: the committee index of A, the signed message M (the claimed header id,
//          Certificate::digest, Vote::digest), k = H(R || A || M) mod l, the s checks and the
//          comb digits of k and s.
//   waves 2-3  R' = [s]B - [k]A: 27 table entries per slot (16 from the committee key's
//          16-bit comb tables, 11 from the 24-bit B comb; both built once per device and
//          committee), 128 / S lanes per slot, summed as a tree across the lanes.
//   then   per slot: R == R' projectively and the strict status, or for a certificate vote
//          its verify_batch record (below); the workgroup that completes a message (an
//          arrival counter when its slots span workgroups) combines its slots in the
//          reference's order and writes status and index straight into the job's pinned
//          host buffer: no copies before or after the launch.
//
// Certificate::verify's verify_batch with no multi-scalar multiplication. dalek's equation is
//   E = sum_i z_i R_i + (z_i k_i mod l) A_i - (sum_i z_i s_i mod l) B == identity.
// With Delta_i = R_i - ([s_i]B - [k_i]A_i) (every vote's own residual, computed here) and
// z_i k_i mod l = z_i k_i - q_i l:  E = sum_i z_i Delta_i - q_i [l]A_i, and [l]A_i =
// [lambda_i]T8 is the key's torsion image (k_key_base). A Delta_i with a prime-order part
// (8 Delta_i != 0) and z_i != 0 makes E != identity except with probability 2^-128 (the
// reference's own soundness bound): Err. Otherwise every Delta_i = [delta_i]T8 and
// E = [sum_i z_i delta_i - q_i lambda_i mod 8] T8 exactly, with q_i = 5 (z_i k_i - c_i) mod 8
// (l = 5 mod 8, 5^-1 = 5 mod 8). So a certificate's status and index equal dalek's for the
// coefficients used: injected z16, or ChaCha20 keyed from the OS CSPRNG.
#include "nw_kernels.h"
#include "nw_point.hpp"
#include "nw_scalar.hpp"
#include "nw_sha512.hpp"
#include "nw_strict.hpp"
#include "nw_consts.hpp"
#include "nw_committee.hpp"
#include "nw_chacha.hpp"
#include "nw_lp.hpp"

#include <mutex>

namespace nw {

namespace {

struct small_consts {
  strict_consts sk;      // curve constants, small-order y values
  torsion_consts tor;    // [j] T8
};
__constant__ small_consts g_sc;

constexpr int kSlotsMax = 64;
// comb entries per slot: at most 16 key-comb digits (W >= 16) + the B comb's
constexpr int kDigits = 16 + kBCombT;
static_assert(kDigits <= 27, "at most 16 key-comb + 11 B-comb digits (LDS per slot)");

// Per-slot record (slot_rec, s_rec).
enum : uint32_t {
  SR_S_HIGH = 1u,       // s has bits 253..255 set (ed25519 Signature::from_bytes)
  SR_A_FAIL = 2u,       // the key does not decode
  SR_S_NONCANON = 4u,   // s >= l
  SR_R_FAIL = 8u,       // R does not decode
  SR_PRIME = 16u,       // residual with a prime-order part (and z != 0): the batch fails
  SR_TOR_SHIFT = 5u,    // 3 bits: z delta - q lambda mod 8
  SR_ST_SHIFT = 8u,     // strict status (header / vote signatures)
};

__device__ __forceinline__ void load8w(uint32_t o[8], const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = p[i];
}

__device__ __forceinline__ ge shfl_down_ge(const ge& p, int off) {
  ge r;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.X.v[i] = (uint32_t)__shfl_down((int)p.X.v[i], off);
    r.Y.v[i] = (uint32_t)__shfl_down((int)p.Y.v[i], off);
    r.Z.v[i] = (uint32_t)__shfl_down((int)p.Z.v[i], off);
    r.T.v[i] = (uint32_t)__shfl_down((int)p.T.v[i], off);
  }
  return r;
}

__device__ __forceinline__ void release_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// z^((p-5)/8) for the four field elements of a wave's rows (nw_lp.hpp: row r = one element,
// limb k in lane 16 r + k), the addition chain of fe_pow22523: 252 squarings and 11
// multiplications, each a limb-parallel product (a dependent chain of ~75 VALU instructions
// instead of a 10-limb serial product on one lane). Every operand is a limb-parallel
// product's output (the T_LP bound, tests/test_field_bounds.py) or the canonical input.
__device__ __forceinline__ uint32_t lp_sqn(const lp_ctx& c, uint32_t x, int n) {
#pragma unroll 1
  for (int i = 0; i < n; ++i) x = lp_mul(c, x, x);
  return x;
}
__device__ __forceinline__ uint32_t lp_pow22523(const lp_ctx& c, uint32_t z) {
  const uint32_t z2 = lp_mul(c, z, z);                          // 2
  uint32_t t = lp_sqn(c, z2, 2);                                // 8
  const uint32_t z9 = lp_mul(c, t, z);                          // 9
  const uint32_t z11 = lp_mul(c, z9, z2);                       // 11
  t = lp_mul(c, z11, z11);                                      // 22
  const uint32_t z5 = lp_mul(c, t, z9);                         // 2^5 - 1
  const uint32_t z10 = lp_mul(c, lp_sqn(c, z5, 5), z5);         // 2^10 - 1
  const uint32_t z20 = lp_mul(c, lp_sqn(c, z10, 10), z10);      // 2^20 - 1
  t = lp_mul(c, lp_sqn(c, z20, 20), z20);                       // 2^40 - 1
  const uint32_t z50 = lp_mul(c, lp_sqn(c, t, 10), z10);        // 2^50 - 1
  const uint32_t z100 = lp_mul(c, lp_sqn(c, z50, 50), z50);     // 2^100 - 1
  t = lp_mul(c, lp_sqn(c, z100, 100), z100);                    // 2^200 - 1
  t = lp_mul(c, lp_sqn(c, t, 50), z50);                         // 2^250 - 1
  return lp_mul(c, lp_sqn(c, t, 2), z);                         // 2^252 - 3
}

// Diagnostic phase stamps (NW_SMALL_STAMPS, small_job_t::stamps): s_memrealtime (100 MHz)
// per workgroup at the phase boundaries below, written by one lane of the wave that ends
// the phase; no output depends on them.
enum { ST_START = 0, ST_DECOMP, ST_MSG, ST_DIGITS, ST_COMB, ST_SYNC, ST_SLOTS, ST_END, ST_N };
__device__ __forceinline__ void stamp(const small_job_t& J, int which) {
  if (J.stamps && (threadIdx.x & 63) == 0)
    J.stamps[(uint64_t)blockIdx.x * ST_N + which] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace

// Header digests of wave 1 (Header::verify's id check, primary/src/messages.rs:48-55).
// SHA-512 is a chain per message, and one lane of a lone wave issues each instruction at the
// wave's full cost (~6.5 us per 128-B block), so a certificate's header (9 blocks at N = 50,
// 18 at N = 100) is a job's longest chain. When the wave owns ONE header of at most
// kSchedBlocks blocks, its message schedules are computed by one lane per block side by side
// into LDS, and the owner runs only the 80 rounds per block, reading W[t] from LDS (the
// schedule is ~35 % of a block's instructions). Otherwise each owner lane hashes its own
// header. dg: the digest's 8 LE words in the owner lane(s).
constexpr uint32_t kSchedBlocks = 32;
__device__ __forceinline__ void header_digest(bool need, const uint8_t* h, uint64_t len,
                                              uint32_t dg[8], uint32_t lane,
                                              uint64_t (*s_w)[80]) {
  const uint64_t mask = __ballot(need);
  if (mask == 0) return;
  if (__popcll(mask) == 1) {
    const int o = __ffsll((unsigned long long)mask) - 1;
    const uint64_t hp = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uintptr_t)h >> 32), o) << 32) |
                        (uint32_t)__shfl((int)(uint32_t)(uintptr_t)h, o);
    const uint64_t L = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(len >> 32), o) << 32) |
                       (uint32_t)__shfl((int)(uint32_t)len, o);
    const uint64_t nb = (L + 17 + 127) / 128;
    if (nb <= kSchedBlocks) {
      const uint8_t* msg = reinterpret_cast<const uint8_t*>(hp);
      if (lane < nb) {
        uint64_t w[16];
        const uint64_t base = 128 * (uint64_t)lane;
        if (base + 128 <= L) {
          uint32_t d[33];
          load_block_raw(d, msg + base);
          block_from_raw(w, d, (uint32_t)((uintptr_t)msg & 3) * 8);
        } else {
          load_block_tail(w, msg, base, L, lane + 1 == nb);
        }
        uint64_t* W = s_w[lane];
#pragma unroll
        for (int t = 0; t < 16; ++t) W[t] = w[t];
#pragma unroll 1
        for (int r = 16; r < 80; r += 16) {
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const uint64_t w15 = w[(j + 1) & 15], w2 = w[(j + 14) & 15];
            const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
            const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
            w[j] = w[j] + s0 + w[(j + 9) & 15] + s1;
            W[r + j] = w[j];
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      if ((int)lane == o) {
        uint64_t st[8];
        sha512_init(st);
#pragma unroll 1
        for (uint64_t b = 0; b < nb; ++b) {
          const uint64_t* W = s_w[b];
          uint64_t a = st[0], bb = st[1], c = st[2], d = st[3], e = st[4], f = st[5],
                   g = st[6], hh = st[7];
#pragma unroll 1
          for (int r = 0; r < 80; r += 16) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
              const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
              const uint64_t t1 = hh + S1 + ch64(e, f, g) + SHA512_K[r + j] + W[r + j];
              const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
              const uint64_t t2 = S0 + maj64(a, bb, c);
              hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
            }
          }
          st[0] += a; st[1] += bb; st[2] += c; st[3] += d; st[4] += e; st[5] += f;
          st[6] += g; st[7] += hh;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dg[2 * j] = __builtin_bswap32((uint32_t)(st[j] >> 32));
          dg[2 * j + 1] = __builtin_bswap32((uint32_t)st[j]);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      return;
    }
  }
  if (need) sha512_digest32_lane(h, len, dg);
}

__global__ __launch_bounds__(256) void k_small(small_job_t J) {
  __shared__ uint32_t s_pks[8 * kLdsAuth], s_stakes[kLdsAuth], s_first[kLdsAuth];
  __shared__ small_slot_t s_slot[kSlotsMax];
  __shared__ fe s_Rx[kSlotsMax], s_Ry[kSlotsMax];
  __shared__ ge s_P[kSlotsMax];
  __shared__ int32_t s_dig[kSlotsMax][kDigits + 1];
  __shared__ uint32_t s_k[kSlotsMax][8];
  __shared__ uint32_t s_key[kSlotsMax], s_kf[kSlotsMax], s_sfl[kSlotsMax], s_rfl[kSlotsMax];
  __shared__ uint32_t s_rec[kSlotsMax];
  __shared__ small_msg_info_t s_minfo[kSlotsMax];
  // a message whose first slot is here: wave 1's header verdict (s_p1, s_x1) and wave 0's
  // quorum verdict (s_p2, s_x2), assembled into s_minfo after the first barrier
  __shared__ int32_t s_p1[kSlotsMax], s_p2[kSlotsMax];
  __shared__ uint64_t s_x1[kSlotsMax], s_x2[kSlotsMax];
  __shared__ uint32_t s_ready;
  __shared__ uint32_t s_lp[64];   // wave 0: the limb-parallel power's rows, gathered
  __shared__ uint64_t s_w[kSchedBlocks][80];   // wave 1: header message schedules

  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
  const uint64_t S = J.slots_per_wg;
  const uint64_t first = (uint64_t)blockIdx.x * S;
  const uint32_t ns = (uint32_t)(J.nslots - first < S ? J.nslots - first : S);
  const bool certs = J.kind == kSmallCerts;

  // ---- phase 0: the committee (sorted keys, stakes) and the slot table into LDS
  const uint32_t na = (uint32_t)J.com.nauth;   // <= kLdsAuth (host check)
  for (uint32_t k = tid; k < 8 * na; k += 256) s_pks[k] = J.com.pks[k];
  for (uint32_t k = tid; k < na; k += 256) s_stakes[k] = J.com.stakes[k];
  for (uint32_t k = tid; k < kLdsAuth; k += 256) s_first[k] = 0xffffffffu;
  if (tid < ns) s_slot[tid] = J.slots[first + tid];
  if (tid == 0) s_ready = 0;
  if (tid == 0) stamp(J, ST_START);
  __syncthreads();
  cert_committee_t com = J.com;
  com.pks = s_pks;
  com.stakes = s_stakes;

  if (wave == 0) {
    // ---- wave 0: R of every slot (dalek decompress; x sign, y taken unreduced)
    auto sig_of = [&](const small_slot_t& sl) -> const uint32_t* {
      return certs ? (sl.j ? J.vsig + 16 * (uint64_t)sl.v : J.hsig + 16 * (uint64_t)sl.m)
                   : (J.kind == kSmallHeaders ? J.hsig : J.sigs) + 16 * (uint64_t)sl.m;
    };
    if (S == 4) {
      // four slots, one per row: the (p-5)/8 power limb-parallel (lp_pow22523), the
      // prologue and the final step (sqrt_ratio_i's checks, x's sign) per row as usual
      const lp_ctx c = lp_init(lane);
      const uint32_t r = c.row;
      uint32_t Rw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (r < ns) load8w(Rw, sig_of(s_slot[r]));
      const curve_consts& K = g_sc.sk.k;
      fe y, u, v, t, v3, v7, uv7, zc;
      fe_frombytes(y, Rw);
      ge_decomp_uv(u, v, y, K);
      fe_sq(t, v);  fe_mul(v3, t, v);
      fe_sq(t, v3); fe_mul(v7, t, v);
      fe_mul(uv7, u, v7);
      fe_canonical(zc, uv7);
      uint32_t zl = 0;
#pragma unroll
      for (int i = 0; i < 10; ++i) zl = c.k == (uint32_t)i ? zc.v[i] : zl;
      const uint32_t tl = lp_pow22523(c, zl);
      s_lp[lane] = tl;
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      __builtin_amdgcn_wave_barrier();
      fe tp;
#pragma unroll
      for (int i = 0; i < 10; ++i) tp.v[i] = s_lp[16 * r + i];
      fe_canonical(t, tp);
      ge R;
      R.Y = y;
      const bool okR = fe_sqrt_ratio_finish(R.X, u, v, t, K);
      fe_neg(t, R.X);
      fe_cmov(R.X, t, (Rw[7] >> 31) != 0);
      const bool smallR = small_order_by_y(R.Y, g_sc.sk.small_y);
      if (r < ns && c.k == 0) {
        s_Rx[r] = R.X;
        s_Ry[r] = R.Y;
        s_rfl[r] = (okR ? 1u : 0u) | (smallR ? 2u : 0u);
      }
    } else if (lane < ns) {
      uint32_t Rw[8];
      load8w(Rw, sig_of(s_slot[lane]));
      ge R;
      const bool okR = ge_frombytes(R, Rw, g_sc.sk.k);
      const bool smallR = small_order_by_y(R.Y, g_sc.sk.small_y);
      s_Rx[lane] = R.X;
      s_Ry[lane] = R.Y;
      s_rfl[lane] = (okR ? 1u : 0u) | (smallR ? 2u : 0u);
    }
    stamp(J, ST_DECOMP);
    const bool own = lane < ns && s_slot[lane].j == 0;
    int32_t p2 = 0;
    uint64_t x2 = 0;
    if (certs) {
      // Certificate::verify's quorum (messages.rs:196-211), per owned certificate (its
      // verdict counts only when the header passed: the combine reads p1 first), lanes
      // over its votes: reuse, then stake, first failure in vote order; else the u32
      // weight against 2 total / 3 + 1 (config/src/lib.rs:167-173).
      uint32_t total = 0;
      for (uint32_t a = lane; a < na; a += 64) total += s_stakes[a];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) total += (uint32_t)__shfl_xor((int)total, off);
      const uint32_t quorum = 2u * total / 3u + 1u;
      uint64_t todo = __ballot(own);
      while (todo) {
        const int o = __ffsll((unsigned long long)todo) - 1;
        todo &= todo - 1;
        const uint32_t sv = s_slot[o].v;          // the certificate's first vote
        const uint32_t q = s_slot[o].cnt - 1;     // its votes
        int kv[2] = {-1, -1};
        uint32_t st[2] = {0, 0};
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          const uint32_t v = 64u * pass + lane;
          if (v < q) {
            uint32_t pk[8];
            load8w(pk, J.vpk + 8 * ((uint64_t)sv + v));
            kv[pass] = committee_find(com, pk);
            st[pass] = committee_stake(com, kv[pass]);
            if (kv[pass] >= 0) atomicMin(&s_first[kv[pass]], v);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        __builtin_amdgcn_wave_barrier();
        int32_t cp2 = 0;
        uint64_t cx2 = 0;
        uint32_t weight = 0;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          const uint32_t v = 64u * pass + lane;
          const bool reuse = v < q && kv[pass] >= 0 && s_first[kv[pass]] < v;
          const bool fail = v < q && (reuse || st[pass] == 0);
          const uint64_t fm = __ballot(fail);
          if (fm && cp2 == 0) {
            const int f = __ffsll((unsigned long long)fm) - 1;
            cp2 = __shfl((int)reuse, f) ? NW_DAG_AUTHORITY_REUSE : NW_DAG_UNKNOWN_AUTHORITY;
            cx2 = 64u * pass + (uint32_t)f;
          }
          weight += v < q ? st[pass] : 0u;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) weight += (uint32_t)__shfl_xor((int)weight, off);
        if (cp2 == 0 && weight < quorum) cp2 = NW_DAG_REQUIRES_QUORUM;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass)
          if (64u * pass + lane < q && kv[pass] >= 0) s_first[kv[pass]] = 0xffffffffu;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        __builtin_amdgcn_wave_barrier();
        if ((int)lane == o) {
          p2 = cp2;
          x2 = cx2;
        }
      }
    }
    s_p2[lane] = p2;
    s_x2[lane] = x2;
  } else if (wave == 1) {
    // ---- wave 1: Header::verify's checks of the messages whose first slot is here (the
    // header digest is the longest serial chain of a certificate job: ~9 SHA-512 blocks at
    // N = 50; the quorum runs on wave 0 beside it)
    const bool own = lane < ns && s_slot[lane].j == 0;
    int32_t p1 = 0;
    uint64_t x1 = 0;
    uint32_t mown = own ? s_slot[lane].m : 0u;
    if (J.kind == kSmallVotes) {
      if (own) {
        uint32_t au[8];
        load8w(au, J.authors + 8 * mown);
        if (committee_stake(com, committee_find(com, au)) == 0) p1 = NW_DAG_UNKNOWN_AUTHORITY;
      }
    } else {
      const uint64_t m = mown;
      const uint8_t* h = nullptr;
      uint64_t len = 0;
      uint32_t id[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      int a = -1;
      bool genesis = false;
      if (own) {
        h = J.hb + J.ho[m];
        len = J.ho[m + 1] - J.ho[m];
        uint32_t author[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          author[t] = ld_le32(h + 4 * t);
          id[t] = J.ids[8 * m + t];
        }
        const uint64_t round = (uint64_t)ld_le32(h + 32) | ((uint64_t)ld_le32(h + 36) << 32);
        a = committee_find(com, author);
        uint32_t idor = 0;
#pragma unroll
        for (int t = 0; t < 8; ++t) idor |= id[t];
        // Certificate::verify: genesis(committee).contains(self) (messages.rs:190-193)
        genesis = certs && idor == 0 && round == 0 && a >= 0;
      }
      uint32_t dg[8];
      header_digest(own && !genesis, h, len, dg, lane, s_w);
      if (own) {
        if (genesis) {
          p1 = -1;
        } else {
          // Header::verify (messages.rs:48-67), in order: id, stake, worker ids
          bool id_ok = true;
#pragma unroll
          for (int t = 0; t < 8; ++t) id_ok &= dg[t] == id[t];
          if (!id_ok) {
            p1 = NW_DAG_INVALID_HEADER_ID;
          } else if (committee_stake(com, a) == 0) {
            p1 = NW_DAG_UNKNOWN_AUTHORITY;
            x1 = ~0ull;
          } else {
            const uint32_t np = J.pc[m];
            const uint64_t wb = J.com.worker_offsets[a], we = J.com.worker_offsets[a + 1];
            for (uint32_t e = 0; e < np && p1 == 0; ++e) {
              const uint32_t wid = ld_le32(h + 40 + 36 * (uint64_t)e + 32);
              bool found = false;
              for (uint64_t w = wb; w < we; ++w) found |= J.com.worker_ids[w] == wid;
              if (!found) { p1 = NW_DAG_MALFORMED_HEADER; x1 = e; }
            }
          }
        }
      }
    }
    s_p1[lane] = p1;
    s_x1[lane] = x1;
    stamp(J, ST_MSG);
    release_vm();
  } else {
    // ---- wave 2: per slot, the signed message, k and the comb digits
    if (wave == 2 && lane < ns) {
      const small_slot_t sl = s_slot[lane];
      const uint64_t m = sl.m;
      const uint32_t *A, *sig;
      uint32_t M[8];
      if (J.kind == kSmallVotes) {
        A = J.authors + 8 * m;
        sig = J.sigs + 16 * m;
        uint32_t id[8], org[8];
        load8w(id, J.ids + 8 * m);
        load8w(org, J.origins + 8 * m);
        sha512_digest72(M, id, J.rounds[m], org);            // Vote::digest
      } else {
        const uint8_t* h = J.hb + J.ho[m];
        A = reinterpret_cast<const uint32_t*>(h);            // header author (4-aligned)
        if (sl.j == 0) {
          sig = J.hsig + 16 * m;
          load8w(M, J.ids + 8 * m);                          // Header::verify signs the id
        } else {
          A = J.vpk + 8 * (uint64_t)sl.v;
          sig = J.vsig + 16 * (uint64_t)sl.v;
          uint32_t id[8], au[8];
          load8w(id, J.ids + 8 * m);
#pragma unroll
          for (int t = 0; t < 8; ++t) au[t] = ld_le32(h + 4 * t);
          const uint64_t round = (uint64_t)ld_le32(h + 32) | ((uint64_t)ld_le32(h + 36) << 32);
          sha512_digest72(M, id, round, au);                 // Certificate::digest
        }
      }
      uint32_t Aw[8], Rw[8], Sw[8];
      if (J.kind != kSmallVotes && sl.j == 0) {
        const uint8_t* h = J.hb + J.ho[m];
#pragma unroll
        for (int t = 0; t < 8; ++t) Aw[t] = ld_le32(h + 4 * t);
      } else {
        load8w(Aw, A);
      }
      load8w(Rw, sig);
      load8w(Sw, sig + 8);
      const int a = committee_find(com, Aw);
      const uint32_t kk = a >= 0 ? (uint32_t)a : kNoKey;
      const uint32_t kf = a >= 0 ? J.kok[a] : 0u;
      sc s;
#pragma unroll
      for (int t = 0; t < 8; ++t) s.w[t] = Sw[t];
      const bool s_high = (Sw[7] >> 29) != 0;
      const bool canon = sc_is_canonical(s);
      const bool doc = a >= 0 && (kf & kKeyDecoded) && !s_high && canon;
      if (doc) {
        uint32_t hx[16];
        sha512_hram96(hx, Rw, Aw, M);
        sc k;
        sc_reduce512(k, hx);
        uint32_t kd[8], sd[8];
        key_recode(kd, k, J.ks);
        bdigits<kBCombW>::recode(sd, s);
#pragma unroll
        for (int t = 0; t < 16; ++t)
          if (t < (int)J.ks.ntab) s_dig[lane][t] = key_digit(kd, t, J.ks);
#pragma unroll
        for (int t = 0; t < kBCombT; ++t)
          s_dig[lane][J.ks.ntab + t] = bdigits<kBCombW>::digit(sd, t);
#pragma unroll
        for (int t = 0; t < 8; ++t) s_k[lane][t] = k.w[t];
      }
      s_key[lane] = kk;
      s_kf[lane] = kf;
      s_sfl[lane] = (s_high ? 1u : 0u) | (canon ? 0u : 2u) | (doc ? 4u : 0u);
    }
    if (wave == 2) {
      stamp(J, ST_DIGITS);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&s_ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      while (__hip_atomic_load(&s_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
        __builtin_amdgcn_s_sleep(1);
    }
    // ---- waves 2-3: R' = [s]B - [k]A, G = 128 / S lanes per slot
    const uint32_t G = 128u / (uint32_t)S;
    const uint32_t c = tid - 128u, sl = c / G, g = c % G;
    const bool live = sl < ns && (s_sfl[sl] & 4u);
    ge acc;
    ge_identity(acc);
    if (live) {
      const uint32_t kk = s_key[sl];
      const ge_niels_pad* kt = J.ktabs + (uint64_t)J.ks.tab * kk;
      const uint32_t KT = J.ks.ntab, ND = KT + (uint32_t)kBCombT;
#pragma unroll 1
      for (uint32_t e = g; e < ND; e += G) {
        const int d = s_dig[sl][e];
        if (d == 0) continue;
        const uint32_t ad = (uint32_t)(d < 0 ? -d : d);
        const bool isA = e < KT;
        const ge_niels_pad* ent = isA ? kt + e * J.ks.nent + ad
                                      : J.bcomb + (e - KT) * kBCombN + ad;
        ge_niels nb = ent->n;
        ge_niels_cneg(nb, isA ? d > 0 : d < 0);   // -[k]A: key digits negated
        ge_add_niels(acc, acc, nb, true);
      }
    }
    // tree over the slot's G lanes (every lane adds; a lane is read once, at the level of
    // its lowest set bit, when it still holds its subtree's sum)
#pragma unroll 1
    for (uint32_t off = G >> 1; off >= 1; off >>= 1) {
      const ge o = shfl_down_ge(acc, (int)off);
      ge_cached oc;
      ge_to_cached(oc, o, g_sc.sk.k.d2);
      ge_add_cached(acc, acc, oc, true);
    }
    if (live && g == 0) s_P[sl] = acc;
    if (wave == 2) stamp(J, ST_COMB);
  }
  __syncthreads();
  if (tid == 0) stamp(J, ST_SYNC);
  // the message info (read by the combine below, and by other workgroups through J.minfo
  // when the message's slots span several)
  if (wave == 1 && lane < ns && s_slot[lane].j == 0) {
    const small_msg_info_t info{s_p1[lane], s_p2[lane], s_x1[lane], s_x2[lane]};
    s_minfo[lane] = info;
    const small_slot_t sl = s_slot[lane];
    if ((first + lane) / S != (first + lane + sl.cnt - 1) / S) J.minfo[sl.m] = info;   // spans
  }

  // ---- per slot: R == R', the strict status or the certificate vote's batch record
  if (wave == 2 && lane < ns) {
    const small_slot_t sl = s_slot[lane];
    const uint32_t kf = s_kf[lane], sfl = s_sfl[lane], rfl = s_rfl[lane];
    const bool s_high = sfl & 1u, canon = !(sfl & 2u), doc = sfl & 4u;
    const bool okA = kf & kKeyDecoded, smallA = kf & kKeySmall;
    const bool okR = rfl & 1u, smallR = rfl & 2u;
    ge R;
    R.X = s_Rx[lane];
    R.Y = s_Ry[lane];
    fe_1(R.Z);
    fe_mul(R.T, R.X, R.Y);
    bool eq = false;
    ge P;
    if (doc) {
      P = s_P[lane];
      if (okR) eq = ge_eq_affine(P, R);
    }
    uint32_t rec;
    if (certs && sl.j != 0) {
      rec = (s_high ? SR_S_HIGH : 0u) | (okA ? 0u : SR_A_FAIL) | (canon ? 0u : SR_S_NONCANON) |
            (okR ? 0u : SR_R_FAIL);
      const uint32_t lam = (kf & kKeyLambdaMask) >> kKeyLambdaShift;
      if (rec == 0 && doc && (!eq || lam != 0)) {
        uint32_t z[4];
        if (J.z16) {
#pragma unroll
          for (int t = 0; t < 4; ++t) z[t] = J.z16[4 * (uint64_t)sl.v + t];
        } else {
          chacha20_z(z, J.zkey, 0, sl.v);
        }
        if ((z[0] | z[1] | z[2] | z[3]) != 0) {
          uint32_t delta = 0;
          bool prime = false;
          if (!eq) {
            ge D, t;
            ge_cached Pc;
            ge_to_cached(Pc, P, g_sc.sk.k.d2);
            ge_sub_cached(D, R, Pc, true);     // Delta = R - R'
            ge_dbl(t, D, false);
            ge_dbl(t, t, false);
            ge_dbl(t, t, false);
            if (!ge_is_identity(t)) {
              prime = true;
            } else {
              const int j8 = torsion_index(D, g_sc.tor);
              delta = j8 > 0 ? (uint32_t)j8 : 0u;
            }
          }
          if (prime) {
            rec |= SR_PRIME;
          } else {
            sc zs, kx, cz;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              zs.w[t] = t < 4 ? z[t] : 0u;
              kx.w[t] = s_k[lane][t];
            }
            sc_mul(cz, zs, kx);                 // c = z k mod l
            const uint32_t q = (5u * ((z[0] & 7u) * (kx.w[0] & 7u) + 8u - (cz.w[0] & 7u))) & 7u;
            const uint32_t term = ((z[0] & 7u) * delta + 8u * 8u - q * lam) & 7u;
            rec |= term << SR_TOR_SHIFT;
          }
        }
      }
    } else {
      // crypto/src/lib.rs:200-204 order: s high bits, A decode, s < l, R decode, R small,
      // A small, equation
      const int st = s_high ? NW_ERR_S_HIGH_BITS : !okA ? NW_ERR_A_DECODE
                   : !canon ? NW_ERR_S_NONCANONICAL : !okR ? NW_ERR_R_DECODE
                   : smallR ? NW_ERR_R_SMALL_ORDER : smallA ? NW_ERR_A_SMALL_ORDER
                   : eq ? NW_OK : NW_ERR_EQUATION;
      rec = (uint32_t)st << SR_ST_SHIFT;
    }
    s_rec[lane] = rec;
    const uint64_t base = first + lane - sl.j;
    if (base / S != (base + sl.cnt - 1) / S) J.srec[first + lane] = rec;   // message spans
    release_vm();
  }
  if (wave == 2) stamp(J, ST_SLOTS);
  __syncthreads();

  // ---- messages: the workgroup that completes one combines its slots
  if (wave != 2) return;
  const bool live = lane < ns;
  const small_slot_t sl = live ? s_slot[lane] : small_slot_t{0, 0, 0, 1};
  if (!certs) {
    // one slot per message, always here
    if (!live) return;
    const small_msg_info_t info = s_minfo[lane];
    const int st = (int)(s_rec[lane] >> SR_ST_SHIFT);
    int32_t status = 0;
    uint64_t index = 0;
    if (info.p1 != 0) {
      status = info.p1;
      index = info.x1;
    } else if (st != 0) {
      status = NW_DAG_INVALID_SIGNATURE + st;
    }
    J.status[sl.m] = status;
    if (J.index) J.index[sl.m] = index;
    __threadfence_system();
    if (lane == 0 && J.done_flags)
      __hip_atomic_store(&J.done_flags[blockIdx.x], J.done_seq, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    stamp(J, ST_END);
    return;
  }
  const uint64_t base = first + lane - sl.j;            // the message's first slot
  const bool start = live && (lane == 0 || s_slot[lane - 1].m != sl.m);
  const uint64_t wlo = base / S, whi = (base + sl.cnt - 1) / S;
  const bool spans = wlo != whi;
  if (__ballot(start && spans)) {
    if (lane == 0) {
      __threadfence();
      release_vm();
    }
    __builtin_amdgcn_wave_barrier();
  }
  bool last = start && !spans;
  if (start && spans) {
    const uint32_t expect = (uint32_t)(whi - wlo + 1);
    const uint32_t old = atomicAdd(&J.mcount[sl.m], 1u);
    last = old == expect - 1;
    if (last) J.mcount[sl.m] = 0;   // no other arrival can follow: ready for the next job
  }
  if (__ballot(last && spans)) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    release_vm();
  }
  uint64_t todo = __ballot(last);
  while (todo) {
    const int o = __ffsll((unsigned long long)todo) - 1;
    todo &= todo - 1;
    const uint32_t m = s_slot[o].m;
    const uint64_t mb = first + (uint32_t)o - s_slot[o].j;
    const uint32_t cnt = s_slot[o].cnt;
    auto rec_of = [&](uint64_t slot) -> uint32_t {
      return (slot >= first && slot < first + ns) ? s_rec[slot - first] : J.srec[slot];
    };
    const small_msg_info_t info = (mb >= first) ? s_minfo[mb - first] : J.minfo[m];
    int32_t status = 0;
    uint64_t index = 0;
    if (info.p1 < 0) {
      status = 0;                                        // genesis
    } else if (info.p1 > 0) {
      status = info.p1;
      index = info.x1;
    } else {
      const int hst = (int)(rec_of(mb) >> SR_ST_SHIFT);
      if (hst != 0) {
        status = NW_DAG_INVALID_SIGNATURE + hst;
      } else if (info.p2 != 0) {
        status = info.p2;
        index = info.x2;
      } else {
        // verify_batch (crypto/src/lib.rs:206-219): per vote in order s high bits / A
        // decode (first failure), then s < l over all, then R decode, then the equation
        const uint32_t q = cnt - 1;
        uint32_t r[2];
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          const uint32_t v = 64u * pass + lane;
          r[pass] = v < q ? rec_of(mb + 1 + v) : 0u;
        }
        int b = 0;
        uint64_t bi = q;
        const uint32_t cls[3] = {SR_S_HIGH | SR_A_FAIL, SR_S_NONCANON, SR_R_FAIL};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            const uint64_t fm = __ballot((r[pass] & cls[c]) != 0);
            if (fm && b == 0) {
              const int f = __ffsll((unsigned long long)fm) - 1;
              const uint32_t rf = (uint32_t)__shfl((int)r[pass], f);
              b = c == 0 ? ((rf & SR_S_HIGH) ? NW_ERR_S_HIGH_BITS : NW_ERR_A_DECODE)
                         : c == 1 ? NW_ERR_S_NONCANONICAL : NW_ERR_R_DECODE;
              bi = 64u * pass + (uint32_t)f;
            }
          }
        }
        if (b == 0) {
          uint32_t tor = ((r[0] >> SR_TOR_SHIFT) & 7u) + ((r[1] >> SR_TOR_SHIFT) & 7u);
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) tor += (uint32_t)__shfl_xor((int)tor, off);
          if (__ballot(((r[0] | r[1]) & SR_PRIME) != 0) || (tor & 7u) != 0) {
            b = NW_ERR_EQUATION;
            bi = q;
          }
        }
        if (b != 0) {
          status = NW_DAG_INVALID_VOTES + b;
          index = bi;
        }
      }
    }
    if (lane == 0) {
      J.status[m] = status;
      if (J.index) J.index[m] = index;
      __threadfence_system();
    }
  }
  if (lane == 0 && J.done_flags) {   // this workgroup's writes are out (small_job_t)
    __threadfence_system();
    __hip_atomic_store(&J.done_flags[blockIdx.x], J.done_seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  stamp(J, ST_END);
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
hipError_t upload_small_consts() {
  static small_consts host;
  static std::once_flag once;
  std::call_once(once, [] {
    ge_niels b128[129];
    compute_strict_consts(host.sk, b128);
    compute_torsion(host.tor);
  });
  return hipMemcpyToSymbol(HIP_SYMBOL(g_sc), &host, sizeof(host), 0, hipMemcpyHostToDevice);
}

hipError_t launch_small(const small_job_t& job, hipStream_t stream) {
  if (job.nslots == 0) return hipSuccess;
  const uint64_t S = job.slots_per_wg;
  if (S < 4 || S > (uint64_t)kSlotsMax || (S & (S - 1)) || job.com.nauth > kLdsAuth ||
      job.com.nauth == 0)
    return hipErrorInvalidValue;
  const uint64_t nwg = (job.nslots + S - 1) / S;
  hipLaunchKernelGGL(k_small, dim3((unsigned)nwg), dim3(256), 0, stream, job);
  return hipGetLastError();
}

}  // namespace nw
