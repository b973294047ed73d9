// nw_kernels.h — launchers for the gfx950 kernels (host side of nw_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "narwhal_amd.h"

namespace nw {

struct z_key_t {
  uint32_t key[8];
  uint64_t nonce;
};

// Computes the curve constants and the B table on the host (from their definitions) and
// copies them to the current device's constant memory.
hipError_t upload_consts();

// hipMalloc for the large per-device tables (strict B tables, keyed B comb, committee key
// tables, strict workspace). Test hook: NW_DEVICE_MEM_LIMIT=bytes makes any such allocation
// above that size fail with hipErrorOutOfMemory, as on a device without the memory.
hipError_t table_malloc(void** p, size_t bytes);

// lengths == nullptr: offsets has n + 1 entries and message i = [offsets[i], offsets[i+1]).
hipError_t launch_sha512_digest32(const uint8_t* data, const uint64_t* offsets,
                                  const uint64_t* lengths, uint64_t n, uint32_t* out,
                                  hipStream_t stream);

// Strict verification; workspace = strict_workspace_bytes() of device memory (per-lane
// tables; reusable across launches on one stream).
size_t strict_workspace_bytes();
// keys (optional): pre-decompressed key tables with vote_key = per-item key index.
// Builds the current device's lazily built strict tables (nw_prepare).
hipError_t prepare_strict_tables();
hipError_t launch_verify_strict(const uint32_t* msgs, uint32_t msg_stride_words,
                                const uint32_t* pks, const uint32_t* sigs, uint64_t n,
                                int32_t* status, uint64_t* bitmap, void* workspace,
                                hipStream_t stream, const struct key_tables_t* keys = nullptr);

hipError_t launch_keypair(const uint32_t* seeds, uint64_t n, uint32_t* pks, hipStream_t stream);

hipError_t launch_sign(const uint32_t* sks, uint32_t sk_stride_words, const uint32_t* msgs,
                       uint32_t msg_stride_words, uint64_t n, uint32_t* sigs,
                       hipStream_t stream);

// crypto::Signature::verify_batch over many batches (nw_batch.hip). offsets: device copy,
// host_offsets: the same nbatches + 1 values in host memory (used to plan the chunks and
// the workspace slices).
hipError_t upload_batch_consts();

// Layout of a committee's key comb tables at digit width W (chosen per committee when its
// tables are built: nw_api.cpp key_width): ntab = ceil(253 / W) comb tables j * 2^(W t) A,
// j = 0..2^(W-1) (affine niels), k's digits signed except the top one when ntab W > 256;
// the keyed vote chunks' second 8-bit table j * 2^128 A is comb table 128 / W when W divides
// 128, else one more table built from 2^128 A. W = 16: 16 tables, 67 MB per key; W = 20:
// 13 + 1 tables, 940 MB per key; W = 24 (NW_KEY_WIDTH=24 only): 11 tables.
// Only these three widths are built (nw_api.cpp key_width / alloc_key_tables); any other W
// (e.g. the 0 of a device without tables) is mapped to 16, so that no caller can divide by
// zero or shift by W - 1 < 0 here, on the host or the device.
#define NW_KS __host__ __device__ __forceinline__
struct keyspec {
  uint32_t W, ntab, nsigned, nent, tab, half;
  uint32_t bias[8];   // k + bias: the recoded digit words (2^(W-1) per signed digit)
};
NW_KS constexpr keyspec keyspec_for(uint32_t W) {
  keyspec ks{};
  if (W != 16 && W != 20 && W != 24) W = 16;
  ks.W = W;
  ks.ntab = (253 + W - 1) / W;
  ks.nsigned = ks.ntab * W > 256 ? ks.ntab - 1 : ks.ntab;
  ks.nent = (1u << (W - 1)) + 1;
  const uint32_t extra = 128 % W ? 1u : 0u;
  ks.tab = (ks.ntab + extra) * ks.nent;
  ks.half = (extra ? ks.ntab : 128 / W) * ks.nent;
  for (uint32_t m = 0; m < ks.nsigned; ++m) {
    const uint32_t b = W * m + W - 1;
    ks.bias[b >> 5] |= 1u << (b & 31);
  }
  return ks;
}
NW_KS constexpr uint32_t keyspec_tables(const keyspec& ks) { return ks.tab / ks.nent; }

// Pre-decompressed public keys (a committee): per key its comb tables (layout ks) and
// whether it decompressed. vote_key[i] = key index of vote i, or kNoKey to decompress that
// vote's key in the kernel (the verdict semantics are unchanged: a key's decompression is
// deterministic). Keyed strict verifications take [k]A from the ntab tables with no
// doublings; chunks whose votes are all keyed run 8-bit A windows over the tables of j * A
// and j * 2^128 A (entries 0..128) and a 128-doubling ladder.
struct key_tables_t {
  const struct ge_niels_pad* tabs;   // nkeys x ks.tab, affine niels (mixed additions)
  const uint32_t* ok;             // nkeys
  const uint32_t* vote_key;       // nitems (global item index)
  keyspec ks;
};
constexpr uint32_t kNoKey = 0xffffffffu;
constexpr uint32_t kKeyWMax = 24;   // widths 16 / 20 / 24 (at most 16 comb digits)
// ok[key]: bit 0 = decompressed, bit 1 = small order (8A == identity), bits 2..4 = lambda
// with [l]A == [lambda]T8 (nw_strict.hpp kKeyLambdaShift: the key's torsion image)
size_t key_tables_bytes(uint64_t nkeys, const keyspec& ks);
// tabs: key_tables_bytes(nkeys) of device memory; ok: nkeys words. saved (nkeys x 8 words)
// and flag (1 word), optional: the keys the tables were last built from; the tables are
// rebuilt only when force or the keys differ (a device-side compare, so the call stays
// asynchronous), and saved is updated — the committee of an epoch is tabulated once.
hipError_t launch_key_tables(const uint32_t* pks, uint64_t nkeys, const keyspec& ks,
                             struct ge_niels_pad* tabs, uint32_t* ok, hipStream_t stream,
                             uint32_t* saved = nullptr, uint32_t* flag = nullptr,
                             bool force = true);
size_t batch_workspace_bytes(uint64_t nbatches, uint64_t nitems);
// True when launch_verify_batch over these batches (no skip list, no fork) writes its outputs
// from ONE kernel, the fused tail of a lone large batch: status / fail_index may then be
// host-mapped (fine-grained) memory, written in place, with no copy back.
bool verify_batch_outputs_direct(uint64_t nbatches, uint64_t nitems);
// Bytes of the fused launches' counters; a caller on that path may pass launch_verify_batch
// a zeroed device array of this size (fuse_ctr, e.g. shipped with its inputs' H2D copy),
// which saves the kernel that would zero them.
size_t verify_batch_fuse_ctr_bytes();
// Input gate of a lone fused batch whose inputs the CPU is still writing into host-mapped
// device memory when the launch is queued (nw_jobs.cpp submit_batch): the head's vote waves
// wait until flags[vote / chunk] == seq (a system-scope load, then a system-scope acquire),
// so the kernels start while the bytes are in flight. digests and offsets must be written
// before the launch. verify_batch_gate_ok: the batch takes the fused head (the only launch
// that honours the gate). chunk: a multiple of 64 votes.
struct input_gate_t {
  const uint32_t* flags;
  uint32_t seq;
  uint32_t chunk;
};
bool verify_batch_gate_ok(uint64_t nbatches, uint64_t nitems);
// done (optional, host-mapped; lone fused batches only, verify_batch_outputs_direct): the
// fused tail stores done_seq there (system scope) right after the verdict, so a host may
// spin on it instead of waiting for the launch's completion signal.
// skip_group_ok (optional, device): batch b is settled (status Ok) when
// skip_group_ok[b / skip_per_group] != 0 (launch_cert_groups, launch_votes_keyed);
// active_frac: the caller's estimate of the fraction of votes not skipped (chunk sizing).
hipError_t launch_verify_batch(const uint32_t* digests, const uint64_t* offsets,
                               const uint64_t* host_offsets, uint64_t nbatches,
                               const uint32_t* pks, const uint32_t* sigs, uint64_t nitems,
                               const uint32_t* z16, const z_key_t& zkey, void* workspace,
                               int32_t* status, uint64_t* fail_index, hipStream_t stream,
                               const key_tables_t* keys = nullptr,
                               const uint32_t* skip_group_ok = nullptr,
                               uint64_t skip_per_group = 0, double active_frac = 1.0,
                               uint32_t* fuse_ctr = nullptr,
                               const input_gate_t* gate = nullptr,
                               uint32_t* done = nullptr, uint32_t done_seq = 0);

// Certificate::verify vote batches merged over groups of certificates (nw_batch.hip):
// cert_group_size() = certificates per group, 0 when the merge does not apply;
// group scratch = cert_groups_bytes(ncert); the batch workspace is the same as
// launch_verify_batch's (batch_workspace_bytes(ncert, nvotes)). *group_ok_out points into
// group_ws (1 per group that passed).
struct ge;
// target_votes: votes per merged group (0 = do not merge); NW_CERT_GROUP_VOTES overrides.
uint64_t cert_group_size(const uint64_t* host_cvo, uint64_t ncert, uint64_t nkeys,
                         bool injected_z, uint64_t target_votes);
bool cert_group_env_fixed();
// fb (host-mapped, 8 words): [0] sequence, [1] groups, [2] groups that failed, [3] tag,
// [4] counted certificates, [5] counted certificates whose vote batch failed. cnt: 3 device
// words, zero before the first call (left zero). Launch after the per-certificate
// verify_batch (batch_st final); group_ok may be null (K = 0).
hipError_t launch_group_feedback(const uint32_t* group_ok, uint64_t ncert, uint64_t K,
                                 uint32_t tag, const int32_t* batch_st, const int32_t* pre1,
                                 const int32_t* pre2, const int32_t* hdr_st, uint32_t* cnt,
                                 uint32_t* fb, hipStream_t stream);
size_t cert_groups_bytes(uint64_t ncert);
const ge* key_tables_base(const ge_niels_pad* tabs, uint64_t nkeys, const keyspec& ks);
hipError_t launch_cert_groups(const uint32_t* cert_digest, const uint64_t* cvo,
                              const uint64_t* host_cvo, uint64_t ncert, const uint32_t* pks,
                              const uint32_t* sigs, uint64_t nvotes, const z_key_t& zkey,
                              void* batch_ws, void* group_ws, const int32_t* pre1,
                              const int32_t* pre2, const int32_t* hdr_st,
                              const key_tables_t& keys, const ge* key_base, uint32_t nkeys,
                              uint64_t K, uint32_t** group_ok_out, hipStream_t stream);
// Small groups: K certificates per keyed Straus check, then the per-certificate
// verify_batch of the certificates of failed groups from the same per-vote items. Writes
// status / fail_index for every certificate (in place of launch_verify_batch);
// cert_sgroup_size() picks K for an estimated fraction p_cert of certificates whose votes
// fail (NW_CERT_SMALL_K fixes it), 0 when merging does not apply; *beats_per_cert: the
// cost model prefers these groups to every certificate's own ladder. keys.vote_key required.
uint64_t cert_sgroup_size(const uint64_t* host_cvo, uint64_t ncert, uint64_t nkeys,
                          bool injected_z, double p_cert, bool* beats_per_cert);
hipError_t launch_cert_sgroups(const uint32_t* cert_digest, const uint64_t* cvo,
                               const uint64_t* host_cvo, uint64_t ncert, const uint32_t* pks,
                               const uint32_t* sigs, uint64_t nvotes, const z_key_t& zkey,
                               void* batch_ws, void* group_ws, const int32_t* pre1,
                               const int32_t* pre2, const int32_t* hdr_st,
                               const key_tables_t& keys, uint32_t nkeys, uint64_t K,
                               double p_cert, int32_t* status, uint64_t* fail_index,
                               uint32_t** group_ok_out, hipStream_t stream);
// Keyed vote checks (nw_kernels.hip): every undecided certificate's votes
// through the keyed comb one by one, R compared in compressed form (no decompression; the
// x parities in batched inversions); cert_ok[c] = 1 when all of them pass (then
// verify_batch is Ok too), 0 otherwise. Follow with launch_verify_batch(skip_group_ok =
// cert_ok, skip_per_group = 1). vote_cert: certificate of each vote (k_cert_prepare);
// cert_ok: ncert words; scratch: >= votes_keyed_fixed_bytes() + 64 x
// votes_keyed_bytes_per_vote() bytes (slices of the votes go through it, each checked in
// key-major order). keys.vote_key required; nkeys = committee size.
// hdr_st may be NULL (votes checked concurrently with the headers); then follow the join
// with launch_cert_ok_headers so header-failed certificates skip their verify_batch.
hipError_t launch_cert_ok_headers(const int32_t* hdr_st, uint64_t ncert, uint32_t* cert_ok,
                                  hipStream_t stream);
size_t votes_keyed_bytes_per_vote();
size_t votes_keyed_fixed_bytes();
hipError_t launch_votes_keyed(const uint32_t* cert_digest, const uint64_t* cvo, uint64_t ncert,
                              const uint32_t* vote_cert, const uint32_t* pks,
                              const uint32_t* sigs, uint64_t nvotes, const int32_t* pre1,
                              const int32_t* pre2, const int32_t* hdr_st,
                              const key_tables_t& keys, uint32_t nkeys, uint32_t* cert_ok,
                              void* scratch, size_t scratch_bytes, hipStream_t stream);

// ---- primary messages (nw_cert.hip) ----------------------------------------------------
struct cert_committee_t {
  uint64_t nauth;
  const uint32_t* pks;              // nauth x 8 words, sorted by bytes
  const uint32_t* stakes;
  const uint64_t* worker_offsets;   // nauth + 1
  const uint32_t* worker_ids;
};

struct cert_stream_t {
  uint64_t n;
  const uint8_t* header_bytes;
  const uint64_t* header_offsets;   // n + 1
  const uint32_t* payload_counts;
  const uint32_t* ids;              // n x 8 words
  const uint64_t* vote_offsets;     // n + 1
  const uint32_t* vote_pks;         // nvotes x 8 words
};

hipError_t launch_cert_prepare(const cert_committee_t& com, const cert_stream_t& cs,
                               int headers_only, const uint32_t* hdr_digest, uint32_t* authors,
                               uint32_t* cert_digest, int32_t* pre1, int32_t* pre2,
                               uint64_t* idx1, uint64_t* idx2, uint32_t* vote_key,
                               uint32_t* author_key, uint32_t* vote_cert, uint64_t nvotes,
                               hipStream_t stream);
hipError_t launch_cert_finalize(uint64_t n, int headers_only, const int32_t* pre1,
                                const int32_t* pre2, const uint64_t* idx1, const uint64_t* idx2,
                                const int32_t* hdr_status, const int32_t* batch_status,
                                const uint64_t* batch_index, int32_t* status, uint64_t* index,
                                hipStream_t stream);
hipError_t launch_vote_prepare(const cert_committee_t& com, uint64_t n, const uint32_t* ids,
                               const uint64_t* rounds, const uint32_t* origins,
                               const uint32_t* authors, uint32_t* digests, int32_t* pre,
                               uint32_t* author_key, hipStream_t stream);
hipError_t launch_vote_finalize(uint64_t n, const int32_t* pre, const int32_t* sig_status,
                                int32_t* status, hipStream_t stream);

// ---- small jobs in one launch (nw_small.hip) --------------------------------------------
// Header / Vote / Certificate checks of a small job (the aggregation service's latency
// path): one launch, no copies (inputs read from and outputs written to the job's pinned
// host buffer), only read access to the committee's key tables and the B comb.
enum : uint32_t { kSmallCerts = 0, kSmallHeaders = 1, kSmallVotes = 2 };
// One signature ("slot"): message m, j = 0 for the header signature (or the vote's own), j >= 1
// for certificate vote j - 1; v = global index of that vote (for j = 0 of a certificate: of
// its first vote); cnt = slots of the message (1 + votes for a certificate, else 1).
struct small_slot_t {
  uint32_t m, j, v, cnt;
};
struct small_msg_info_t {
  int32_t p1, p2;   // pre-signature verdicts: header level (-1 = genesis) / quorum
  uint64_t x1, x2;
};
struct small_job_t {
  uint32_t kind;           // kSmall*
  uint32_t slots_per_wg;   // S: 4, 8, 16, 32 or 64
  uint64_t nmsg, nslots;
  cert_committee_t com;    // 1..256 authorities
  // headers / certificates (nw_certificates layout; header offsets rebased to 0)
  const uint8_t* hb;
  const uint64_t* ho;
  const uint32_t* pc;
  const uint32_t* ids;     // also the votes' header ids
  const uint32_t* hsig;
  const uint32_t* vpk;     // certificate votes
  const uint32_t* vsig;
  const uint32_t* z16;     // optional injected batch coefficients (per vote)
  // votes (Vote::verify)
  const uint64_t* rounds;
  const uint32_t* origins;
  const uint32_t* authors;
  const uint32_t* sigs;
  const small_slot_t* slots;
  // device: the committee's key tables (built for exactly these keys) and the B comb
  const struct ge_niels_pad* ktabs;
  const uint32_t* kok;
  keyspec ks;              // the key tables' layout
  const struct ge_niels_pad* bcomb;
  uint32_t zkey[8];        // ChaCha20 key of the batch coefficients when z16 is null
  // device scratch: message info and slot records of messages spanning workgroups, and
  // the per-message arrival counters (zero before the launch, left zero after it)
  small_msg_info_t* minfo;
  uint32_t* srec;
  uint32_t* mcount;
  // outputs (pinned host memory)
  int32_t* status;
  uint64_t* index;
  uint64_t* stamps;        // diagnostics (NW_SMALL_STAMPS): 8 phase times per workgroup, or null
  // optional (pinned): workgroup w stores done_seq into done_flags[w] (system scope) after
  // its last status / index write, so the host sees the job finished before its completion
  // event (a workgroup that stored nothing just leaves the host waiting for the event)
  uint32_t* done_flags;
  uint32_t done_seq;
};
hipError_t upload_small_consts();
hipError_t launch_small(const small_job_t& job, hipStream_t stream);
// The keyed comb's B tables of the current device (built on first use).
hipError_t bcomb_table(const struct ge_niels_pad** out);

}  // namespace nw
