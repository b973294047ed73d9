// nw_api.cpp — C ABI (include/narwhal_amd.h) over the gfx950 kernels.
//
// Runtime model: one host thread may drive any device; each thread owns, per device, one
// HIP stream and grow-only device/pinned staging buffers (no allocation on the steady
// path, no shared mutable state between threads, so the ABI is re-entrant the way the
// reference's Send + Sync crypto types are). Constants are uploaded once per device.
// There is no CPU fallback: without a gfx950 device every call fails with NW_E_NO_DEVICE.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "narwhal_amd.h"
#include "nw_kernels.h"
#include "nw_runtime.h"

namespace {

constexpr int kMaxDevices = 64;

std::once_flag g_init_once;
int g_init_status = NW_E_NO_DEVICE;   // device count or negative error
int g_ndev = 0;
int g_dev_ids[kMaxDevices];           // HIP ordinal of usable device i

struct DevCtx {
  hipStream_t stream = nullptr;
  void* dbuf = nullptr;
  size_t dcap = 0;
};

// Per-device buffers shared by all threads and streams, ordered by an event chain
// (nw::rt::Lease, nw_runtime.h).
struct SharedDev {
  std::mutex m;
  void* strict_ws = nullptr;   // per-lane tables of k_verify_strict (fixed size)
  void* ktabs = nullptr;       // committee key tables (grow-only)
  uint32_t* kok = nullptr;
  size_t kcap = 0;             // keys
  uint32_t kW = 0;             // their comb width (nw::keyspec)
  uint32_t* ksaved = nullptr;  // the keys the tables were last built from (device)
  uint32_t* kflag = nullptr;   // rebuild flag (device, written by k_key_cmp)
  size_t ksaved_n = 0;         // their count; 0 = none
  hipEvent_t last = nullptr;   // completion of the last leased launch sequence
  bool last_valid = false;
  std::vector<uint8_t> khost;  // host copy of the keys the tables hold (empty = unknown)
  // 16-bit tables of the same committee for small jobs while ktabs are wider (Lease::
  // small_tables): their allocation (keys), their ok words, the keys they hold (host)
  void* stabs = nullptr;
  uint32_t* sok = nullptr;
  size_t scap = 0;
  std::vector<uint8_t> shost;
  std::vector<hipEvent_t> readers;   // small jobs (ReadLease) queued since the last Lease
  std::vector<hipEvent_t> rpool;     // recycled reader events
};
SharedDev g_shared[kMaxDevices];

struct ThreadState {
  int device = 0;
  std::string err;
  DevCtx ctx[kMaxDevices];
  ~ThreadState() {
    for (int i = 0; i < kMaxDevices; ++i) {
      if (ctx[i].stream || ctx[i].dbuf) {
        (void)hipSetDevice(g_dev_ids[i]);
        if (ctx[i].dbuf) (void)hipFree(ctx[i].dbuf);
        if (ctx[i].stream) (void)hipStreamDestroy(ctx[i].stream);
      }
    }
  }
};
thread_local ThreadState t_state;

int set_err(int code, const char* what, hipError_t e = hipSuccess) {
  char buf[256];
  if (e != hipSuccess)
    snprintf(buf, sizeof(buf), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
  else
    snprintf(buf, sizeof(buf), "%s", what);
  t_state.err = buf;
  return code;
}

void do_init() {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    g_init_status = NW_E_NO_DEVICE;
    return;
  }
  int n = 0;
  for (int d = 0; d < count && n < kMaxDevices; ++d) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) != hipSuccess) continue;
    if (strncmp(p.gcnArchName, "gfx950", 6) != 0) continue;
    g_dev_ids[n++] = d;   // constants are uploaded on the device's first use (activate)
  }
  g_ndev = n;
  g_init_status = n > 0 ? n : NW_E_NO_DEVICE;
}

// Per-device first use: the constant tables go to a device only when a call selects it, so a
// process that drives one GPU (one rank per GPU) never loads the module on the others.
std::once_flag g_dev_once[kMaxDevices];
hipError_t g_dev_status[kMaxDevices];

int activate(int dev) {
  hipError_t e = hipSetDevice(g_dev_ids[dev]);
  if (e != hipSuccess) return set_err(NW_E_DEVICE, "hipSetDevice", e);
  std::call_once(g_dev_once[dev], [dev] { g_dev_status[dev] = nw::upload_consts(); });
  if (g_dev_status[dev] != hipSuccess)
    return set_err(NW_E_DEVICE, "device initialisation (constant upload)", g_dev_status[dev]);
  return 0;
}

int ensure_init() {
  std::call_once(g_init_once, do_init);
  if (g_init_status < 0)
    return set_err(g_init_status, g_init_status == NW_E_NO_DEVICE
                                      ? "no gfx950 (MI355X) device visible"
                                      : "device initialisation failed");
  return 0;
}

// Select the thread's device, create its stream lazily.
int begin(DevCtx** out) {
  int rc = ensure_init();
  if (rc) return rc;
  int dev = t_state.device;
  if (dev == NW_ALL_DEVICES)
    return set_err(NW_E_INVALID_ARG, "this entry point runs on one device: nw_set_device(d), "
                                     "d >= 0 (NW_ALL_DEVICES fans out host-buffer calls only)");
  if (dev < 0 || dev >= g_ndev) return set_err(NW_E_INVALID_ARG, "bad device index");
  rc = activate(dev);
  if (rc) return rc;
  DevCtx& c = t_state.ctx[dev];
  if (!c.stream) {
    hipError_t e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
    if (e != hipSuccess) return set_err(NW_E_DEVICE, "hipStreamCreate", e);
  }
  *out = &c;
  return 0;
}

int reserve(DevCtx& c, size_t bytes) {
  if (bytes <= c.dcap) return 0;
  if (c.dbuf) {
    (void)hipStreamSynchronize(c.stream);
    (void)hipFree(c.dbuf);
    c.dbuf = nullptr;
    c.dcap = 0;
  }
  size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
  hipError_t e = hipMalloc(&c.dbuf, cap);
  if (e != hipSuccess) return set_err(NW_E_OUT_OF_MEMORY, "hipMalloc", e);
  c.dcap = cap;
  return 0;
}

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

int os_random(void* buf, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = getrandom(static_cast<char*>(buf) + got, n - got, 0);
    if (r <= 0) return set_err(NW_E_DEVICE, "getrandom failed");
    got += (size_t)r;
  }
  return 0;
}

#define NW_HIP(call, what)                                                              \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err(e_ == hipErrorOutOfMemory ? NW_E_OUT_OF_MEMORY : NW_E_DEVICE, what, e_); \
  } while (0)

hipStream_t pick_stream(void* s, DevCtx* c) {
  return s ? static_cast<hipStream_t>(s) : c->stream;
}

}  // namespace

extern "C" {

int nw_init(void) {
  int rc = ensure_init();
  return rc ? rc : g_ndev;
}

int nw_device_count(void) {
  std::call_once(g_init_once, do_init);
  return g_init_status > 0 ? g_ndev : 0;
}

int nw_set_device(int device) {
  int rc = ensure_init();
  if (rc) return rc;
  if (device != NW_ALL_DEVICES && (device < 0 || device >= g_ndev))
    return set_err(NW_E_INVALID_ARG, "bad device index");
  t_state.device = device;
  return 0;
}

int nw_get_device(void) { return t_state.device; }

const char* nw_last_error(void) { return t_state.err.c_str(); }

const char* nw_version(void) { return "narwhal_amd 0.1.0 gfx950"; }

int nw_prepare(void) {
  int rc = ensure_init();
  if (rc) return rc;
  const int dev = t_state.device;
  if (dev != NW_ALL_DEVICES && (dev < 0 || dev >= g_ndev))
    return set_err(NW_E_INVALID_ARG, "bad device index");
  for (int d = dev == NW_ALL_DEVICES ? 0 : dev; d < (dev == NW_ALL_DEVICES ? g_ndev : dev + 1);
       ++d) {
    rc = activate(d);
    if (rc) return rc;
    const hipError_t e = nw::prepare_strict_tables();
    if (e == hipErrorOutOfMemory)
      return set_err(NW_E_OUT_OF_MEMORY,
                     "device memory for the strict B tables (2.15 GB) or the keyed B comb "
                     "(11.8 GB); without the comb, committee checks run without key tables",
                     e);
    NW_HIP(e, "strict table build");
  }
  return 0;
}

int nw_synchronize(void) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  NW_HIP(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  return 0;
}

// ------------------------------------------------------------------------------------
int nw_dev_sha512_digest32_many(const void* data, const uint64_t* offsets,
                                const uint64_t* lengths, size_t n, void* out32, void* stream) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (n && (!data || !offsets || !lengths || !out32))
    return set_err(NW_E_INVALID_ARG, "null pointer");
  NW_HIP(nw::launch_sha512_digest32(static_cast<const uint8_t*>(data), offsets, lengths, n,
                                    static_cast<uint32_t*>(out32), pick_stream(stream, c)),
         "k_sha512_digest32 launch");
  return 0;
}

// ------------------------------------------------------------------------------------
int nw_dev_verify_strict_many(const void* digests, size_t digest_stride, const void* pks,
                              const void* sigs, size_t n, int32_t* status_out,
                              void* bitmap_out, void* stream) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (n == 0) return 0;
  if (!digests || !pks || !sigs || !status_out || !bitmap_out)
    return set_err(NW_E_INVALID_ARG, "null pointer (status_out and bitmap_out are required)");
  if (digest_stride != 0 && digest_stride != 32)
    return set_err(NW_E_INVALID_ARG, "digest_stride must be 0 or 32");
  const hipStream_t s = pick_stream(stream, c);
  nw::rt::Lease lease;
  void* ws;
  rc = lease.acquire(t_state.device, s);
  if (!rc) rc = lease.strict_ws(&ws);
  if (rc) return rc;
  NW_HIP(nw::launch_verify_strict(static_cast<const uint32_t*>(digests),
                                  (uint32_t)(digest_stride / 4),
                                  static_cast<const uint32_t*>(pks),
                                  static_cast<const uint32_t*>(sigs), n, status_out,
                                  static_cast<uint64_t*>(bitmap_out), ws, s),
         "k_verify_strict launch");
  return lease.release();
}

// ------------------------------------------------------------------------------------
int nw_dev_keypair_from_seed_many(const void* seeds, size_t n, void* pks_out, void* stream) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (n && (!seeds || !pks_out)) return set_err(NW_E_INVALID_ARG, "null pointer");
  NW_HIP(nw::launch_keypair(static_cast<const uint32_t*>(seeds), n,
                            static_cast<uint32_t*>(pks_out), pick_stream(stream, c)),
         "k_keypair launch");
  return 0;
}

int nw_dev_sign_many(const void* sks, size_t sk_stride, const void* digests,
                     size_t digest_stride, size_t n, void* sigs_out, void* stream) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (n && (!sks || !digests || !sigs_out)) return set_err(NW_E_INVALID_ARG, "null pointer");
  if ((sk_stride != 0 && sk_stride != 64) || (digest_stride != 0 && digest_stride != 32))
    return set_err(NW_E_INVALID_ARG, "sk_stride must be 0/64, digest_stride 0/32");
  NW_HIP(nw::launch_sign(static_cast<const uint32_t*>(sks), (uint32_t)(sk_stride / 4),
                         static_cast<const uint32_t*>(digests), (uint32_t)(digest_stride / 4),
                         n, static_cast<uint32_t*>(sigs_out), pick_stream(stream, c)),
         "k_sign launch");
  return 0;
}

int nw_keypair_from_seed_many(const uint8_t* seeds, size_t n, uint8_t* pks_out) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (n == 0) return 0;
  if (!seeds || !pks_out) return set_err(NW_E_INVALID_ARG, "null pointer");
  rc = reserve(*c, 2 * a256(32 * n));
  if (rc) return rc;
  uint8_t* d_in = static_cast<uint8_t*>(c->dbuf);
  uint8_t* d_out = d_in + a256(32 * n);
  hipStream_t s = c->stream;
  NW_HIP(hipMemcpyAsync(d_in, seeds, 32 * n, hipMemcpyHostToDevice, s), "H2D seeds");
  NW_HIP(nw::launch_keypair(reinterpret_cast<const uint32_t*>(d_in), n,
                            reinterpret_cast<uint32_t*>(d_out), s), "k_keypair launch");
  NW_HIP(hipMemcpyAsync(pks_out, d_out, 32 * n, hipMemcpyDeviceToHost, s), "D2H pks");
  NW_HIP(hipStreamSynchronize(s), "sync");
  return 0;
}

int nw_sign_many(const uint8_t* sks, size_t sk_stride, const uint8_t* digests,
                 size_t digest_stride, size_t n, uint8_t* sigs_out) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (n == 0) return 0;
  if (!sks || !digests || !sigs_out) return set_err(NW_E_INVALID_ARG, "null pointer");
  if ((sk_stride != 0 && sk_stride != 64) || (digest_stride != 0 && digest_stride != 32))
    return set_err(NW_E_INVALID_ARG, "sk_stride must be 0/64, digest_stride 0/32");
  const size_t nk = sk_stride ? n : 1, nm = digest_stride ? n : 1;
  const size_t b_k = a256(64 * nk), b_m = a256(32 * nm), b_s = a256(64 * n);
  rc = reserve(*c, b_k + b_m + b_s);
  if (rc) return rc;
  uint8_t* d_k = static_cast<uint8_t*>(c->dbuf);
  uint8_t* d_m = d_k + b_k;
  uint8_t* d_s = d_m + b_m;
  hipStream_t s = c->stream;
  NW_HIP(hipMemcpyAsync(d_k, sks, 64 * nk, hipMemcpyHostToDevice, s), "H2D sks");
  NW_HIP(hipMemcpyAsync(d_m, digests, 32 * nm, hipMemcpyHostToDevice, s), "H2D digests");
  NW_HIP(nw::launch_sign(reinterpret_cast<const uint32_t*>(d_k), (uint32_t)(sk_stride / 4),
                         reinterpret_cast<const uint32_t*>(d_m), (uint32_t)(digest_stride / 4),
                         n, reinterpret_cast<uint32_t*>(d_s), s), "k_sign launch");
  NW_HIP(hipMemcpyAsync(sigs_out, d_s, 64 * n, hipMemcpyDeviceToHost, s), "D2H sigs");
  NW_HIP(hipStreamSynchronize(s), "sync");
  return 0;
}

// ------------------------------------------------------------------------------------
size_t nw_dev_verify_batch_workspace(size_t nbatches, size_t nitems) {
  return nw::batch_workspace_bytes(nbatches, nitems);
}

static int fill_key(nw::z_key_t& k, const uint8_t* key32) {
  if (key32) {
    memcpy(k.key, key32, 32);
  } else {
    int rc = os_random(k.key, 32);
    if (rc) return rc;
  }
  k.nonce = 0;
  return 0;
}

// Host copy of the batch offsets: the caller's, or read back from the device (blocking).
static int host_offsets_of(const uint64_t* dev_offsets, const uint64_t* host_offsets,
                           size_t nbatches, hipStream_t s, std::vector<uint64_t>& tmp,
                           const uint64_t** out) {
  if (host_offsets) {
    *out = host_offsets;
    return 0;
  }
  tmp.resize(nbatches + 1);
  NW_HIP(hipMemcpyAsync(tmp.data(), dev_offsets, 8 * (nbatches + 1), hipMemcpyDeviceToHost, s),
         "D2H offsets");
  NW_HIP(hipStreamSynchronize(s), "sync (offsets)");
  *out = tmp.data();
  return 0;
}

int nw_dev_verify_batch_many(const void* digests, const void* pks, const void* sigs,
                             const uint64_t* offsets, const uint64_t* host_offsets,
                             size_t nbatches, size_t nitems, const void* z16,
                             const uint8_t* zkey32, void* workspace, int32_t* status_out,
                             uint64_t* fail_index, void* stream) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (nbatches == 0) return 0;
  if (!digests || !offsets || !workspace || !status_out || (nitems && (!pks || !sigs)))
    return set_err(NW_E_INVALID_ARG, "null pointer");
  nw::z_key_t key;
  rc = fill_key(key, zkey32);
  if (rc) return rc;
  hipStream_t s = pick_stream(stream, c);
  std::vector<uint64_t> tmp;
  const uint64_t* ho;
  rc = host_offsets_of(offsets, host_offsets, nbatches, s, tmp, &ho);
  if (rc) return rc;
  if (ho[0] != 0 || ho[nbatches] != nitems)
    return set_err(NW_E_INVALID_ARG, "offsets must run from 0 to nitems");
  NW_HIP(nw::launch_verify_batch(static_cast<const uint32_t*>(digests), offsets, ho, nbatches,
                                 static_cast<const uint32_t*>(pks),
                                 static_cast<const uint32_t*>(sigs), nitems,
                                 static_cast<const uint32_t*>(z16), key, workspace, status_out,
                                 fail_index, s),
         "verify_batch launch");
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// Primary messages: Header::verify / Vote::verify / Certificate::verify
// (primary/src/messages.rs:48-67, 131-142, 189-215). The device pipelines below serve the
// device-pointer entry point here and the job entry points (nw_submit_certificates_* /
// nw_submit_headers_* / nw_submit_votes_*, nw_jobs.cpp), which the blocking calls wrap.
// ------------------------------------------------------------------------------------
namespace {

struct CertWs {
  uint32_t *hdr_digest, *authors, *cert_digest;
  int32_t *pre1, *pre2, *hdr_st, *batch_st;
  uint64_t *idx1, *idx2, *batch_idx, *bitmap;
  void* batch_ws;
  uint32_t* vote_key;
  uint32_t* author_key;
  void* group_ws;
  uint32_t* vote_cert;
  size_t batch_ws_bytes;
};

size_t cert_ws_layout(size_t n, size_t nvotes, char* base, CertWs* w) {
  const size_t m = n ? n : 1;
  // the verify_batch workspace doubles as the keyed vote checks' scratch (they run first)
  const size_t bws = nvotes ? a256(std::max(nw::batch_workspace_bytes(n, nvotes),
                                            nw::votes_keyed_fixed_bytes() +
                                                64 * nw::votes_keyed_bytes_per_vote()))
                            : 256;
  const size_t sizes[16] = {a256(32 * m), a256(32 * m), a256(32 * m), a256(4 * m), a256(4 * m),
                            a256(4 * m),  a256(4 * m),  a256(8 * m),  a256(8 * m), a256(8 * m),
                            a256(8 * ((m + 63) / 64)), bws,
                            a256(4 * (nvotes ? nvotes : 1)), a256(4 * m),
                            nvotes ? a256(nw::cert_groups_bytes(n)) : 256,
                            a256(4 * (nvotes ? nvotes : 1))};
  size_t off[16], tot = 0;
  for (int k = 0; k < 16; ++k) { off[k] = tot; tot += sizes[k]; }
  if (w) {
    w->hdr_digest = reinterpret_cast<uint32_t*>(base + off[0]);
    w->authors = reinterpret_cast<uint32_t*>(base + off[1]);
    w->cert_digest = reinterpret_cast<uint32_t*>(base + off[2]);
    w->pre1 = reinterpret_cast<int32_t*>(base + off[3]);
    w->pre2 = reinterpret_cast<int32_t*>(base + off[4]);
    w->hdr_st = reinterpret_cast<int32_t*>(base + off[5]);
    w->batch_st = reinterpret_cast<int32_t*>(base + off[6]);
    w->idx1 = reinterpret_cast<uint64_t*>(base + off[7]);
    w->idx2 = reinterpret_cast<uint64_t*>(base + off[8]);
    w->batch_idx = reinterpret_cast<uint64_t*>(base + off[9]);
    w->bitmap = reinterpret_cast<uint64_t*>(base + off[10]);
    w->batch_ws = base + off[11];
    w->vote_key = reinterpret_cast<uint32_t*>(base + off[12]);
    w->author_key = reinterpret_cast<uint32_t*>(base + off[13]);
    w->group_ws = base + off[14];
    w->vote_cert = reinterpret_cast<uint32_t*>(base + off[15]);
    w->batch_ws_bytes = bws;
  }
  return tot;
}

// Certificate vote policy. The default is the keyed vote checks (every vote
// of an undecided certificate through its committee key's comb tables, R compared in
// compressed form; verify_batch only for certificates with a failing vote): faster than
// merged groups at every committee size (config 2 all-valid, N = 4 / 10 / 50 / 100: 113.6 /
// 60.8 / 15.1 / 7.84 vs 95.2 / 48.9 / 11.6 / 6.08 M certs/s with big groups,
// gpurun_out/r03a) and with nothing shared that a bad vote can spoil. With NW_CERT_KEYED=0
// the merged-group policy runs instead, adaptive on the fraction p of counted certificates
// whose vote batch failed in earlier calls (k_grp_count / k_grp_publish, host-mapped):
//   big    Pippenger groups of ~32k votes (launch_cert_groups) while at most a quarter of
//          them would fail at that p, 1 - (1 - p)^K <= 1/4;
//   small  otherwise (or when merging does not apply) K-certificate keyed Straus groups with
//          the fallback ladders run from the same per-vote items (launch_cert_sgroups), K
//          cost-optimal at that p (cert_sgroup_size), when they beat every certificate's own
//          ladder; per-certificate otherwise.
// In keyed mode the reported p only sizes the fallback batches' chunks. Verdicts never
// depend on the choice; NW_CERT_GROUP_VOTES fixes big groups of that size,
// NW_CERT_SMALL_K small groups of K certificates, NW_CERT_MERGE=0 turns merging (and the
// keyed checks) off: every certificate's own verify_batch.
constexpr uint32_t kGroupDefault = 32768;

// The default certificate vote policy: the keyed vote checks (see above).
bool keyed_policy(size_t nauth) {
  const char* ke = getenv("NW_CERT_KEYED");
  const char* me = getenv("NW_CERT_MERGE");
  return nauth > 0 && !(ke && atoi(ke) == 0) && !(me && me[0] == '0') &&
         !getenv("NW_CERT_SMALL_K") && !nw::cert_group_env_fixed();
}

struct GroupPolicy {
  uint32_t* fb = nullptr;       // host-mapped: seq, groups, failed, tag, counted, bad
  uint32_t* fb_dev = nullptr;
  uint32_t* cnt = nullptr;      // device: k_grp_count's sums (zero between calls)
  uint32_t seen = 0;
  double p = 0.0;               // fraction of counted certificates whose votes failed
};
struct DevPolicies {
  std::mutex m;
  std::unordered_map<uint64_t, GroupPolicy> by_committee;
};
DevPolicies g_policies[kMaxDevices];

// The latest failure-rate report for this committee (key hash, or size), and where this
// call's goes.
double group_failure_rate(int dev, uint64_t nkeys, hipStream_t s, uint32_t** fb_dev,
                          uint32_t** cnt) {
  DevPolicies& d = g_policies[dev];
  std::lock_guard<std::mutex> g(d.m);
  GroupPolicy& p = d.by_committee[nkeys];
  *fb_dev = nullptr;
  *cnt = nullptr;
  if (!p.fb) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 32, hipHostMallocMapped) != hipSuccess) return p.p;
    memset(h, 0, 32);
    void* dp = nullptr;
    void* c = nullptr;
    if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess || hipMalloc(&c, 16) != hipSuccess ||
        hipMemsetAsync(c, 0, 16, s) != hipSuccess) {   // ordered before this call's count
      (void)hipHostFree(h);
      return p.p;
    }
    p.fb = static_cast<uint32_t*>(h);
    p.fb_dev = static_cast<uint32_t*>(dp);
    p.cnt = static_cast<uint32_t*>(c);
  }
  volatile uint32_t* fb = p.fb;
  const uint32_t seq = fb[0];
  if (seq != p.seen) {          // a report from a call that has finished since
    p.seen = seq;
    const uint32_t counted = fb[4], bad = fb[5];
    if (counted) p.p = (double)bad / (double)counted;
  }
  *fb_dev = p.fb_dev;
  *cnt = p.cnt;
  return p.p;
}

}  // namespace

namespace nw {
namespace rt {

size_t cert_workspace_bytes(size_t n, size_t nvotes) {
  return cert_ws_layout(n, nvotes, nullptr, nullptr);
}

// Key tables for a keyed pipeline, or (out of device memory for them or for the keyed B
// comb) *use_keys = false and 0: the caller then runs unkeyed.
static int keyed_tables_or_fallback(Lease& lease, size_t nauth, void** tabs, uint32_t** ok,
                                    nw::keyspec* ks, uint32_t** saved, uint32_t** flag,
                                    bool* force, bool* use_keys) {
  const nw::ge_niels_pad* bc = nullptr;
  const hipError_t eb = nw::bcomb_table(&bc);
  if (eb == hipErrorOutOfMemory) {
    *use_keys = false;
    return 0;
  }
  if (eb != hipSuccess) return ::set_err(NW_E_DEVICE, "keyed B comb build", eb);
  const int rc = lease.key_tables(nauth, tabs, ok, ks, saved, flag, force);
  if (rc == NW_E_OUT_OF_MEMORY) {
    *use_keys = false;
    return 0;
  }
  return rc;
}

// The whole device pipeline; every pointer is a device pointer.
uint64_t committee_hash(const nw_committee* com) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < 32 * com->nauth; ++i) h = (h ^ com->pks[i]) * 1099511628211ull;
  return h ? h : 1;
}

int cert_pipeline(int dev, const nw_committee& com, const nw_certificates& cs,
                  const uint64_t* host_vote_offsets, int headers_only, const void* z16,
                  const uint8_t zkey32[32], void* workspace, int32_t* status, uint64_t* index,
                  hipStream_t s, uint64_t committee_tag, const Fork* fork,
                  const uint8_t* host_pks) {
  // the failure-rate policy is kept per committee: keyed by the committee's key
  // hash when the caller knows it, else by the committee size
  const uint64_t policy_key = committee_tag ? committee_tag : (uint64_t)com.nauth;
  const uint64_t n = cs.n;
  if (n == 0) return 0;
  nw::z_key_t key;
  int rc = fill_key(key, zkey32);
  if (rc) return rc;
  CertWs w;
  cert_ws_layout(n, headers_only ? 0 : cs.nvotes, static_cast<char*>(workspace), &w);
  nw::cert_committee_t dc{com.nauth, reinterpret_cast<const uint32_t*>(com.pks), com.stakes,
                          com.worker_offsets, com.worker_ids};
  nw::cert_stream_t ds{n, cs.header_bytes, cs.header_offsets, cs.payload_counts,
                       reinterpret_cast<const uint32_t*>(cs.ids), cs.vote_offsets,
                       reinterpret_cast<const uint32_t*>(cs.vote_pks)};
  NW_HIP(nw::launch_sha512_digest32(cs.header_bytes, cs.header_offsets, nullptr, n,
                                    w.hdr_digest, s), "k_sha512 (header digests)");
  // The committee's keys are decompressed once per call (k_key_base / k_key_tabs) and their
  // tables shared by every header (author) and vote that names a committee member; any
  // other key cannot decide a verdict (k_cert_prepare fails its message first) and is
  // decompressed in the kernel as usual. Key tables and the strict workspace are the
  // device's shared buffers: the lease orders this call after every earlier user.
  nw::rt::Lease lease;
  void* ktabs_v = nullptr;
  uint32_t* kok = nullptr;
  void* sws = nullptr;
  rc = lease.acquire(dev, s);
  uint32_t* ksaved = nullptr;
  uint32_t* kflag = nullptr;
  bool kforce = true;
  // Without device memory for the keyed B comb (11.8 GB) or the committee's key tables
  // (67 MB per key) every check still runs, unkeyed: headers through the strict ladder,
  // votes through each certificate's own verify_batch (same statuses).
  bool use_keys = com.nauth > 0;
  nw::keyspec ks{};
  if (!rc && use_keys) rc = keyed_tables_or_fallback(lease, com.nauth, &ktabs_v, &kok, &ks,
                                                     &ksaved, &kflag, &kforce, &use_keys);
  if (!rc) rc = lease.strict_ws(&sws);
  if (rc) return rc;
  nw::ge_niels_pad* ktabs = static_cast<nw::ge_niels_pad*>(ktabs_v);
  if (use_keys) {
    NW_HIP(nw::launch_key_tables(reinterpret_cast<const uint32_t*>(com.pks), com.nauth, ks,
                                 ktabs, kok, s, ksaved, kflag, kforce),
           "k_key_tables");
    lease.keys_built(com.nauth, host_pks);
    rc = lease.small_tables(reinterpret_cast<const uint32_t*>(com.pks), com.nauth, host_pks);
    if (rc) return rc;
  }
  NW_HIP(nw::launch_cert_prepare(dc, ds, headers_only, w.hdr_digest, w.authors, w.cert_digest,
                                 w.pre1, w.pre2, w.idx1, w.idx2,
                                 headers_only ? nullptr : w.vote_key, w.author_key,
                                 headers_only ? nullptr : w.vote_cert,
                                 headers_only ? 0 : cs.nvotes, s),
         "k_cert_prepare");
  const nw::key_tables_t hk{ktabs, kok, w.author_key, ks};
  // With a fork stream (host-buffer jobs) and the keyed vote checks, the headers run on the
  // fork stream while the votes run here: the votes then do not skip header-failed
  // certificates (k_cert_ok_headers settles those after the join), and the two latency
  // chains of a small call (each a keyed check and one batched inversion) overlap.
  const bool fork_ok = fork && fork->s2 && !headers_only && use_keys && keyed_policy(com.nauth);
  if (fork_ok) {
    NW_HIP(hipEventRecord(fork->ev_fork, s), "hipEventRecord (fork)");
    NW_HIP(hipStreamWaitEvent(fork->s2, fork->ev_fork, 0), "hipStreamWaitEvent (fork)");
  }
  NW_HIP(nw::launch_verify_strict(reinterpret_cast<const uint32_t*>(cs.ids), 8, w.authors,
                                  reinterpret_cast<const uint32_t*>(cs.header_sigs), n, w.hdr_st,
                                  w.bitmap, sws, fork_ok ? fork->s2 : s, use_keys ? &hk : nullptr),
         "k_verify_strict (headers)");
  if (fork_ok) NW_HIP(hipEventRecord(fork->ev_join, fork->s2), "hipEventRecord (join)");
  // every exit (errors included) joins the fork stream back before the lease is released
  struct JoinGuard {
    hipStream_t s = nullptr;
    hipEvent_t e = nullptr;
    ~JoinGuard() {
      if (s) (void)hipStreamWaitEvent(s, e, 0);
    }
  } join_guard;
  if (fork_ok) {
    join_guard.s = s;
    join_guard.e = fork->ev_join;
  }
  if (!headers_only) {
    const nw::key_tables_t kt{ktabs, kok, w.vote_key, ks};
    // Default: the keyed vote checks (launch_votes_keyed): every vote of an undecided
    // certificate through its committee key's comb tables, R compared in compressed form,
    // then verify_batch only for the certificates with a failing vote. A vote that passes
    // its strict check has a zero term in ANY random linear combination, so a certificate
    // whose votes all pass is Ok under verify_batch for every z (random or injected); every
    // other certificate gets its own verify_batch with the call's z. Nothing is shared that
    // one bad vote can spoil, so invalid certificates cost only their own batches.
    // NW_CERT_KEYED=0 selects the merged-group policy instead (big Pippenger groups / small
    // keyed Straus groups, adaptive on the failure rate the previous calls reported),
    // NW_CERT_MERGE=0 every certificate's own verify_batch.
    const bool keyed = use_keys && keyed_policy(com.nauth);
    uint32_t* fb_dev = nullptr;
    uint32_t* fb_cnt = nullptr;
    double p_cert = 0.0;
    uint64_t K = 1;
    bool small = false;
    if (keyed) {
      // the reported failure rate only sizes the fallback batches' chunks
      p_cert = group_failure_rate(dev, policy_key, s, &fb_dev, &fb_cnt);
    } else if (!use_keys) {
      K = 0;   // no key tables: every certificate's own verify_batch, unkeyed
    } else {
      K = nw::cert_group_size(host_vote_offsets, n, com.nauth, z16 != nullptr, kGroupDefault);
      small = getenv("NW_CERT_SMALL_K") != nullptr;
      if (!z16 && !small && !nw::cert_group_env_fixed()) {
        p_cert = group_failure_rate(dev, policy_key, s, &fb_dev, &fb_cnt);
        // merging does not apply, or most big groups would fail at the measured rate
        if (!K || 1.0 - std::pow(1.0 - p_cert, (double)K) > 0.25) small = true;
      }
      if (small) {
        bool wins = false;
        K = nw::cert_sgroup_size(host_vote_offsets, n, com.nauth, z16 != nullptr, p_cert, &wins);
        if (!wins) K = 0;
      }
    }
    if (getenv("NW_DEBUG_GROUPS"))
      fprintf(stderr, "[narwhal_amd] certificates: n=%zu keys=%zu %s K=%llu p=%.4g\n", (size_t)n,
              (size_t)com.nauth, keyed ? "keyed" : small ? "small" : "big",
              (unsigned long long)K, p_cert);
    uint32_t* group_ok = nullptr;
    if (keyed) {
      group_ok = static_cast<uint32_t*>(w.group_ws);
      NW_HIP(nw::launch_votes_keyed(w.cert_digest, cs.vote_offsets, n, w.vote_cert,
                                    reinterpret_cast<const uint32_t*>(cs.vote_pks),
                                    reinterpret_cast<const uint32_t*>(cs.vote_sigs), cs.nvotes,
                                    w.pre1, w.pre2, fork_ok ? nullptr : w.hdr_st, kt,
                                    (uint32_t)com.nauth, group_ok, w.batch_ws,
                                    w.batch_ws_bytes, s),
             "keyed vote checks");
      if (fork_ok) {
        join_guard.s = nullptr;   // joined here
        NW_HIP(hipStreamWaitEvent(s, fork->ev_join, 0), "hipStreamWaitEvent (join)");
        NW_HIP(nw::launch_cert_ok_headers(w.hdr_st, n, group_ok, s), "k_cert_ok_headers");
      }
    } else if (K && !small)
      NW_HIP(nw::launch_cert_groups(w.cert_digest, cs.vote_offsets, host_vote_offsets, n,
                                    reinterpret_cast<const uint32_t*>(cs.vote_pks),
                                    reinterpret_cast<const uint32_t*>(cs.vote_sigs), cs.nvotes,
                                    key, w.batch_ws, w.group_ws, w.pre1, w.pre2, w.hdr_st, kt,
                                    nw::key_tables_base(ktabs, com.nauth, ks), (uint32_t)com.nauth,
                                    K, &group_ok, s),
             "certificate groups (votes)");
    if (K && small)
      NW_HIP(nw::launch_cert_sgroups(w.cert_digest, cs.vote_offsets, host_vote_offsets, n,
                                     reinterpret_cast<const uint32_t*>(cs.vote_pks),
                                     reinterpret_cast<const uint32_t*>(cs.vote_sigs), cs.nvotes,
                                     key, w.batch_ws, w.group_ws, w.pre1, w.pre2, w.hdr_st, kt,
                                     (uint32_t)com.nauth, K, p_cert, w.batch_st, w.batch_idx,
                                     &group_ok, s),
             "small certificate groups (votes)");
    else
      NW_HIP(nw::launch_verify_batch(w.cert_digest, cs.vote_offsets, host_vote_offsets, n,
                                     reinterpret_cast<const uint32_t*>(cs.vote_pks),
                                     reinterpret_cast<const uint32_t*>(cs.vote_sigs), cs.nvotes,
                                     static_cast<const uint32_t*>(z16), key, w.batch_ws,
                                     w.batch_st, w.batch_idx, s, use_keys ? &kt : nullptr,
                                     group_ok, K, keyed ? std::max(p_cert, 1e-3) : 1.0),
             "verify_batch (votes)");
    if (fb_dev)
      NW_HIP(nw::launch_group_feedback(group_ok, n, K,
                                       ((keyed ? 2u : small ? 1u : 0u) << 24) | (uint32_t)K,
                                       w.batch_st, w.pre1, w.pre2, w.hdr_st, fb_cnt, fb_dev,
                                       s),
             "group feedback");
  }
  NW_HIP(nw::launch_cert_finalize(n, headers_only, w.pre1, w.pre2, w.idx1, w.idx2, w.hdr_st,
                                  w.batch_st, w.batch_idx, status, index, s), "k_cert_finalize");
  return lease.release();
}

// Vote::verify: k_vote_prepare (stake, Vote::digest, the author's committee index), then the
// strict check with the committee's key tables — an author that is a committee member (the
// only kind whose signature can decide a verdict) takes the ladder-free keyed comb.
size_t votes_workspace_bytes(size_t n) {
  const size_t m = n ? n : 1;
  return a256(32 * m) + 4 * a256(4 * m) + a256(8 * ((m + 63) / 64));
}

int votes_pipeline(int dev, const nw_committee& com, size_t n, const uint8_t* ids,
                   const uint64_t* rounds, const uint8_t* origins, const uint8_t* authors,
                   const uint8_t* sigs, void* workspace, int32_t* status, hipStream_t s,
                   const uint8_t* host_pks) {
  if (n == 0) return 0;
  char* p = static_cast<char*>(workspace);
  uint32_t* d_dig = reinterpret_cast<uint32_t*>(p); p += a256(32 * n);
  int32_t* d_pre = reinterpret_cast<int32_t*>(p); p += a256(4 * n);
  int32_t* d_sst = reinterpret_cast<int32_t*>(p); p += a256(4 * n);
  uint32_t* d_key = reinterpret_cast<uint32_t*>(p); p += a256(4 * n);
  p += a256(4 * n);
  uint64_t* d_bm = reinterpret_cast<uint64_t*>(p);
  nw::cert_committee_t dc{com.nauth, reinterpret_cast<const uint32_t*>(com.pks), com.stakes,
                          com.worker_offsets, com.worker_ids};
  NW_HIP(nw::launch_vote_prepare(dc, n, reinterpret_cast<const uint32_t*>(ids), rounds,
                                 reinterpret_cast<const uint32_t*>(origins),
                                 reinterpret_cast<const uint32_t*>(authors), d_dig, d_pre, d_key,
                                 s),
         "k_vote_prepare");
  nw::rt::Lease lease;
  void* ktabs = nullptr;
  uint32_t* kok = nullptr;
  uint32_t* ksaved = nullptr;
  uint32_t* kflag = nullptr;
  bool kforce = true;
  void* sws = nullptr;
  int rc = lease.acquire(dev, s);
  bool use_keys = com.nauth > 0;
  nw::keyspec ks{};
  if (!rc && use_keys)
    rc = keyed_tables_or_fallback(lease, com.nauth, &ktabs, &kok, &ks, &ksaved, &kflag,
                                  &kforce, &use_keys);
  if (!rc) rc = lease.strict_ws(&sws);
  if (rc) return rc;
  if (use_keys) {
    NW_HIP(nw::launch_key_tables(reinterpret_cast<const uint32_t*>(com.pks), com.nauth, ks,
                                 static_cast<nw::ge_niels_pad*>(ktabs), kok, s, ksaved, kflag,
                                 kforce),
           "k_key_tables");
    lease.keys_built(com.nauth, host_pks);
    rc = lease.small_tables(reinterpret_cast<const uint32_t*>(com.pks), com.nauth, host_pks);
    if (rc) return rc;
  }
  const nw::key_tables_t kt{static_cast<nw::ge_niels_pad*>(ktabs), kok, d_key, ks};
  NW_HIP(nw::launch_verify_strict(d_dig, 8, reinterpret_cast<const uint32_t*>(authors),
                                  reinterpret_cast<const uint32_t*>(sigs), n, d_sst, d_bm, sws, s,
                                  use_keys ? &kt : nullptr),
         "k_verify_strict (votes)");
  rc = lease.release();
  if (rc) return rc;
  NW_HIP(nw::launch_vote_finalize(n, d_pre, d_sst, status, s), "k_vote_finalize");
  return 0;
}

int check_committee(const nw_committee* com) {
  if (!com || (com->nauth && (!com->pks || !com->stakes || !com->worker_offsets)))
    return set_err(NW_E_INVALID_ARG, "committee: null pointer");
  for (size_t a = 1; a < com->nauth; ++a)
    if (memcmp(com->pks + 32 * (a - 1), com->pks + 32 * a, 32) >= 0)
      return set_err(NW_E_INVALID_ARG, "committee keys must be strictly increasing");
  for (size_t a = 0; a < com->nauth; ++a)
    if (com->worker_offsets[a + 1] < com->worker_offsets[a])
      return set_err(NW_E_INVALID_ARG, "committee worker_offsets not monotone");
  if (com->nauth && com->worker_offsets[com->nauth] && !com->worker_ids)
    return set_err(NW_E_INVALID_ARG, "committee: null worker_ids");
  return 0;
}

int check_certificates(const nw_certificates* cs, int headers_only, size_t* nvotes) {
  *nvotes = 0;
  if (!cs) return set_err(NW_E_INVALID_ARG, "null pointer");
  const size_t n = cs->n;
  if (n == 0) return 0;
  if (!cs->header_bytes || !cs->header_offsets || !cs->payload_counts || !cs->ids ||
      !cs->header_sigs)
    return set_err(NW_E_INVALID_ARG, "certificates: null pointer");
  for (size_t i = 0; i < n; ++i) {
    if (cs->header_offsets[i + 1] < cs->header_offsets[i])
      return set_err(NW_E_INVALID_ARG, "header_offsets not monotone");
    const uint64_t len = cs->header_offsets[i + 1] - cs->header_offsets[i];
    const uint64_t fixed = 40 + 36 * (uint64_t)cs->payload_counts[i];
    if (len < fixed || (len - fixed) % 32 != 0)
      return set_err(NW_E_INVALID_ARG, "header bytes do not match payload_counts");
  }
  if (headers_only) return 0;
  if (!cs->vote_offsets) return set_err(NW_E_INVALID_ARG, "vote_offsets is NULL");
  if (cs->vote_offsets[0] != 0) return set_err(NW_E_INVALID_ARG, "vote_offsets[0] must be 0");
  for (size_t i = 0; i < n; ++i)
    if (cs->vote_offsets[i + 1] < cs->vote_offsets[i])
      return set_err(NW_E_INVALID_ARG, "vote_offsets not monotone");
  *nvotes = cs->vote_offsets[n];
  if (*nvotes && (!cs->vote_pks || !cs->vote_sigs))
    return set_err(NW_E_INVALID_ARG, "votes: null pointer");
  return 0;
}

}  // namespace rt
}  // namespace nw

extern "C" {

size_t nw_dev_certificates_workspace(size_t n, size_t nvotes) {
  return cert_ws_layout(n, nvotes, nullptr, nullptr);
}

int nw_dev_certificates_verify_many(const nw_committee* committee, const nw_certificates* certs,
                                    int headers_only, const void* z16, const uint8_t* zkey32,
                                    void* workspace, int32_t* status_out, uint64_t* index_out,
                                    void* stream) {
  DevCtx* c;
  int rc = begin(&c);
  if (rc) return rc;
  if (!committee || !certs || !workspace || !status_out)
    return set_err(NW_E_INVALID_ARG, "null pointer");
  if (certs->n == 0) return 0;
  hipStream_t s = pick_stream(stream, c);
  std::vector<uint64_t> tmp;
  const uint64_t* hvo = nullptr;
  if (!headers_only) {
    rc = host_offsets_of(certs->vote_offsets, certs->host_vote_offsets, certs->n, s, tmp, &hvo);
    if (rc) return rc;
    if (hvo[0] != 0 || hvo[certs->n] != certs->nvotes)
      return set_err(NW_E_INVALID_ARG, "vote_offsets must run from 0 to nvotes");
  }
  return nw::rt::cert_pipeline(t_state.device, *committee, *certs, hvo, headers_only, z16, zkey32,
                               workspace, status_out, index_out, s);
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// Internal runtime helpers for nw_jobs.cpp (nw_runtime.h).
// ------------------------------------------------------------------------------------
namespace nw {
namespace rt {

int ensure_init() { return ::ensure_init(); }

int select_device(int* dev_index) {
  int rc = ::ensure_init();
  if (rc) return rc;
  const int dev = t_state.device;
  if (dev < 0 || dev >= g_ndev) return ::set_err(NW_E_INVALID_ARG, "bad device index");
  rc = ::activate(dev);
  if (rc) return rc;
  *dev_index = dev;
  return 0;
}

int use_device(int dev_index) {
  int rc = ::ensure_init();
  if (rc) return rc;
  if (dev_index < 0 || dev_index >= g_ndev) return ::set_err(NW_E_INVALID_ARG, "bad device index");
  return ::activate(dev_index);
}

int thread_device() { return t_state.device; }

void set_thread_device(int dev_index) { t_state.device = dev_index; }

int device_count() { return g_init_status > 0 ? g_ndev : 0; }

std::vector<int> fanout_devices() {
  std::vector<int> out;
  if (t_state.device != NW_ALL_DEVICES || ::ensure_init()) return out;
  // NW_FANOUT_PARTS=k (test hook): k parts dealt round-robin over the devices, so the
  // split/merge logic runs on a one-GPU machine too
  int parts = g_ndev;
  if (const char* e = getenv("NW_FANOUT_PARTS")) {
    const int k = atoi(e);
    if (k > 0 && k <= 64) parts = k;
  }
  for (int p = 0; p < parts; ++p) out.push_back(p % g_ndev);
  return out;
}

int set_err(int code, const char* what, hipError_t e) { return ::set_err(code, what, e); }

int os_random(void* buf, size_t n) { return ::os_random(buf, n); }

int Lease::acquire(int dev_index, hipStream_t stream) {
  if (held_) return ::set_err(NW_E_INVALID_ARG, "lease already held");
  if (dev_index < 0 || dev_index >= kMaxDevices) return ::set_err(NW_E_INVALID_ARG, "bad device");
  // The event chain cannot be captured into a hipGraph (a replay would skip the lease and
  // race other callers on the shared buffers): refuse, before taking the lock.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
    return ::set_err(NW_E_INVALID_ARG, "strict / Header / Vote / Certificate launches use the "
                                       "device's shared tables and cannot be graph-captured");
  SharedDev& d = g_shared[dev_index];
  d.m.lock();
  dev_ = dev_index;
  stream_ = stream;
  held_ = true;
  hipError_t e = hipSuccess;
  if (!d.last) e = hipEventCreateWithFlags(&d.last, hipEventDisableTiming);
  if (e == hipSuccess && d.last_valid) e = hipStreamWaitEvent(stream, d.last, 0);
  // and after every small job queued since (they read the tables this holder may rewrite);
  // a wait binds to the event's current record, so the events can be recycled at once
  for (size_t i = 0; e == hipSuccess && i < d.readers.size(); ++i)
    e = hipStreamWaitEvent(stream, d.readers[i], 0);
  if (e != hipSuccess) {
    held_ = false;
    d.m.unlock();
    return ::set_err(NW_E_DEVICE, "lease: event chain", e);
  }
  d.rpool.insert(d.rpool.end(), d.readers.begin(), d.readers.end());
  d.readers.clear();
  return 0;
}

int ReadLease::acquire(int dev_index, hipStream_t stream, const uint8_t* pks, size_t nkeys,
                       const void** tabs, const uint32_t** ok, nw::keyspec* ks) {
  if (held_) return ::set_err(NW_E_INVALID_ARG, "read lease already held");
  if (dev_index < 0 || dev_index >= kMaxDevices) return ::set_err(NW_E_INVALID_ARG, "bad device");
  SharedDev& d = g_shared[dev_index];
  d.m.lock();
  if (!pks || !nkeys || d.ksaved_n != nkeys || !d.ktabs || d.khost.size() != 32 * nkeys ||
      memcmp(d.khost.data(), pks, 32 * nkeys) != 0) {
    d.m.unlock();
    return 1;
  }
  hipError_t e = hipSuccess;
  if (d.last_valid) e = hipStreamWaitEvent(stream, d.last, 0);
  if (e != hipSuccess) {
    d.m.unlock();
    return ::set_err(NW_E_DEVICE, "read lease: event chain", e);
  }
  dev_ = dev_index;
  stream_ = stream;
  held_ = true;
  if (d.kW > 16 && d.stabs && d.shost.size() == 32 * nkeys &&
      memcmp(d.shost.data(), pks, 32 * nkeys) == 0) {   // Lease::small_tables
    *tabs = d.stabs;
    *ok = d.sok;
    *ks = nw::keyspec_for(16);
    return 0;
  }
  *tabs = d.ktabs;
  *ok = d.kok;
  *ks = nw::keyspec_for(d.kW);
  return 0;
}

int ReadLease::release() {
  if (!held_) return 0;
  SharedDev& d = g_shared[dev_];
  hipEvent_t ev = nullptr;
  hipError_t e = hipSuccess;
  if (!d.rpool.empty()) {
    ev = d.rpool.back();
    d.rpool.pop_back();
  } else {
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventRecord(ev, stream_);
  if (e == hipSuccess) {
    d.readers.push_back(ev);
    if (d.readers.size() > 32) {   // keep the list short: drop readers that have finished
      size_t keep = 0;
      for (hipEvent_t r : d.readers) {
        if (hipEventQuery(r) == hipErrorNotReady) d.readers[keep++] = r;
        else d.rpool.push_back(r);
      }
      d.readers.resize(keep);
    }
  } else if (ev) {
    d.rpool.push_back(ev);
  }
  held_ = false;
  d.m.unlock();
  // without its event a later Lease could overwrite the tables under the launch: wait
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(stream_);
    return ::set_err(NW_E_DEVICE, "read lease: hipEventRecord", e);
  }
  return 0;
}

int Lease::strict_ws(void** out) {
  SharedDev& d = g_shared[dev_];
  if (!d.strict_ws) {
    hipError_t e = nw::table_malloc(&d.strict_ws, nw::strict_workspace_bytes());
    if (e != hipSuccess) {
      d.strict_ws = nullptr;
      return ::set_err(NW_E_OUT_OF_MEMORY, "hipMalloc (strict workspace)", e);
    }
  }
  *out = d.strict_ws;
  return 0;
}

// Comb width of a committee's key tables: 20 bits (13 tables, 940 MB per key: three fewer
// additions per keyed check) up to kKeyW20Keys keys, 16 bits (16 tables, 67 MB per key)
// above. Measured (config 2, alternating runs): N = 4 / 10 +7 / +9 % (profiles/r05kw),
// N = 50 +6 % over 16-bit once its votes are sorted by key (r05kw2; unsorted it lost 18 %,
// r05k20), the service at N = 50 unchanged (r05svc20); N = 100 (94 GB of tables, ~1 s to
// rebuild when the committee changes) stays at 16 bits. NW_KEY_WIDTH = 16 / 20 / 24 forces
// one width.
constexpr size_t kKeyW20Keys = 64;
static uint32_t key_width(size_t nkeys) {
  static const uint32_t forced = [] {
    const char* e = getenv("NW_KEY_WIDTH");
    const uint32_t w = e ? (uint32_t)atoi(e) : 0u;
    return (w == 16 || w == 20 || w == 24) ? w : 0u;
  }();
  if (forced) return forced;
  return nkeys <= kKeyW20Keys ? 20u : 16u;
}

// Frees the device's key tables (every earlier user is ordered before d.last).
static void free_key_tables(SharedDev& d) {
  if (d.last_valid) (void)hipEventSynchronize(d.last);
  if (d.ktabs) (void)hipFree(d.ktabs);
  if (d.kok) (void)hipFree(d.kok);
  if (d.ksaved) (void)hipFree(d.ksaved);
  if (d.kflag) (void)hipFree(d.kflag);
  d.ktabs = nullptr;
  d.kok = d.ksaved = d.kflag = nullptr;
  d.kcap = d.ksaved_n = 0;
  d.kW = 0;
  d.khost.clear();
  d.shost.clear();   // the small-job set describes no committee until rebuilt
}

// Key tables of width W for nkeys keys (room for 16 keys at 16 bits, 1 GB; for the committee
// itself at wider combs). NW_KEYTAB_LIMIT=bytes (test hook) fails a key-table allocation above
// it, as a device shared with other ranks or tenants would.
static hipError_t alloc_key_tables(SharedDev& d, size_t nkeys, uint32_t W) {
  const size_t cap = W == 16 ? (nkeys < 16 ? 16 : nkeys) : nkeys;
  const size_t bytes = nw::key_tables_bytes(cap, nw::keyspec_for(W));
  static const unsigned long long limit = [] {
    const char* e = getenv("NW_KEYTAB_LIMIT");
    return e ? strtoull(e, nullptr, 10) : 0ull;
  }();
  hipError_t e = limit && bytes > limit ? hipErrorOutOfMemory
                                        : nw::table_malloc(&d.ktabs, bytes);
  static const bool klog = getenv("NW_KEYTAB_LOG") != nullptr;   // diagnostics
  if (klog) {
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    fprintf(stderr, "[keytab] keys %zu width %u bytes %zu -> %s (free %zu of %zu)\n", nkeys, W,
            bytes, e == hipSuccess ? "ok" : "FAILED", fr, tot);
  }
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d.kok), 4 * cap);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d.ksaved), 32 * cap);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d.kflag), 4);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    free_key_tables(d);
    return e;
  }
  d.kcap = cap;
  d.kW = W;
  return hipSuccess;
}

int Lease::key_tables(size_t nkeys, void** tabs, uint32_t** ok, nw::keyspec* ks,
                      uint32_t** saved, uint32_t** flag, bool* force) {
  SharedDev& d = g_shared[dev_];
  const uint32_t W = key_width(nkeys);
  // Tables that hold nkeys keys are kept when they have the preferred width, or when they are
  // 16-bit tables and the preferred width is wider (a device alternating between committees of
  // 50 and 100 keys keeps its 16-bit tables instead of reallocating 47-94 GB per switch; the
  // keys themselves are rebuilt in place, k_key_cmp).
  const bool usable = d.ktabs && nkeys <= d.kcap && (d.kW == W || (d.kW == 16 && W > 16));
  if (!usable) {
    free_key_tables(d);
    hipError_t e = alloc_key_tables(d, nkeys, W);
    // no room at the wider comb: 16 bits (67 MB per key) still run the keyed checks, several
    // times faster than the unkeyed fallback the caller takes on NW_E_OUT_OF_MEMORY
    if (e == hipErrorOutOfMemory && W != 16) e = alloc_key_tables(d, nkeys, 16);
    if (e != hipSuccess) return ::set_err(NW_E_OUT_OF_MEMORY, "hipMalloc (key tables)", e);
  }
  *tabs = d.ktabs;
  *ok = d.kok;
  *ks = nw::keyspec_for(d.kW);
  if (saved) *saved = d.ksaved;
  if (flag) *flag = d.kflag;
  if (force) *force = d.ksaved_n != nkeys;
  d.ksaved_n = 0;   // until keys_built: a failed launch leaves no tables to keep
  d.khost.clear();
  return 0;
}

int Lease::small_tables(const uint32_t* dpks, size_t nkeys, const uint8_t* host_pks) {
  static const bool on = [] {
    const char* e = getenv("NW_SMALL_KEYW16");
    return !(e && *e == '0');
  }();
  SharedDev& d = g_shared[dev_];
  if (!on || d.kW <= 16 || !host_pks || !nkeys || d.ksaved_n != nkeys) return 0;
  if (d.shost.size() == 32 * nkeys && memcmp(d.shost.data(), host_pks, 32 * nkeys) == 0)
    return 0;   // built for this committee (every earlier reader is ordered before us)
  d.shost.clear();
  const nw::keyspec ks = nw::keyspec_for(16);
  if (nkeys > d.scap) {
    if (d.stabs) (void)hipFree(d.stabs);
    if (d.sok) (void)hipFree(d.sok);
    d.stabs = nullptr;
    d.sok = nullptr;
    d.scap = 0;
    hipError_t e = nw::table_malloc(&d.stabs, nw::key_tables_bytes(nkeys, ks));
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d.sok), 4 * nkeys);
    if (e != hipSuccess) {   // no room: small jobs keep reading the wide tables
      (void)hipGetLastError();
      if (d.stabs) (void)hipFree(d.stabs);
      if (d.sok) (void)hipFree(d.sok);
      d.stabs = nullptr;
      d.sok = nullptr;
      return 0;
    }
    d.scap = nkeys;
  }
  const hipError_t e = nw::launch_key_tables(dpks, nkeys, ks,
                                             static_cast<nw::ge_niels_pad*>(d.stabs), d.sok,
                                             stream_, nullptr, nullptr, true);
  if (e != hipSuccess) return ::set_err(NW_E_DEVICE, "k_key_tables (16-bit, small jobs)", e);
  d.shost.assign(host_pks, host_pks + 32 * nkeys);
  return 0;
}

void Lease::keys_built(size_t nkeys, const uint8_t* host_pks) {
  SharedDev& d = g_shared[dev_];
  d.ksaved_n = nkeys;
  if (host_pks) d.khost.assign(host_pks, host_pks + 32 * nkeys);
  else d.khost.clear();
}

int Lease::release() {
  if (!held_) return 0;
  SharedDev& d = g_shared[dev_];
  hipError_t e = hipEventRecord(d.last, stream_);
  d.last_valid = d.last_valid || e == hipSuccess;
  held_ = false;
  d.m.unlock();
  return e == hipSuccess ? 0 : ::set_err(NW_E_DEVICE, "lease: hipEventRecord", e);
}

}  // namespace rt
}  // namespace nw
