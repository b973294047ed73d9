// nw_jobs.cpp — asynchronous host-buffer entry points (nw_submit_* / nw_job_*), and the
// blocking host-buffer calls built on them.
//
// A job owns a HIP stream, a completion event, a pinned host staging buffer and a device
// buffer, all grow-only and recycled through a per-device pool, so the steady state does
// no allocation. Submit copies the caller's inputs into the pinned buffer (the caller may
// reuse its input memory as soon as submit returns), queues one H2D copy, the kernels and
// one D2H copy of the outputs on the job's stream, records the event and returns. Poll /
// wait deliver the outputs from pinned memory into the caller's output buffers. This is
// the shape the reference's async callers need: Narwhal's primary and workers run on
// tokio (node/Cargo.toml:8), and Core / Processor loops must not block on the device
// (crypto/src/lib.rs:222-250 SignatureService is the reference's own async-service pattern).
//
// Strict verification uses the device's shared table workspace (nw::rt::Lease): launches
// from different jobs and streams are ordered on it with an event chain (the copies of one
// job still overlap the kernels of another).
//
// Fan-out (nw_set_device(NW_ALL_DEVICES)): a submit splits its items into contiguous parts,
// one per device (strict: 64-item aligned so bitmap bytes concatenate; verify_batch: whole
// batches, about equal votes per part; SHA-512: whole messages, about equal bytes), submits
// each part as an ordinary job on its device and returns a parent job over them; poll /
// wait / notify / release act on every part, and each part delivers straight into its slice
// of the caller's outputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <new>
#include <vector>

#include "narwhal_amd.h"
#include "nw_kernels.h"
#include "nw_runtime.h"

struct nw_job {
  int dev = -1;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  char* hbuf = nullptr;   // pinned: inputs, then outputs
  size_t hcap = 0;
  char* dbuf = nullptr;   // device: same layout (+ workspace)
  size_t dcap = 0;
  char* hdev = nullptr;   // the device's address of hbuf (small jobs read it directly)
  char* vbuf = nullptr;   // NW_SMALL_VRAM: fine-grained device memory for small jobs' inputs
  char* vhost = nullptr;  // ... and the host's mapping of it (the CPU writes the inputs there)
  size_t vcap = 0;
  uint32_t vseq = 0;      // NW_BATCH_GATE: the last input-gate sequence number
  // NW_BATCH_SPIN: the fused tail's done word in the pinned buffer (host view) and the value
  // it will hold; `early`: outputs delivered from it while the launch may still be counting
  // out (the job is synchronised before its next use, job_acquire)
  volatile uint32_t* spin = nullptr;
  uint32_t spin_seq = 0;
  bool early = false;
  // small jobs (NW_SMALL_DONE): one done flag per workgroup in the pinned buffer (host view)
  volatile uint32_t* small_flags = nullptr;
  uint32_t small_nwg = 0;
  uint32_t* dcnt = nullptr;   // small jobs' per-message arrival counters (kept zero)
  size_t ccap = 0;
  uint32_t* dfz = nullptr;    // config-1 fused launches' counters (the tail leaves them zero)
  bool dfz_dirty = false;     // a launch failed after the head ran: clear before reuse
  struct Out {
    void* dst;
    size_t off;
    size_t bytes;
  } outs[3];
  int nouts = 0;
  bool pending = false;   // device work queued, outputs not yet delivered
  std::vector<nw_job*> parts;   // fan-out parent (dev = -1): one ordinary job per part
  nw::rt::Fork fork{nullptr, nullptr, nullptr};   // certificate jobs: header checks' stream
};

namespace {

using nw::rt::set_err;

constexpr int kMaxDev = 64;

struct DevPool {
  std::mutex m;
  std::vector<nw_job*> free;
  // jobs released early (outputs delivered from done words / flags) whose launch may still be
  // finishing: they rejoin `free` once their completion event has fired, so a submit never
  // blocks on a launch that is counting out while an idle job exists
  std::vector<nw_job*> retiring;
};
DevPool g_pool[kMaxDev];

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

#define JOB_HIP(call, what)                                      \
  do {                                                           \
    hipError_t e_ = (call);                                      \
    if (e_ != hipSuccess) return set_err(NW_E_DEVICE, what, e_); \
  } while (0)

int job_acquire(int dev, nw_job** out) {
  int rc = nw::rt::use_device(dev);
  if (rc) return rc;
  DevPool& p = g_pool[dev];
  nw_job* j = nullptr;
  {
    std::lock_guard<std::mutex> g(p.m);
    if (!p.retiring.empty()) {   // finished early releases rejoin the free list
      size_t keep = 0;
      for (nw_job* x : p.retiring) {
        const hipError_t e = hipEventQuery(x->done);
        if (e == hipErrorNotReady) {
          p.retiring[keep++] = x;
          continue;
        }
        if (e != hipSuccess && x->dfz) x->dfz_dirty = true;
        x->pending = false;
        x->early = false;
        p.free.push_back(x);
      }
      p.retiring.resize(keep);
    }
    if (!p.free.empty()) {
      j = p.free.back();
      p.free.pop_back();
    } else if (!p.retiring.empty()) {   // none idle: the oldest early release (nearly done)
      j = p.retiring.front();
      p.retiring.erase(p.retiring.begin());
    }
  }
  if (!j) {
    j = new (std::nothrow) nw_job;
    if (!j) return set_err(NW_E_OUT_OF_MEMORY, "job allocation");
    j->dev = dev;
    hipError_t e = hipStreamCreateWithFlags(&j->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&j->done, hipEventDisableTiming);
    if (e != hipSuccess) {
      if (j->stream) (void)hipStreamDestroy(j->stream);
      delete j;
      return set_err(NW_E_DEVICE, "job stream/event", e);
    }
  }
  if (j->pending) {   // released early (NW_BATCH_SPIN): its launch may still be finishing
    if (hipEventSynchronize(j->done) != hipSuccess && j->dfz) j->dfz_dirty = true;
  }
  j->nouts = 0;
  j->pending = false;
  j->early = false;
  j->spin = nullptr;
  j->small_flags = nullptr;
  *out = j;
  return 0;
}

void job_recycle(nw_job* j) {
  if (!j) return;
  if (!j->parts.empty() || j->dev < 0) {   // fan-out parent: recycle the parts
    for (nw_job* x : j->parts) job_recycle(x);
    delete j;
    return;
  }
  if (j->pending && !j->early) (void)hipEventSynchronize(j->done);
  if (!j->early) j->pending = false;   // an early job syncs on its next acquire
  j->nouts = 0;
  j->spin = nullptr;
  j->small_flags = nullptr;
  std::lock_guard<std::mutex> g(g_pool[j->dev].m);
  if (j->early && j->pending) g_pool[j->dev].retiring.push_back(j);
  else g_pool[j->dev].free.push_back(j);
}

// Fail a submit after work may have been queued: drain the stream, recycle, report.
int job_abort(nw_job* j, int rc) {
  (void)hipStreamSynchronize(j->stream);
  j->pending = false;
  j->early = false;
  // a fused config-1 launch may have queued: its counters are no longer known to be zero
  if (j->dfz) j->dfz_dirty = true;
  job_recycle(j);
  return rc;
}

int job_counters(nw_job* j, size_t n);

// Growth log (nw::rt::job_growth_log): a staging buffer that grows inside a burst pins or
// allocates memory on the submitting thread, which the service's debug timeline must show.
struct GrowEv {
  uint64_t t_ns, cap, us, kind;
};
constexpr size_t kGrowLog = 4096;
GrowEv g_grow[kGrowLog];
std::atomic<size_t> g_ngrow{0};
void log_growth(uint64_t kind, size_t cap, std::chrono::steady_clock::time_point t0) {
  const auto t1 = std::chrono::steady_clock::now();
  const size_t i = g_ngrow.fetch_add(1, std::memory_order_relaxed);
  if (i < kGrowLog)
    g_grow[i] = {(uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                     t0.time_since_epoch()).count(),
                 cap, (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0)
                          .count(), kind};
}

int job_reserve(nw_job* j, size_t hbytes, size_t dbytes) {
  if (hbytes > j->hcap) {
    const auto t0 = std::chrono::steady_clock::now();
    if (j->hbuf) (void)hipHostFree(j->hbuf);
    j->hbuf = nullptr;
    j->hcap = 0;
    const size_t cap = hbytes < (1u << 20) ? (1u << 20) : hbytes + hbytes / 4;
    // coherent (fine-grained): small jobs' kernels read their inputs from it and write their
    // outputs into it directly, and a recycled buffer must never be served from a GPU cache
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&j->hbuf), cap,
                                 hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return set_err(NW_E_OUT_OF_MEMORY, "hipHostMalloc (job staging)", e);
    j->hcap = cap;
    void* dp = nullptr;
    e = hipHostGetDevicePointer(&dp, j->hbuf, 0);
    if (e != hipSuccess) return set_err(NW_E_DEVICE, "hipHostGetDevicePointer (job staging)", e);
    j->hdev = static_cast<char*>(dp);
    log_growth(0, cap, t0);
  }
  if (dbytes > j->dcap) {
    const auto t0 = std::chrono::steady_clock::now();
    if (j->dbuf) (void)hipFree(j->dbuf);
    j->dbuf = nullptr;
    j->dcap = 0;
    const size_t cap = dbytes < (1u << 20) ? (1u << 20) : dbytes + dbytes / 4;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&j->dbuf), cap);
    if (e != hipSuccess) return set_err(NW_E_OUT_OF_MEMORY, "hipMalloc (job buffer)", e);
    j->dcap = cap;
    log_growth(1, cap, t0);
  }
  return 0;
}

// NW_SMALL_VRAM=1 (A/B hook, read once): a small job's inputs travel as the CPU's writes into
// fine-grained device memory mapped through the BAR, so its kernel reads device memory only
// (the episodes in which the device's reads of pinned host memory stall).
// Outputs stay in the pinned buffer. Falls back to the pinned inputs when the device memory
// has no host mapping.
bool small_vram() {
  static const bool on = [] {
    const char* e = getenv("NW_SMALL_VRAM");
    return e && *e == '1';
  }();
  return on;
}
bool test_fuse_abort() {
  static std::atomic<long> left{[] {
    const char* e = getenv("NW_TEST_FUSE_ABORT");
    return e && *e ? atol(e) : 0L;
  }()};
  if (left.load(std::memory_order_relaxed) <= 0) return false;
  return left.fetch_sub(1, std::memory_order_relaxed) > 0;
}
bool test_stale_flags() {
  static const bool on = [] {
    const char* e = getenv("NW_TEST_STALE_FLAGS");
    const bool v = e && *e == '1';
    if (v) fprintf(stderr, "[narwhal_amd] NW_TEST_STALE_FLAGS: small-job flag words poisoned\n");
    return v;
  }();
  return on;
}
// Sequence numbers of done words / flags: unique across every job of the process (a job's own
// counter would repeat values another job's stale flags still hold), never 0.
uint32_t next_done_seq() {
  static std::atomic<uint32_t> seq{0};
  uint32_t v = seq.fetch_add(1, std::memory_order_relaxed) + 1;
  if (v == 0) v = seq.fetch_add(1, std::memory_order_relaxed) + 1;
  return v;
}
bool small_done() {   // on unless NW_SMALL_DONE=0
  static const bool on = [] {
    const char* e = getenv("NW_SMALL_DONE");
    return !(e && *e == '0');
  }();
  return on;
}
// Outputs delivered from a job whose kernels have written them (done word / flags) while the
// launch may still be finishing: the job stays pending and is synchronised on its next
// acquire (job_acquire), not at release.
void job_deliver_early(nw_job* j) {
  std::atomic_thread_fence(std::memory_order_acquire);
  for (int i = 0; i < j->nouts; ++i)
    memcpy(j->outs[i].dst, j->hbuf + j->outs[i].off, j->outs[i].bytes);
  j->nouts = 0;
  j->early = true;
  j->spin = nullptr;
  j->small_flags = nullptr;
}
bool small_flags_done(const nw_job* j) {
  for (uint32_t w = 0; w < j->small_nwg; ++w)
    if (j->small_flags[w] != j->spin_seq) return false;
  return true;
}
bool batch_spin() {   // on unless NW_BATCH_SPIN=0 (profiles/r06n: wait 258 vs 264 us)
  static const bool on = [] {
    const char* e = getenv("NW_BATCH_SPIN");
    return !(e && *e == '0');
  }();
  return on;
}
bool batch_stamps() {
  static const bool on = [] {
    const char* e = getenv("NW_BATCH_STAMPS");
    return e && *e == '1';
  }();
  return on;
}
// votes per input-gate flag, a multiple of 64 (NW_GATE_CHUNK=k, A/B hook, rounded up to 64)
const uint64_t kGateChunk = [] {
  const char* e = getenv("NW_GATE_CHUNK");
  const long v = e && *e ? atol(e) : 1024L;
  return (uint64_t)(v < 64 ? 64 : (v + 63) / 64 * 64);
}();
bool batch_gate() {
  static const bool on = [] {
    const char* e = getenv("NW_BATCH_GATE");
    return e && *e == '1';
  }();
  return on;
}
bool batch_vram() {   // on unless NW_BATCH_VRAM=0 (profiles/r06d: config 1 0.303 vs 0.321 ms)
  static const bool on = [] {
    const char* e = getenv("NW_BATCH_VRAM");
    return !(e && *e == '0');
  }();
  return on;
}
bool mapped_rw(const void* p, size_t bytes) {
  // one whole /proc/self/maps line per read (getline: no line is split, however long its
  // path), and only a writable shared mapping of a GPU device node counts
  FILE* f = fopen("/proc/self/maps", "r");
  if (!f) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  char* line = nullptr;
  size_t cap = 0;
  bool ok = false;
  while (!ok && getline(&line, &cap, f) > 0) {
    unsigned long lo = 0, hi = 0;
    char perm[5] = {0};
    if (sscanf(line, "%lx-%lx %4s", &lo, &hi, perm) == 3 && a >= lo && a + bytes <= hi)
      ok = perm[0] == 'r' && perm[1] == 'w' && perm[3] == 's' &&
           (strstr(line, "/dev/dri/") != nullptr || strstr(line, "/dev/kfd") != nullptr);
  }
  free(line);
  fclose(f);
  return ok;
}
int job_reserve_vram(nw_job* j, size_t bytes) {
  if (bytes <= j->vcap) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  if (j->vbuf) (void)hipFree(j->vbuf);
  j->vbuf = j->vhost = nullptr;
  j->vcap = 0;
  const size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, cap, hipDeviceMallocFinegrained);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  hipPointerAttribute_t at{};
  e = hipPointerGetAttributes(&at, p);
  void* hp = e == hipSuccess ? at.hostPointer : nullptr;
  // The runtime reports no host pointer for fine-grained device memory, but on this
  // platform the device address itself is mapped into the process (a shared mapping of the
  // render node, tools/ubench/bar_probe.hip): use it when /proc/self/maps shows the whole
  // buffer mapped writable.
  if (!hp && mapped_rw(p, cap)) hp = p;
  if (!hp) {
    (void)hipGetLastError();
    (void)hipFree(p);
    return 1;
  }
  j->vbuf = static_cast<char*>(p);
  j->vhost = static_cast<char*>(hp);
  j->vcap = cap;
  memset(j->vhost, 0, cap);   // input-gate flags start below every sequence number
  std::atomic_thread_fence(std::memory_order_seq_cst);
  j->vseq = 0;

  log_growth(3, cap, t0);
  return 0;
}

void job_out(nw_job* j, void* dst, size_t off, size_t bytes) {
  if (dst && bytes) j->outs[j->nouts++] = {dst, off, bytes};
}

void job_deliver(nw_job* j) {
  for (int i = 0; i < j->nouts; ++i) memcpy(j->outs[i].dst, j->hbuf + j->outs[i].off, j->outs[i].bytes);
  j->nouts = 0;
  j->pending = false;
}

// Queue: H2D of [0, in_bytes), `launch`, D2H of [out_off, out_off + out_bytes), event.
template <class Launch>
int job_run(nw_job* j, size_t in_bytes, size_t out_off, size_t out_bytes, Launch launch) {
  if (in_bytes)
    JOB_HIP(hipMemcpyAsync(j->dbuf, j->hbuf, in_bytes, hipMemcpyHostToDevice, j->stream),
            "H2D (job inputs)");
  int rc = launch();
  if (rc) return rc;
  if (out_bytes)
    JOB_HIP(hipMemcpyAsync(j->hbuf + out_off, j->dbuf + out_off, out_bytes,
                           hipMemcpyDeviceToHost, j->stream),
            "D2H (job outputs)");
  JOB_HIP(hipEventRecord(j->done, j->stream), "hipEventRecord");
  j->pending = true;
  return 0;
}

// The job's second stream and two events (created once per pooled job); without them the
// callers run their sequential form.
void ensure_fork(nw_job* j) {
  if (j->fork.s2) return;
  hipStream_t s2 = nullptr;
  hipEvent_t e1 = nullptr, e2 = nullptr;
  if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) == hipSuccess &&
      hipEventCreateWithFlags(&e1, hipEventDisableTiming) == hipSuccess &&
      hipEventCreateWithFlags(&e2, hipEventDisableTiming) == hipSuccess) {
    j->fork = nw::rt::Fork{s2, e1, e2};
  } else {
    if (e1) (void)hipEventDestroy(e1);
    if (s2) (void)hipStreamDestroy(s2);
  }
}

}  // namespace

size_t nw::rt::job_growth_log(uint64_t* out, size_t max) {
  const size_t n = std::min(g_ngrow.load(std::memory_order_acquire), kGrowLog);
  for (size_t i = 0; i < n && i < max; ++i) {
    out[4 * i] = g_grow[i].t_ns;
    out[4 * i + 1] = g_grow[i].cap;
    out[4 * i + 2] = g_grow[i].us;
    out[4 * i + 3] = g_grow[i].kind;
  }
  return n;
}

// Puts `count` jobs with their streams, fork streams and `hbytes` / `dbytes` of staging into
// device dev's pool (nw_service_create: a service's first burst then finds its jobs made,
// instead of creating streams and pinning memory on the flusher's path).
int nw::rt::jobs_prewarm(int dev, int count, size_t hbytes, size_t dbytes) {
  std::vector<nw_job*> got;
  int rc = 0;
  for (int i = 0; i < count && !rc; ++i) {
    nw_job* j = nullptr;
    rc = job_acquire(dev, &j);
    if (rc) break;
    got.push_back(j);
    rc = job_reserve(j, hbytes, dbytes);
    // small jobs' arrival counters too: a first small job on a job without them would
    // allocate (hipMalloc + hipMemsetAsync) on the submitting thread in the middle of a burst
    if (!rc) rc = job_counters(j, 4096);
    if (!rc && small_vram()) (void)job_reserve_vram(j, hbytes);
    if (!rc) ensure_fork(j);
  }
  for (nw_job* j : got) job_recycle(j);
  return rc;
}

namespace {

int fill_key(nw::z_key_t& k) {
  int rc = nw::rt::os_random(k.key, 32);
  k.nonce = 0;
  return rc;
}

// ---- one device --------------------------------------------------------------------
int submit_strict(int dev, const uint8_t* digests, size_t digest_stride, const uint8_t* pks,
                  const uint8_t* sigs, size_t n, int32_t* status_out, uint8_t* bitmap_out,
                  nw_job** job) {
  nw_job* j;
  int rc = job_acquire(dev, &j);
  if (rc) return rc;
  if (n == 0) {
    *job = j;
    return 0;
  }
  const size_t nmsg = digest_stride ? n : 1;
  const size_t o_m = 0, o_pk = o_m + a256(32 * nmsg), o_sig = o_pk + a256(32 * n),
               o_st = o_sig + a256(64 * n), o_bm = o_st + a256(4 * n),
               end = o_bm + a256(8 * ((n + 63) / 64));
  rc = job_reserve(j, end, end);
  if (rc) return job_abort(j, rc);
  memcpy(j->hbuf + o_m, digests, 32 * nmsg);
  memcpy(j->hbuf + o_pk, pks, 32 * n);
  memcpy(j->hbuf + o_sig, sigs, 64 * n);
  rc = job_run(j, o_st, o_st, end - o_st, [&]() -> int {
    // the device's shared strict workspace, ordered after its previous user (nw_runtime.h)
    nw::rt::Lease lease;
    void* ws = nullptr;
    int lrc = lease.acquire(j->dev, j->stream);
    if (!lrc) lrc = lease.strict_ws(&ws);
    if (lrc) return lrc;
    JOB_HIP(nw::launch_verify_strict(reinterpret_cast<const uint32_t*>(j->dbuf + o_m),
                                     (uint32_t)(digest_stride / 4),
                                     reinterpret_cast<const uint32_t*>(j->dbuf + o_pk),
                                     reinterpret_cast<const uint32_t*>(j->dbuf + o_sig), n,
                                     reinterpret_cast<int32_t*>(j->dbuf + o_st),
                                     reinterpret_cast<uint64_t*>(j->dbuf + o_bm), ws,
                                     j->stream),
            "k_verify_strict launch");
    return lease.release();
  });
  if (rc) return job_abort(j, rc);
  job_out(j, status_out, o_st, 4 * n);
  job_out(j, bitmap_out, o_bm, (n + 7) / 8);
  *job = j;
  return 0;
}

// offsets: nbatches + 1 host values from 0
int submit_batch(int dev, const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                 const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                 int32_t* status_out, uint64_t* fail_index_out, nw_job** job) {
  const size_t nitems = nbatches ? offsets[nbatches] : 0;
  nw_job* j;
  int rc = job_acquire(dev, &j);
  if (rc) return rc;
  if (nbatches == 0) {
    *job = j;
    return 0;
  }
  const size_t m = nitems ? nitems : 1;
  // a lone batch on the fused path: the launches write the verdict into the pinned buffer
  // (no copy back) and use the job's own counters (zero between calls)
  const bool direct = nw::verify_batch_outputs_direct(nbatches, nitems);
  const size_t o_d = 0, o_off = o_d + a256(32 * nbatches), o_pk = o_off + a256(8 * (nbatches + 1)),
               o_sig = o_pk + a256(32 * m), o_z = o_sig + a256(64 * m),
               o_st = o_z + (z16 ? a256(16 * m) : 0),
               o_fi = o_st + a256(4 * nbatches),
               o_dn = o_fi + a256(8 * nbatches),   // NW_BATCH_SPIN's done word
               o_ws = o_dn + 256,
               end = o_ws + a256(nw::batch_workspace_bytes(nbatches, nitems));
  rc = job_reserve(j, o_ws, end);
  if (rc) return job_abort(j, rc);
  // A lone fused batch's inputs go straight from the caller's buffers into host-mapped
  // fine-grained device memory: no pinned staging copy, no H2D (NW_BATCH_VRAM=0: the pinned
  // buffer and one H2D copy, as before round 6)
  // NW_BATCH_GATE=1 (A/B hook): the kernels are queued first and the votes written after,
  // chunk by chunk, each chunk released by a flag the head's waves wait for (input_gate_t):
  // the launch and the head's first waves overlap the CPU's writes.
  const uint64_t nchunks = (nitems + kGateChunk - 1) / kGateChunk;
  const size_t o_gf = o_st;   // the flags follow the inputs in the device-memory buffer
  const bool vram = direct && batch_vram() &&
                    job_reserve_vram(j, o_st + (batch_gate() ? a256(4 * nchunks) : 0)) == 0;
  const bool gate = vram && batch_gate() && nitems && nw::verify_batch_gate_ok(nbatches, nitems);
  char* const stage = vram ? j->vhost : j->hbuf;
  const auto ts0 = std::chrono::steady_clock::now();   // NW_BATCH_STAMPS (diagnostics)
  memcpy(stage + o_d, digests, 32 * nbatches);
  memcpy(stage + o_off, offsets, 8 * (nbatches + 1));
  if (nitems && !gate) {
    memcpy(stage + o_pk, pks, 32 * nitems);
    memcpy(stage + o_sig, sigs, 64 * nitems);
    if (z16) memcpy(stage + o_z, z16, 16 * nitems);
  }
  if (vram) std::atomic_thread_fence(std::memory_order_seq_cst);   // drain write combining
  const auto ts1 = std::chrono::steady_clock::now();
  uint32_t seq = 0;
  if (gate) {
    seq = ++j->vseq;
    if (seq == 0) seq = j->vseq = 1;   // the flags were zeroed at allocation
    static std::once_flag said;
    std::call_once(said, [] {
      fprintf(stderr, "[narwhal_amd] NW_BATCH_GATE: lone batches launched before their votes "
              "are written (input gate)\n");
    });
  }
  bool launched = false;
  // the votes, chunk by chunk, each followed by its flag (fence between: write-combined
  // stores are not ordered among themselves; PCIe keeps the posted writes in order)
  const auto release_votes = [&]() {
    volatile uint32_t* fl = reinterpret_cast<volatile uint32_t*>(j->vhost + o_gf);
    for (uint64_t c = 0; c < nchunks; ++c) {
      const uint64_t v0 = c * kGateChunk, v = std::min<uint64_t>(kGateChunk, nitems - v0);
      memcpy(stage + o_pk + 32 * v0, pks + 32 * v0, 32 * v);
      memcpy(stage + o_sig + 64 * v0, sigs + 64 * v0, 64 * v);
      if (z16) memcpy(stage + o_z + 16 * v0, z16 + 16 * v0, 16 * v);
      std::atomic_thread_fence(std::memory_order_seq_cst);
      fl[c] = seq;
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);
  };
  nw::z_key_t key;
  rc = fill_key(key);
  if (rc) return job_abort(j, rc);
  const nw::input_gate_t gt{reinterpret_cast<const uint32_t*>(j->vbuf + o_gf), seq,
                            (uint32_t)kGateChunk};
  // (planning reads the offsets on the host: the caller's array, never the mapped copy)
  const uint64_t* h_off = offsets;
  // (The Pippenger digit lanes and sorts on a second stream beside the decompressions
  // measured slower for config 1's one call, 0.405 vs 0.371 ms: the cross-stream event waits
  // cost more than the 25 us sort they hid; the fused head runs them side by side instead.)
  const bool out_direct = direct;
  if (out_direct && (!j->dfz || j->dfz_dirty)) {
    if (!j->dfz &&
        hipMalloc(reinterpret_cast<void**>(&j->dfz), nw::verify_batch_fuse_ctr_bytes()) != hipSuccess) {
      j->dfz = nullptr;
      return job_abort(j, set_err(NW_E_OUT_OF_MEMORY, "hipMalloc (fused counters)"));
    }
    if (hipMemsetAsync(j->dfz, 0, nw::verify_batch_fuse_ctr_bytes(), j->stream) != hipSuccess)
      return job_abort(j, set_err(NW_E_DEVICE, "hipMemsetAsync (fused counters)"));
    j->dfz_dirty = false;
  }
  char* const obuf = out_direct ? j->hdev : j->dbuf;
  char* const ibuf = vram ? j->vbuf : j->dbuf;
  // The tail stores a fresh sequence number into the pinned done word right after the
  // verdict; nw_job_wait spins on it instead of waiting for the launch's completion event
  // (NW_BATCH_SPIN=0: the event only)
  uint32_t* done = nullptr;
  uint32_t dseq = 0;
  if (out_direct && batch_spin()) {
    dseq = next_done_seq();
    volatile uint32_t* dh = reinterpret_cast<volatile uint32_t*>(j->hbuf + o_dn);
    *dh = dseq - 1;   // anything but dseq
    done = reinterpret_cast<uint32_t*>(j->hdev + o_dn);
  }
  rc = job_run(j, vram ? 0 : o_st, o_st, out_direct ? 0 : o_ws - o_st, [&]() -> int {
    // from here on a gated head may be queued (even if a later launch fails): the votes
    // and their flags are written whatever happens, so no wave is left waiting
    launched = gate;
    const hipError_t e = nw::launch_verify_batch(
        reinterpret_cast<const uint32_t*>(ibuf + o_d),
        reinterpret_cast<const uint64_t*>(ibuf + o_off), h_off, nbatches,
        reinterpret_cast<const uint32_t*>(ibuf + o_pk),
        reinterpret_cast<const uint32_t*>(ibuf + o_sig), nitems,
        z16 ? reinterpret_cast<const uint32_t*>(ibuf + o_z) : nullptr, key, j->dbuf + o_ws,
        reinterpret_cast<int32_t*>(obuf + o_st), reinterpret_cast<uint64_t*>(obuf + o_fi),
        j->stream, nullptr, nullptr, 0, 1.0, out_direct ? j->dfz : nullptr,
        gate ? &gt : nullptr, done, dseq);
    if (e != hipSuccess && out_direct) j->dfz_dirty = true;   // the head may have run
    JOB_HIP(e, "verify_batch launch");
    return 0;
  });
  const auto ts2 = std::chrono::steady_clock::now();
  if (launched) release_votes();   // also on failure after the launch: no wave waits 2 s
  if (rc) return job_abort(j, rc);
  if (batch_stamps()) {
    const auto ts3 = std::chrono::steady_clock::now();
    const auto us = [](std::chrono::steady_clock::time_point a,
                       std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::micro>(b - a).count();
    };
    fprintf(stderr, "[narwhal_amd] batch stamps: n=%zu vram=%d gate=%d inputs %.1f us, "
            "launch %.1f us, gated writes %.1f us\n", (size_t)nitems, (int)vram, (int)gate,
            us(ts0, ts1), us(ts1, ts2), us(ts2, ts3));
  }
  if (out_direct && test_fuse_abort()) {
    // test hook (NW_TEST_FUSE_ABORT=k: the first k such calls): a failure after the fused
    // launches were queued, with their counters left non-zero — the job's next call must
    // clear them (dfz_dirty, set by job_abort) instead of spinning on stale tickets
    (void)hipStreamSynchronize(j->stream);
    (void)hipMemsetAsync(j->dfz, 0x01, nw::verify_batch_fuse_ctr_bytes(), j->stream);
    return job_abort(j, set_err(NW_E_DEVICE, "NW_TEST_FUSE_ABORT"));
  }
  job_out(j, status_out, o_st, 4 * nbatches);
  job_out(j, fail_index_out, o_fi, 8 * nbatches);
  if (done) {
    j->spin = reinterpret_cast<volatile uint32_t*>(j->hbuf + o_dn);
    j->spin_seq = dseq;
  }
  *job = j;
  return 0;
}

int submit_sha(int dev, const uint8_t* data, const uint64_t* offsets, const uint64_t* lengths,
               size_t n, uint8_t* out32, nw_job** job) {
  nw_job* j;
  int rc = job_acquire(dev, &j);
  if (rc) return rc;
  if (n == 0) {
    *job = j;
    return 0;
  }
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += lengths[i];
  const size_t o_data = 0, o_off = a256(total ? total : 1), o_len = o_off + a256(8 * n),
               o_out = o_len + a256(8 * n), end = o_out + a256(32 * n);
  rc = job_reserve(j, end, end);
  if (rc) return job_abort(j, rc);
  // Pack the referenced bytes contiguously (messages may live anywhere in `data`);
  // contiguous runs are copied in one go.
  uint64_t* offs = reinterpret_cast<uint64_t*>(j->hbuf + o_off);
  uint64_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    offs[i] = pos;
    pos += lengths[i];
  }
  size_t i = 0;
  while (i < n) {
    size_t k = i + 1;
    while (k < n && offsets[k] == offsets[k - 1] + lengths[k - 1]) ++k;
    const uint64_t bytes = offs[k - 1] + lengths[k - 1] - offs[i];
    if (bytes) memcpy(j->hbuf + o_data + offs[i], data + offsets[i], bytes);
    i = k;
  }
  memcpy(j->hbuf + o_len, lengths, 8 * n);
  rc = job_run(j, o_out, o_out, 32 * n, [&]() -> int {
    JOB_HIP(nw::launch_sha512_digest32(reinterpret_cast<const uint8_t*>(j->dbuf + o_data),
                                       reinterpret_cast<const uint64_t*>(j->dbuf + o_off),
                                       reinterpret_cast<const uint64_t*>(j->dbuf + o_len), n,
                                       reinterpret_cast<uint32_t*>(j->dbuf + o_out), j->stream),
            "k_sha512_digest32 launch");
    return 0;
  });
  if (rc) return job_abort(j, rc);
  job_out(j, out32, o_out, 32 * n);
  *job = j;
  return 0;
}

// ---- primary messages ------------------------------------------------------------------
// 256-byte aligned sections of a job's staging buffers (pinned and device share one layout).
struct Packer {
  size_t off = 0;
  size_t add(size_t bytes) {
    const size_t o = off;
    off += a256(bytes ? bytes : 1);
    return o;
  }
};

void put(nw_job* j, size_t off, const void* src, size_t bytes) {
  if (bytes) memcpy(j->hbuf + off, src, bytes);
}

// The committee's arrays in the staging buffer; returns its device view.
struct CommitteeOffs {
  size_t pks, stakes, wo, wi;
};
CommitteeOffs plan_committee(Packer& P, const nw_committee* com) {
  const size_t na = com->nauth, nwk = na ? com->worker_offsets[na] : 0;
  CommitteeOffs o;
  o.pks = P.add(32 * na);
  o.stakes = P.add(4 * na);
  o.wo = P.add(8 * (na + 1));
  o.wi = P.add(4 * nwk);
  return o;
}
nw_committee stage_committee(nw_job* j, const CommitteeOffs& o, const nw_committee* com) {
  const size_t na = com->nauth, nwk = na ? com->worker_offsets[na] : 0;
  put(j, o.pks, com->pks, 32 * na);
  put(j, o.stakes, com->stakes, 4 * na);
  put(j, o.wo, com->worker_offsets, 8 * (na + 1));
  put(j, o.wi, com->worker_ids, 4 * nwk);
  nw_committee d;
  d.nauth = na;
  d.pks = reinterpret_cast<const uint8_t*>(j->dbuf + o.pks);
  d.stakes = reinterpret_cast<const uint32_t*>(j->dbuf + o.stakes);
  d.worker_offsets = reinterpret_cast<const uint64_t*>(j->dbuf + o.wo);
  d.worker_ids = reinterpret_cast<const uint32_t*>(j->dbuf + o.wi);
  return d;
}

// ---- small jobs: one launch (nw_small.hip) ----------------------------------------------
// NW_SMALL=0 turns the small-job path off, NW_SMALL=1 takes it whenever it applies whatever
// the size (test hook); NW_SMALL_MAX_SLOTS = the largest job (signatures) it takes by default.
int small_mode() {
  const char* e = getenv("NW_SMALL");
  return e && *e ? atoi(e) : -1;
}
uint64_t small_max_slots() {
  const char* e = getenv("NW_SMALL_MAX_SLOTS");
  const long long v = e && *e ? atoll(e) : 0;
  return v > 0 ? (uint64_t)v : 65536;
}
// Slots per workgroup: the fewest (shortest comb chains) that keep the grid within ~2
// workgroups per CU.
uint32_t small_slots_per_wg(uint64_t nslots) {
  const char* e = getenv("NW_SMALL_S");   // test hook: a fixed S (4, 8, 16, 32 or 64)
  if (e && *e) {
    const int s = atoi(e);
    if (s == 4 || s == 8 || s == 16 || s == 32 || s == 64) return (uint32_t)s;
  }
  uint32_t S = 4;
  while (S < 64 && (nslots + S - 1) / S > 512) S *= 2;
  return S;
}

// Message jobs by path (nw_path_stats).
std::atomic<uint64_t> g_small_jobs{0}, g_pipeline_jobs{0};

// The per-message arrival counters of a job (device, zero; kernels leave them zero).
int job_counters(nw_job* j, size_t n) {
  if (n <= j->ccap) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  if (j->dcnt) (void)hipFree(j->dcnt);
  j->dcnt = nullptr;
  j->ccap = 0;
  const size_t cap = n < 4096 ? 4096 : n + n / 4;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&j->dcnt), 4 * cap);
  if (e == hipSuccess) e = hipMemsetAsync(j->dcnt, 0, 4 * cap, j->stream);
  if (e != hipSuccess) return set_err(NW_E_OUT_OF_MEMORY, "hipMalloc (job counters)", e);
  j->ccap = cap;
  log_growth(2, 4 * cap, t0);
  return 0;
}

// Header / Vote / Certificate checks of a small job in one launch. Returns 0 with *job set
// when it took the job, 1 when the job does not qualify (size, committee, key tables not
// built for this committee yet: the caller runs the ordinary pipeline, which builds them),
// or a negative NW_E_*. cs: certificates / headers; for votes the vote arrays.
struct VoteArrays {
  const uint8_t *ids, *origins, *authors, *sigs;
  const uint64_t* rounds;
  size_t n;
};
int submit_small(int dev, uint32_t kind, const nw_committee* com, const nw_certificates* cs,
                 const VoteArrays* va, const uint8_t* z16, int32_t* status_out,
                 uint64_t* index_out, nw_job** job) {
  const int mode = small_mode();
  if (mode == 0) return 1;
  const size_t na = com->nauth;
  if (na == 0 || na > 256) return 1;
  const size_t n = kind == nw::kSmallVotes ? va->n : cs->n;
  if (n == 0 || n >= (1ull << 31)) return 1;
  size_t nv = 0;
  if (kind == nw::kSmallCerts) {
    nv = cs->vote_offsets[n];
    for (size_t i = 0; i < n; ++i)
      if (cs->vote_offsets[i + 1] - cs->vote_offsets[i] > 128) return 1;   // quorum pass limit
  }
  const uint64_t nslots = n + nv;
  if (mode != 1 && nslots > small_max_slots()) return 1;
  if (nslots >= (1ull << 31)) return 1;
  const nw::ge_niels_pad* bcomb = nullptr;
  {
    int rc = nw::rt::use_device(dev);
    if (rc) return rc;
    hipError_t e = nw::bcomb_table(&bcomb);
    if (e != hipSuccess) return 1;   // the ordinary pipeline reports what failed
  }
  nw_job* j;
  int rc = job_acquire(dev, &j);
  if (rc) return rc;
  Packer P;
  const size_t nwk = com->worker_offsets[na];
  const size_t o_pk = P.add(32 * na), o_stk = P.add(4 * na), o_wo = P.add(8 * (na + 1)),
               o_wi = P.add(4 * nwk);
  size_t o_hb = 0, o_ho = 0, o_pc = 0, o_id = 0, o_hs = 0, o_vp = 0, o_vs = 0, o_z = 0;
  size_t o_rd = 0, o_or = 0, o_au = 0, o_sg = 0;
  uint64_t hb0 = 0, hlen = 0;
  if (kind == nw::kSmallVotes) {
    o_id = P.add(32 * n); o_rd = P.add(8 * n); o_or = P.add(32 * n); o_au = P.add(32 * n);
    o_sg = P.add(64 * n);
  } else {
    hb0 = cs->header_offsets[0];
    hlen = cs->header_offsets[n] - hb0;
    o_hb = P.add(hlen); o_ho = P.add(8 * (n + 1)); o_pc = P.add(4 * n); o_id = P.add(32 * n);
    o_hs = P.add(64 * n);
    if (kind == nw::kSmallCerts) {
      o_vp = P.add(32 * nv); o_vs = P.add(64 * nv);
      if (z16) o_z = P.add(16 * nv);
    }
  }
  const size_t o_sl = P.add(sizeof(nw::small_slot_t) * nslots);
  const size_t o_st = P.add(4 * n), o_ix = P.add(8 * n);
  const uint32_t S_wg = small_slots_per_wg(nslots);
  const uint64_t nwg_all = (nslots + S_wg - 1) / S_wg;
  const size_t o_df = P.add(4 * nwg_all), hend = P.off;   // NW_SMALL_DONE flags
  Packer D;
  const size_t d_mi = D.add(sizeof(nw::small_msg_info_t) * n), d_sr = D.add(4 * nslots);
  rc = job_reserve(j, hend, D.off);
  if (!rc) rc = job_counters(j, n);
  if (rc) return job_abort(j, rc);
  char* H = j->hbuf;
  put(j, o_pk, com->pks, 32 * na);
  put(j, o_stk, com->stakes, 4 * na);
  put(j, o_wo, com->worker_offsets, 8 * (na + 1));
  put(j, o_wi, com->worker_ids, 4 * nwk);
  nw::small_slot_t* sl = reinterpret_cast<nw::small_slot_t*>(H + o_sl);
  if (kind == nw::kSmallVotes) {
    put(j, o_id, va->ids, 32 * n);
    put(j, o_rd, va->rounds, 8 * n);
    put(j, o_or, va->origins, 32 * n);
    put(j, o_au, va->authors, 32 * n);
    put(j, o_sg, va->sigs, 64 * n);
    for (size_t i = 0; i < n; ++i) sl[i] = {(uint32_t)i, 0u, 0u, 1u};
  } else {
    put(j, o_hb, cs->header_bytes + hb0, hlen);
    uint64_t* ho = reinterpret_cast<uint64_t*>(H + o_ho);
    for (size_t i = 0; i <= n; ++i) ho[i] = cs->header_offsets[i] - hb0;
    put(j, o_pc, cs->payload_counts, 4 * n);
    put(j, o_id, cs->ids, 32 * n);
    put(j, o_hs, cs->header_sigs, 64 * n);
    if (kind == nw::kSmallCerts) {
      put(j, o_vp, cs->vote_pks, 32 * nv);
      put(j, o_vs, cs->vote_sigs, 64 * nv);
      if (z16) put(j, o_z, z16, 16 * nv);
      size_t s = 0;
      for (size_t i = 0; i < n; ++i) {
        const uint32_t v0 = (uint32_t)cs->vote_offsets[i];
        const uint32_t q = (uint32_t)(cs->vote_offsets[i + 1] - v0);
        for (uint32_t t = 0; t <= q; ++t) sl[s++] = {(uint32_t)i, t, v0 + (t ? t - 1 : 0), q + 1};
      }
    } else {
      for (size_t i = 0; i < n; ++i) sl[i] = {(uint32_t)i, 0u, 0u, 1u};
    }
  }
  char* X = j->hdev;   // the device's view of the staging buffer
  if (small_vram() && job_reserve_vram(j, o_st) == 0) {
    static std::once_flag said;   // (the opt-in path announces itself once per process)
    std::call_once(said, [] {
      fprintf(stderr, "[narwhal_amd] NW_SMALL_VRAM: small jobs' inputs written into "
              "host-mapped fine-grained device memory\n");
    });
    memcpy(j->vhost, H, o_st);   // the inputs (everything before the outputs)
    std::atomic_thread_fence(std::memory_order_seq_cst);   // drain the write-combining buffers
    X = j->vbuf;
  }
  nw::small_job_t J{};
  J.kind = kind;
  J.slots_per_wg = small_slots_per_wg(nslots);
  J.nmsg = n;
  J.nslots = nslots;
  J.com = nw::cert_committee_t{na, reinterpret_cast<const uint32_t*>(X + o_pk),
                               reinterpret_cast<const uint32_t*>(X + o_stk),
                               reinterpret_cast<const uint64_t*>(X + o_wo),
                               reinterpret_cast<const uint32_t*>(X + o_wi)};
  if (kind == nw::kSmallVotes) {
    J.ids = reinterpret_cast<const uint32_t*>(X + o_id);
    J.rounds = reinterpret_cast<const uint64_t*>(X + o_rd);
    J.origins = reinterpret_cast<const uint32_t*>(X + o_or);
    J.authors = reinterpret_cast<const uint32_t*>(X + o_au);
    J.sigs = reinterpret_cast<const uint32_t*>(X + o_sg);
  } else {
    J.hb = reinterpret_cast<const uint8_t*>(X + o_hb);
    J.ho = reinterpret_cast<const uint64_t*>(X + o_ho);
    J.pc = reinterpret_cast<const uint32_t*>(X + o_pc);
    J.ids = reinterpret_cast<const uint32_t*>(X + o_id);
    J.hsig = reinterpret_cast<const uint32_t*>(X + o_hs);
    if (kind == nw::kSmallCerts) {
      J.vpk = reinterpret_cast<const uint32_t*>(X + o_vp);
      J.vsig = reinterpret_cast<const uint32_t*>(X + o_vs);
      J.z16 = z16 ? reinterpret_cast<const uint32_t*>(X + o_z) : nullptr;
    }
  }
  J.slots = reinterpret_cast<const nw::small_slot_t*>(X + o_sl);
  J.bcomb = bcomb;
  if (!z16) {
    rc = nw::rt::os_random(J.zkey, 32);
    if (rc) return job_abort(j, rc);
  }
  J.minfo = reinterpret_cast<nw::small_msg_info_t*>(j->dbuf + d_mi);
  J.srec = reinterpret_cast<uint32_t*>(j->dbuf + d_sr);
  J.mcount = j->dcnt;
  J.status = reinterpret_cast<int32_t*>(j->hdev + o_st);
  J.index = kind == nw::kSmallVotes ? nullptr : reinterpret_cast<uint64_t*>(j->hdev + o_ix);
  uint32_t dseq = 0;
  if (small_done() && J.slots_per_wg == S_wg) {
    dseq = next_done_seq();
    // the flag words start at 0 (never a sequence number): a staging buffer reallocated from
    // another job's freed pinned memory may hold that job's old flags, and its sequence may
    // equal ours (profiles/r06aa: rare stale verdicts before this line)
    if (test_stale_flags()) {
      // test hook (NW_TEST_STALE_FLAGS=1): the buffer arrives holding this very sequence in
      // every flag word, the worst a recycled buffer can hold; the memset below must clear it
      uint32_t* f = reinterpret_cast<uint32_t*>(H + o_df);
      for (uint64_t w = 0; w < nwg_all; ++w) f[w] = dseq;
    }
#ifndef NW_NO_FLAG_CLEAR   // negative control build only (tools/r06/gpu_ae.sh)
    memset(H + o_df, 0, 4 * nwg_all);
#endif
    J.done_flags = reinterpret_cast<uint32_t*>(j->hdev + o_df);
    J.done_seq = dseq;
  }
  nw::rt::ReadLease rl;
  const void* tabs = nullptr;
  const uint32_t* ok = nullptr;
  nw::keyspec ks{};
  rc = rl.acquire(dev, j->stream, com->pks, na, &tabs, &ok, &ks);
  if (rc) {   // 1: no tables for this committee yet (or an error): not taken here
    job_recycle(j);
    return rc;
  }
  J.ktabs = static_cast<const nw::ge_niels_pad*>(tabs);
  J.kok = ok;
  J.ks = ks;
  const char* se = getenv("NW_SMALL_STAMPS");   // diagnostics: per-phase times of this launch
  const uint64_t nwg = (nslots + J.slots_per_wg - 1) / J.slots_per_wg;
  if (se && *se && *se != '0') (void)hipMalloc(reinterpret_cast<void**>(&J.stamps), 64 * nwg);
  hipError_t e = nw::launch_small(J, j->stream);
  const int rrc = rl.release();
  if (e != hipSuccess) return job_abort(j, set_err(NW_E_DEVICE, "k_small launch", e));
  if (rrc) return job_abort(j, rrc);
  if (J.stamps) {
    std::vector<uint64_t> st(8 * nwg);
    if (hipMemcpyAsync(st.data(), J.stamps, 64 * nwg, hipMemcpyDeviceToHost, j->stream) ==
            hipSuccess &&
        hipStreamSynchronize(j->stream) == hipSuccess) {
      // per phase: median over workgroups of (stamp - the workgroup's start), microseconds
      double med[8];
      for (int p = 0; p < 8; ++p) {
        std::vector<double> v;
        for (uint64_t w = 0; w < nwg; ++w)
          if (st[8 * w + p] >= st[8 * w]) v.push_back((double)(st[8 * w + p] - st[8 * w]) * 0.01);
        std::sort(v.begin(), v.end());
        med[p] = v.empty() ? -1.0 : v[v.size() / 2];
      }
      uint64_t t0 = ~0ull, t1 = 0, s1 = 0, wl = 0;
      for (uint64_t w = 0; w < nwg; ++w) {
        t0 = std::min(t0, st[8 * w]);
        s1 = std::max(s1, st[8 * w]);
        if (st[8 * w + 7] > t1) {
          t1 = st[8 * w + 7];
          wl = w;
        }
      }
      // the workgroup that ended last: its phases relative to its own start
      double last[8];
      for (int p = 0; p < 8; ++p)
        last[p] = st[8 * wl + p] >= st[8 * wl] ? (double)(st[8 * wl + p] - st[8 * wl]) * 0.01 : -1.0;
      fprintf(stderr, "[narwhal_amd] k_small kind=%u slots=%llu S=%u wgs=%llu: decomp %.1f msg %.1f "
              "digits %.1f comb %.1f sync %.1f slots %.1f end %.1f us (median per workgroup); "
              "first start -> last end %.1f us, last start +%.1f us; last-ending wg %llu "
              "(start +%.1f): decomp %.1f msg %.1f digits %.1f comb %.1f sync %.1f slots %.1f "
              "end %.1f\n", kind, (unsigned long long)nslots,
              J.slots_per_wg, (unsigned long long)nwg, med[1], med[2], med[3], med[4], med[5],
              med[6], med[7], (double)(t1 - t0) * 0.01, (double)(s1 - t0) * 0.01,
              (unsigned long long)wl, (double)(st[8 * wl] - t0) * 0.01, last[1], last[2],
              last[3], last[4], last[5], last[6], last[7]);
    }
    (void)hipFree(J.stamps);
  }
  e = hipEventRecord(j->done, j->stream);
  if (e != hipSuccess) return job_abort(j, set_err(NW_E_DEVICE, "hipEventRecord", e));
  j->pending = true;
  job_out(j, status_out, o_st, 4 * n);
  if (kind != nw::kSmallVotes) job_out(j, index_out, o_ix, 8 * n);
  if (J.done_flags) {
    j->small_flags = reinterpret_cast<volatile uint32_t*>(H + o_df);
    j->small_nwg = (uint32_t)nwg_all;
    j->spin_seq = dseq;
  }
  g_small_jobs.fetch_add(1, std::memory_order_relaxed);
  *job = j;
  return 0;
}

// Header::verify / Certificate::verify over one device: the committee and the stream are
// packed into the job's pinned buffer (one H2D copy), then the device pipeline
// (nw::rt::cert_pipeline: shared lease, committee key tables kept across calls, adaptive
// grouping) and one D2H copy of the statuses and indices.
int submit_certs(int dev, const nw_committee* com, const nw_certificates* cs, int headers_only,
                 const uint8_t* z16, int32_t* status_out, uint64_t* index_out, nw_job** job) {
  size_t nv = 0;
  int rc = nw::rt::check_committee(com);
  if (!rc) rc = nw::rt::check_certificates(cs, headers_only, &nv);
  if (rc) return rc;
  if (cs->n && !status_out) return set_err(NW_E_INVALID_ARG, "null status_out");
  if (cs->n) {   // a small job: one launch (nw_small.hip), when it qualifies
    rc = submit_small(dev, headers_only ? nw::kSmallHeaders : nw::kSmallCerts, com, cs, nullptr,
                      z16, status_out, index_out, job);
    if (rc <= 0) return rc;
    g_pipeline_jobs.fetch_add(1, std::memory_order_relaxed);
  }
  nw_job* j;
  rc = job_acquire(dev, &j);
  if (rc) return rc;
  const size_t n = cs->n;
  if (n == 0) {
    *job = j;
    return 0;
  }
  const uint64_t hb0 = cs->header_offsets[0], hlen = cs->header_offsets[n] - hb0;
  Packer P;
  const CommitteeOffs oc = plan_committee(P, com);
  const size_t o_hb = P.add(hlen), o_ho = P.add(8 * (n + 1)), o_pc = P.add(4 * n),
               o_id = P.add(32 * n), o_hs = P.add(64 * n);
  size_t o_vo = 0, o_vp = 0, o_vs = 0, o_z = 0;
  if (!headers_only) {
    o_vo = P.add(8 * (n + 1));
    o_vp = P.add(32 * nv);
    o_vs = P.add(64 * nv);
    if (z16) o_z = P.add(16 * nv);
  }
  const size_t o_st = P.add(4 * n), o_ix = P.add(8 * n), out_end = P.off;
  const size_t o_ws = P.add(nw::rt::cert_workspace_bytes(n, nv));
  rc = job_reserve(j, out_end, P.off);
  if (rc) return job_abort(j, rc);
  const nw_committee dcom = stage_committee(j, oc, com);
  const uint64_t ctag = nw::rt::committee_hash(com);
  put(j, o_hb, cs->header_bytes + hb0, hlen);
  uint64_t* ho = reinterpret_cast<uint64_t*>(j->hbuf + o_ho);
  for (size_t i = 0; i <= n; ++i) ho[i] = cs->header_offsets[i] - hb0;
  put(j, o_pc, cs->payload_counts, 4 * n);
  put(j, o_id, cs->ids, 32 * n);
  put(j, o_hs, cs->header_sigs, 64 * n);
  nw_certificates d{};
  d.n = n;
  d.header_bytes = reinterpret_cast<const uint8_t*>(j->dbuf + o_hb);
  d.header_offsets = reinterpret_cast<const uint64_t*>(j->dbuf + o_ho);
  d.payload_counts = reinterpret_cast<const uint32_t*>(j->dbuf + o_pc);
  d.ids = reinterpret_cast<const uint8_t*>(j->dbuf + o_id);
  d.header_sigs = reinterpret_cast<const uint8_t*>(j->dbuf + o_hs);
  d.header_bytes_len = hlen;
  const uint64_t* hvo = nullptr;
  if (!headers_only) {
    put(j, o_vo, cs->vote_offsets, 8 * (n + 1));
    put(j, o_vp, cs->vote_pks, 32 * nv);
    put(j, o_vs, cs->vote_sigs, 64 * nv);
    if (z16) put(j, o_z, z16, 16 * nv);
    d.vote_offsets = reinterpret_cast<const uint64_t*>(j->dbuf + o_vo);
    d.vote_pks = reinterpret_cast<const uint8_t*>(j->dbuf + o_vp);
    d.vote_sigs = reinterpret_cast<const uint8_t*>(j->dbuf + o_vs);
    d.nvotes = nv;
    hvo = reinterpret_cast<const uint64_t*>(j->hbuf + o_vo);   // read while planning only
  }
  if (!headers_only) ensure_fork(j);
  rc = job_run(j, o_st, o_st, out_end - o_st, [&]() -> int {
    return nw::rt::cert_pipeline(dev, dcom, d, hvo, headers_only, z16 ? j->dbuf + o_z : nullptr,
                                 nullptr, j->dbuf + o_ws,
                                 reinterpret_cast<int32_t*>(j->dbuf + o_st),
                                 reinterpret_cast<uint64_t*>(j->dbuf + o_ix), j->stream, ctag,
                                 j->fork.s2 ? &j->fork : nullptr, com->pks);
  });
  if (rc) return job_abort(j, rc);
  job_out(j, status_out, o_st, 4 * n);
  job_out(j, index_out, o_ix, 8 * n);
  *job = j;
  return 0;
}

// Vote::verify over one device (nw::rt::votes_pipeline: committee members' signatures take
// the keyed comb over the shared key tables).
int submit_votes(int dev, const nw_committee* com, const uint8_t* ids, const uint64_t* rounds,
                 const uint8_t* origins, const uint8_t* authors, const uint8_t* sigs, size_t n,
                 int32_t* status_out, nw_job** job) {
  int rc = nw::rt::check_committee(com);
  if (rc) return rc;
  if (n && (!ids || !rounds || !origins || !authors || !sigs || !status_out))
    return set_err(NW_E_INVALID_ARG, "null pointer");
  if (n) {   // a small job: one launch (nw_small.hip), when it qualifies
    const VoteArrays va{ids, origins, authors, sigs, rounds, n};
    rc = submit_small(dev, nw::kSmallVotes, com, nullptr, &va, nullptr, status_out, nullptr, job);
    if (rc <= 0) return rc;
    g_pipeline_jobs.fetch_add(1, std::memory_order_relaxed);
  }
  nw_job* j;
  rc = job_acquire(dev, &j);
  if (rc) return rc;
  if (n == 0) {
    *job = j;
    return 0;
  }
  Packer P;
  const CommitteeOffs oc = plan_committee(P, com);
  const size_t o_id = P.add(32 * n), o_rd = P.add(8 * n), o_or = P.add(32 * n),
               o_au = P.add(32 * n), o_sg = P.add(64 * n);
  const size_t o_st = P.add(4 * n), out_end = P.off;
  const size_t o_ws = P.add(nw::rt::votes_workspace_bytes(n));
  rc = job_reserve(j, out_end, P.off);
  if (rc) return job_abort(j, rc);
  const nw_committee dcom = stage_committee(j, oc, com);
  put(j, o_id, ids, 32 * n);
  put(j, o_rd, rounds, 8 * n);
  put(j, o_or, origins, 32 * n);
  put(j, o_au, authors, 32 * n);
  put(j, o_sg, sigs, 64 * n);
  rc = job_run(j, o_st, o_st, out_end - o_st, [&]() -> int {
    const auto* b = reinterpret_cast<const uint8_t*>(j->dbuf);
    return nw::rt::votes_pipeline(dev, dcom, n, b + o_id,
                                  reinterpret_cast<const uint64_t*>(b + o_rd), b + o_or,
                                  b + o_au, b + o_sg, j->dbuf + o_ws,
                                  reinterpret_cast<int32_t*>(j->dbuf + o_st), j->stream,
                                  com->pks);
  });
  if (rc) return job_abort(j, rc);
  job_out(j, status_out, o_st, 4 * n);
  *job = j;
  return 0;
}

// ---- fan-out --------------------------------------------------------------------------
// Runs submit(device, begin, end, &job) for each non-empty part [b[p], b[p+1]) and returns a
// parent over the parts (or, for a single device without NW_ALL_DEVICES, the job itself).
template <class Submit>
int fan_out(const std::vector<int>& devs, const std::vector<size_t>& b, Submit submit,
            nw_job** job) {
  nw_job* parent = new (std::nothrow) nw_job;
  if (!parent) return set_err(NW_E_OUT_OF_MEMORY, "job allocation");
  for (size_t p = 0; p + 1 < b.size(); ++p) {
    if (b[p + 1] == b[p] && !(p == 0 && b.back() == 0)) continue;
    nw_job* sub = nullptr;
    const int rc = submit(devs[p], b[p], b[p + 1], &sub);
    if (rc) {
      job_recycle(parent);
      return rc;
    }
    parent->parts.push_back(sub);
  }
  *job = parent;
  return 0;
}

// Part p of n items over P parts, boundaries rounded down to a multiple of `align`.
std::vector<size_t> even_bounds(size_t n, size_t P, size_t align) {
  std::vector<size_t> b(P + 1);
  for (size_t p = 0; p <= P; ++p) b[p] = p == P ? n : std::min(n, n * p / P / align * align);
  return b;
}

// Boundaries (indices into n units) with about equal weight prefix[i] per part.
std::vector<size_t> weighted_bounds(size_t n, size_t P, const std::vector<uint64_t>& prefix) {
  std::vector<size_t> b(P + 1, 0);
  const uint64_t tot = prefix[n];
  size_t i = 0;
  for (size_t p = 1; p < P; ++p) {
    const uint64_t target = tot * p / P;
    while (i < n && prefix[i] < target) ++i;
    b[p] = i;
  }
  b[P] = n;
  return b;
}

// Header / Certificate submits: one device, or whole messages per device with about equal
// work (1 per header + 1 per vote).
int submit_messages(const nw_committee* com, const nw_certificates* cs, int headers_only,
                    const uint8_t* z16, int32_t* status_out, uint64_t* index_out,
                    nw_job** job) {
  const std::vector<int> devs = nw::rt::fanout_devices();
  if (devs.empty()) {
    int dev = 0;
    int rc = nw::rt::select_device(&dev);
    return rc ? rc : submit_certs(dev, com, cs, headers_only, z16, status_out, index_out, job);
  }
  size_t nv = 0;
  int rc = nw::rt::check_committee(com);
  if (!rc) rc = nw::rt::check_certificates(cs, headers_only, &nv);
  if (rc) return rc;
  const size_t n = cs->n;
  std::vector<uint64_t> w(n + 1, 0);
  for (size_t i = 0; i < n; ++i)
    w[i + 1] = w[i] + 1 + (headers_only ? 0 : cs->vote_offsets[i + 1] - cs->vote_offsets[i]);
  return fan_out(devs, weighted_bounds(n, devs.size(), w),
                 [&](int dev, size_t a, size_t e, nw_job** sub) {
                   nw_certificates part = *cs;
                   part.n = e - a;
                   part.header_offsets = cs->header_offsets + a;   // absolute: rebased
                   part.payload_counts = cs->payload_counts + a;
                   part.ids = cs->ids + 32 * a;
                   part.header_sigs = cs->header_sigs + 64 * a;
                   std::vector<uint64_t> vo;
                   const uint8_t* pz = z16;
                   if (!headers_only) {
                     const uint64_t v0 = cs->vote_offsets[a];
                     vo.resize(e - a + 1);
                     for (size_t i = a; i <= e; ++i) vo[i - a] = cs->vote_offsets[i] - v0;
                     part.vote_offsets = vo.data();   // copied into the part's staging
                     part.vote_pks = cs->vote_pks ? cs->vote_pks + 32 * v0 : nullptr;
                     part.vote_sigs = cs->vote_sigs ? cs->vote_sigs + 64 * v0 : nullptr;
                     if (z16) pz = z16 + 16 * v0;
                   }
                   return submit_certs(dev, com, &part, headers_only, pz,
                                       status_out ? status_out + a : nullptr,
                                       index_out ? index_out + a : nullptr, sub);
                 },
                 job);
}

}  // namespace

extern "C" {

int nw_submit_verify_strict(const uint8_t* digests, size_t digest_stride, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, int32_t* status_out,
                            uint8_t* bitmap_out, nw_job** job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job pointer");
  *job = nullptr;
  if (n && (!digests || !pks || !sigs)) return set_err(NW_E_INVALID_ARG, "null pointer");
  if (digest_stride != 0 && digest_stride != 32)
    return set_err(NW_E_INVALID_ARG, "digest_stride must be 0 or 32");
  const std::vector<int> devs = nw::rt::fanout_devices();
  if (devs.empty()) {
    int dev = 0;
    int rc = nw::rt::select_device(&dev);
    return rc ? rc : submit_strict(dev, digests, digest_stride, pks, sigs, n, status_out,
                                   bitmap_out, job);
  }
  return fan_out(devs, even_bounds(n, devs.size(), 64),
                 [&](int dev, size_t a, size_t e, nw_job** sub) {
                   return submit_strict(dev, digests + (digest_stride ? 32 * a : 0),
                                        digest_stride, pks + 32 * a, sigs + 64 * a, e - a,
                                        status_out ? status_out + a : nullptr,
                                        bitmap_out ? bitmap_out + a / 8 : nullptr, sub);
                 },
                 job);
}

int nw_submit_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                                const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                                int32_t* status_out, uint64_t* fail_index_out, nw_job** job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job pointer");
  *job = nullptr;
  if (nbatches && (!digests || !offsets)) return set_err(NW_E_INVALID_ARG, "null pointer");
  if (nbatches) {
    if (offsets[0] != 0) return set_err(NW_E_INVALID_ARG, "offsets[0] must be 0");
    for (size_t b = 0; b < nbatches; ++b)
      if (offsets[b + 1] < offsets[b]) return set_err(NW_E_INVALID_ARG, "offsets not monotone");
  }
  const size_t nitems = nbatches ? offsets[nbatches] : 0;
  if (nitems && (!pks || !sigs)) return set_err(NW_E_INVALID_ARG, "null pointer");
  const std::vector<int> devs = nw::rt::fanout_devices();
  if (devs.empty()) {
    int dev = 0;
    int rc = nw::rt::select_device(&dev);
    return rc ? rc : submit_batch(dev, digests, pks, sigs, offsets, nbatches, z16, status_out,
                                  fail_index_out, job);
  }
  // whole batches per part, about equal votes (+1 per batch for its fixed tail)
  std::vector<uint64_t> w(nbatches + 1);
  for (size_t b = 0; b <= nbatches; ++b) w[b] = offsets[b] + b;
  return fan_out(devs, weighted_bounds(nbatches, devs.size(), w),
                 [&](int dev, size_t a, size_t e, nw_job** sub) {
                   std::vector<uint64_t> off(e - a + 1);
                   for (size_t b = a; b <= e; ++b) off[b - a] = offsets[b] - offsets[a];
                   const uint64_t v0 = offsets[a];
                   return submit_batch(dev, digests + 32 * a, pks ? pks + 32 * v0 : nullptr,
                                       sigs ? sigs + 64 * v0 : nullptr, off.data(), e - a,
                                       z16 ? z16 + 16 * v0 : nullptr,
                                       status_out ? status_out + a : nullptr,
                                       fail_index_out ? fail_index_out + a : nullptr, sub);
                 },
                 job);
}

int nw_submit_sha512_digest32_many(const uint8_t* data, const uint64_t* offsets,
                                   const uint64_t* lengths, size_t n, uint8_t* out32,
                                   nw_job** job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job pointer");
  *job = nullptr;
  if (n && (!data || !offsets || !lengths || !out32))
    return set_err(NW_E_INVALID_ARG, "null pointer");
  const std::vector<int> devs = nw::rt::fanout_devices();
  if (devs.empty()) {
    int dev = 0;
    int rc = nw::rt::select_device(&dev);
    return rc ? rc : submit_sha(dev, data, offsets, lengths, n, out32, job);
  }
  // whole messages per part, about equal bytes (+1 per message)
  std::vector<uint64_t> w(n + 1, 0);
  for (size_t i = 0; i < n; ++i) w[i + 1] = w[i] + lengths[i] + 1;
  return fan_out(devs, weighted_bounds(n, devs.size(), w),
                 [&](int dev, size_t a, size_t e, nw_job** sub) {
                   return submit_sha(dev, data, offsets + a, lengths + a, e - a, out32 + 32 * a,
                                     sub);
                 },
                 job);
}

int nw_submit_certificates_verify_many(const nw_committee* committee,
                                       const nw_certificates* certs, const uint8_t* z16,
                                       int32_t* status_out, uint64_t* index_out, nw_job** job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job pointer");
  *job = nullptr;
  return submit_messages(committee, certs, 0, z16, status_out, index_out, job);
}

int nw_submit_headers_verify_many(const nw_committee* committee, const nw_certificates* headers,
                                  int32_t* status_out, uint64_t* index_out, nw_job** job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job pointer");
  *job = nullptr;
  return submit_messages(committee, headers, 1, nullptr, status_out, index_out, job);
}

int nw_submit_votes_verify_many(const nw_committee* committee, const uint8_t* ids,
                                const uint64_t* rounds, const uint8_t* origins,
                                const uint8_t* authors, const uint8_t* sigs, size_t n,
                                int32_t* status_out, nw_job** job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job pointer");
  *job = nullptr;
  if (n && (!ids || !rounds || !origins || !authors || !sigs || !status_out))
    return set_err(NW_E_INVALID_ARG, "null pointer");
  const std::vector<int> devs = nw::rt::fanout_devices();
  if (devs.empty()) {
    int dev = 0;
    int rc = nw::rt::select_device(&dev);
    return rc ? rc : submit_votes(dev, committee, ids, rounds, origins, authors, sigs, n,
                                  status_out, job);
  }
  int rc = nw::rt::check_committee(committee);
  if (rc) return rc;
  return fan_out(devs, even_bounds(n, devs.size(), 1),
                 [&](int dev, size_t a, size_t e, nw_job** sub) {
                   return submit_votes(dev, committee, ids + 32 * a, rounds + a, origins + 32 * a,
                                       authors + 32 * a, sigs + 64 * a, e - a, status_out + a,
                                       sub);
                 },
                 job);
}

int nw_job_poll(nw_job* job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job");
  if (!job->parts.empty()) {
    int done = 1;
    for (nw_job* x : job->parts) {
      const int rc = nw_job_poll(x);
      if (rc < 0) return rc;
      done &= rc;
    }
    return done;
  }
  if (!job->pending) return 1;
  if (job->early) return 1;
  if (job->small_flags && small_flags_done(job)) {   // every workgroup's writes are out
    job_deliver_early(job);
    return 1;
  }
  hipError_t e = hipEventQuery(job->done);
  if (e == hipErrorNotReady) return 0;
  if (e != hipSuccess) {
    if (job->dfz) job->dfz_dirty = true;   // counters of a failed fused launch: clear on reuse
    return set_err(NW_E_DEVICE, "hipEventQuery", e);
  }
  job_deliver(job);
  return 1;
}

int nw_job_wait(nw_job* job) {
  if (!job) return set_err(NW_E_INVALID_ARG, "null job");
  if (!job->parts.empty()) {
    int first = 0;
    for (nw_job* x : job->parts) {
      const int rc = nw_job_wait(x);
      if (rc && !first) first = rc;
    }
    return first;
  }
  if (!job->pending) return 0;
  if (job->early) return 0;
  if (job->small_flags) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!small_flags_done(job)) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    if (small_flags_done(job)) {
      job_deliver_early(job);
      return 0;
    }
    job->small_flags = nullptr;
  }
  if (job->spin) {
    // NW_BATCH_SPIN: the tail's done word, for up to 20 ms (then the event, as usual)
    const auto t0 = std::chrono::steady_clock::now();
    while (*job->spin != job->spin_seq) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) break;
    }
    if (*job->spin == job->spin_seq) {
      job_deliver_early(job);   // pending stays set: the next acquire synchronises
      return 0;
    }
    job->spin = nullptr;
  }
  const hipError_t e = hipEventSynchronize(job->done);
  if (e != hipSuccess) {
    if (job->dfz) job->dfz_dirty = true;   // counters of a failed fused launch: clear on reuse
    return set_err(NW_E_DEVICE, "hipEventSynchronize", e);
  }
  job_deliver(job);
  return 0;
}

namespace {
// fn(arg) once every part of a fan-out job has finished (from the last part's callback),
// unless arming failed (cancelled: the last tick only frees the countdown).
struct Countdown {
  std::atomic<int> left;
  std::atomic<bool> cancelled{false};
  void (*fn)(void*);
  void* arg;
};
void countdown_tick(void* p) {
  Countdown* c = static_cast<Countdown*>(p);
  if (c->left.fetch_sub(1) == 1) {
    if (!c->cancelled.load()) c->fn(c->arg);
    delete c;
  }
}

// Completion callbacks. A host function on the job's stream (hipLaunchHostFunc) is run by
// the HIP runtime's own thread some hundreds of microseconds after the stream reaches it
// and holds the stream until it returns; instead one watcher thread polls a marker event
// recorded behind each armed job and calls fn(arg) as soon as that event completes, in
// whatever order jobs finish. The stream never waits on the callback. Marker events are
// pooled. While anything is armed the watcher yields for a few polls, then naps 20 us, and
// 200 us once nothing has completed for ~2 ms (long bulk jobs: a wakeup a tenth of a
// millisecond late is noise, a core spinning for seconds is not); with nothing armed it
// sleeps on a condition variable. Callbacks of all jobs run one after another on this one
// thread. At process exit (atexit, registered after the HIP runtime's own teardown handlers
// so it runs before them) the watcher is stopped: callbacks still armed then never run.
struct Armed {
  int dev;
  hipEvent_t ev;
  void (*fn)(void*);
  void* arg;
};
struct Watcher {
  std::mutex m;
  std::condition_variable cv;
  std::vector<Armed> armed;        // guarded by m
  std::vector<hipEvent_t> pool[kMaxDev];   // per device, guarded by m
  bool started = false;
  bool stopping = false, stopped = false;   // guarded by m

  int arm(int dev, hipStream_t s, void (*fn)(void*), void* arg) {
    int rc = nw::rt::use_device(dev);
    if (rc) return rc;
    hipEvent_t ev = nullptr;
    {
      std::lock_guard<std::mutex> g(m);
      if (!pool[dev].empty()) {
        ev = pool[dev].back();
        pool[dev].pop_back();
      }
      if (stopping) return set_err(NW_E_DEVICE, "notify during process exit");
      if (!started) {
        std::thread(&Watcher::run, this).detach();
        started = true;
        atexit(quiesce_at_exit);
      }
    }
    hipError_t e = hipSuccess;
    if (!ev) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, s);
    if (e != hipSuccess) {
      if (ev) {
        std::lock_guard<std::mutex> g(m);
        pool[dev].push_back(ev);
      }
      return set_err(NW_E_DEVICE, "notify marker event", e);
    }
    {
      std::lock_guard<std::mutex> g(m);
      armed.push_back({dev, ev, fn, arg});
    }
    cv.notify_one();
    return 0;
  }

  void run() {
    std::vector<Armed> mine, ready;
    int idle = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m);
        for (const Armed& a : ready) pool[a.dev].push_back(a.ev);
        ready.clear();
        mine.insert(mine.end(), armed.begin(), armed.end());
        armed.clear();
        if (mine.empty()) cv.wait(g, [&] { return !armed.empty() || stopping; });
        mine.insert(mine.end(), armed.begin(), armed.end());
        armed.clear();
        if (stopping) {
          stopped = true;
          cv.notify_all();
          return;
        }
      }
      size_t keep = 0;
      for (const Armed& a : mine) {
        // a device error also ends the wait: the caller's poll / wait reports it
        if (hipEventQuery(a.ev) == hipErrorNotReady) mine[keep++] = a;
        else ready.push_back(a);
      }
      mine.resize(keep);
      for (const Armed& a : ready) a.fn(a.arg);
      if (!ready.empty()) idle = 0;
      else if (++idle > 64 + 100) std::this_thread::sleep_for(std::chrono::microseconds(200));
      else if (idle > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
      else std::this_thread::yield();
    }
  }

  // stop polling before the HIP runtime tears down; bounded, so a callback stuck in a
  // finalising interpreter cannot hang the exit
  void quiesce() {
    std::unique_lock<std::mutex> g(m);
    stopping = true;
    cv.notify_all();
    cv.wait_for(g, std::chrono::milliseconds(200), [&] { return stopped; });
  }
  static void quiesce_at_exit();
};
// never destroyed: a static destructor would destroy the condition variable the detached
// watcher waits on (pthread_cond_destroy blocks on waiters: a hang at process exit)
Watcher& g_watcher = *new Watcher;
void Watcher::quiesce_at_exit() { g_watcher.quiesce(); }
}  // namespace

int nw_job_notify(nw_job* job, void (*fn)(void*), void* arg) {
  if (!job || !fn) return set_err(NW_E_INVALID_ARG, "null job or callback");
  if (!job->parts.empty()) {
    Countdown* c = new (std::nothrow) Countdown;
    if (!c) return set_err(NW_E_OUT_OF_MEMORY, "notify");
    c->left = (int)job->parts.size() + 1;   // +1: released below, after every part is armed
    c->fn = fn;
    c->arg = arg;
    int first = 0;
    for (nw_job* x : job->parts) {
      const int rc = nw_job_notify(x, countdown_tick, c);
      if (rc) {
        if (!first) first = rc;
        countdown_tick(c);   // this part will never tick: count it now
      }
    }
    // our hold (+1) keeps the count above zero until here, so no part's tick can have
    // called fn yet: after an error, cancel before releasing it
    if (first) c->cancelled.store(true);
    countdown_tick(c);
    return first;
  }
  if (!job->pending) {
    fn(arg);
    return 0;
  }
  return g_watcher.arm(job->dev, job->stream, fn, arg);
}

void nw_job_release(nw_job* job) { job_recycle(job); }

int nw_path_stats(uint64_t* small_jobs, uint64_t* pipeline_jobs) {
  if (small_jobs) *small_jobs = g_small_jobs.load(std::memory_order_relaxed);
  if (pipeline_jobs) *pipeline_jobs = g_pipeline_jobs.load(std::memory_order_relaxed);
  return 0;
}

// ---- blocking host-buffer entry points = submit + wait ------------------------------
static int run_blocking(int rc, nw_job* j) {
  if (rc) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  rc = nw_job_wait(j);
  if (batch_stamps())
    fprintf(stderr, "[narwhal_amd] wait %.1f us\n",
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                .count());
  nw_job_release(j);
  return rc;
}

int nw_sha512_digest32_many(const uint8_t* data, const uint64_t* offsets,
                            const uint64_t* lengths, size_t n, uint8_t* out32) {
  nw_job* j = nullptr;
  return run_blocking(nw_submit_sha512_digest32_many(data, offsets, lengths, n, out32, &j), j);
}

int nw_verify_strict_many(const uint8_t* digests, size_t digest_stride, const uint8_t* pks,
                          const uint8_t* sigs, size_t n, int32_t* status_out,
                          uint8_t* bitmap_out) {
  nw_job* j = nullptr;
  return run_blocking(nw_submit_verify_strict(digests, digest_stride, pks, sigs, n, status_out,
                                              bitmap_out, &j),
                      j);
}

int nw_signature_verify(const uint8_t sig[64], const uint8_t digest[32], const uint8_t pk[32]) {
  int32_t st = 0;
  int rc = nw_verify_strict_many(digest, 32, pk, sig, 1, &st, nullptr);
  return rc ? rc : st;
}

int nw_signature_verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs,
                              size_t n, const uint8_t* z16, size_t* fail_index) {
  if (!digest || (n && (!pks || !sigs))) return set_err(NW_E_INVALID_ARG, "null pointer");
  if (n == 0) {   // crypto::verify_batch over no votes: dalek MSM of [0]B -> Ok
    int rc = nw::rt::ensure_init();
    if (rc) return rc;
    if (fail_index) *fail_index = 0;
    return NW_OK;
  }
  const uint64_t offs[2] = {0, n};
  int32_t st = 0;
  uint64_t fi = 0;
  nw_job* j = nullptr;
  int rc = run_blocking(nw_submit_verify_batch_many(digest, pks, sigs, offs, 1, z16, &st, &fi, &j),
                        j);
  if (rc) return rc;
  if (fail_index) *fail_index = (size_t)fi;
  return st;
}

int nw_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                         const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                         int32_t* status_out) {
  if (nbatches == 0) return nw::rt::ensure_init();
  if (!status_out) return set_err(NW_E_INVALID_ARG, "null pointer");
  nw_job* j = nullptr;
  return run_blocking(nw_submit_verify_batch_many(digests, pks, sigs, offsets, nbatches, z16,
                                                  status_out, nullptr, &j),
                      j);
}

int nw_certificates_verify_many(const nw_committee* committee, const nw_certificates* certs,
                                const uint8_t* z16, int32_t* status_out, uint64_t* index_out) {
  nw_job* j = nullptr;
  return run_blocking(
      nw_submit_certificates_verify_many(committee, certs, z16, status_out, index_out, &j), j);
}

int nw_headers_verify_many(const nw_committee* committee, const nw_certificates* headers,
                           int32_t* status_out, uint64_t* index_out) {
  nw_job* j = nullptr;
  return run_blocking(nw_submit_headers_verify_many(committee, headers, status_out, index_out, &j),
                      j);
}

int nw_votes_verify_many(const nw_committee* committee, const uint8_t* ids,
                         const uint64_t* rounds, const uint8_t* origins,
                         const uint8_t* authors, const uint8_t* sigs, size_t n,
                         int32_t* status_out) {
  nw_job* j = nullptr;
  return run_blocking(nw_submit_votes_verify_many(committee, ids, rounds, origins, authors, sigs,
                                                  n, status_out, &j),
                      j);
}

}  // extern "C"
