// nw_service.cpp — native aggregation service (nw_service_*): single Header / Vote /
// Certificate / Signature::verify / Signature::verify_batch requests coalesced into device
// jobs.
//
// Why: Narwhal's primary verifies one message at a time on its single Core task
// (primary/src/core.rs:306-346: sanitize_header / sanitize_vote / sanitize_certificate call
// Header/Vote/Certificate::verify inline), and a certificate carries only 3..67 signatures,
// far too little work for a GPU launch. crypto::SignatureService (crypto/src/lib.rs:222-250)
// is the reference's own shape for this: requests over a channel, replies over oneshot
// channels. A Rust crypto-gpu crate binds these entry points and completes a oneshot
// channel from the verdict callback, so its tokio tasks never block.
//
// Structure: one service per committee, one open batch per request kind, in the SoA form of
// that kind's nw_submit_* entry point, in fixed-capacity arrays.
//   ingest   lock-free: a request reserves its place with one compare-and-swap on the
//            batch's cursor (request count, header bytes, votes packed in one word), then
//            copies its signatures, keys, header bytes, offsets and callback into the
//            reserved ranges. At 10^6 N = 50 certificates per second (~3.4 GB/s of requests
//            from several threads) a mutex around that bookkeeping made producers queue on
//            one lock and fall behind their arrivals, in runs that stayed slow once behind.
//            The mutex is taken only by a batch's first request (to wake the flusher, or to
//            submit the batch itself when a job slot is free), when the arrays are full (the
//            batch is sealed for submission and a spare of the same room opened: no
//            allocation on the producers' path unless one request alone needs more room), and
//            when a batch reaches max_items units (sealed too: a job holds about max_items).
//   flusher  submits a batch as ONE device job (the committee-aware pipeline, or the
//            one-launch small-job kernel) when it is sealed, max_delay has passed since its
//            first request, or fewer than eager_jobs (2) jobs are open (a device with a free
//            slot gains nothing from a bigger batch: small-job launches only read the shared
//            tables and run side by side, so a lone request goes at once and batches grow
//            only while the device is busy). Taking an open batch seals its cursor (later reservations fail
//            and go to the next batch) and waits for the requests still copying into it.
//            Kinds with ready batches take turns, so a flood of certificates cannot starve
//            a trickle of votes.
//   completer waits for the jobs in submission order and calls every request's verdict
//            callback. At most max_inflight jobs are on the device at once (backpressure on
//            the flusher; requests keep accumulating into the next, larger batch meanwhile,
//            which is what keeps the device efficient under load).
//   hedge    (nw_service_set_hedge; on by default) a request whose verdict has not arrived
//            `deadline` after its batch's first request is verified on the host as well
//            (nw_host.cpp: the kernels' own arithmetic compiled for the CPU, same statuses
//            and indices), and whichever verdict comes first is delivered, exactly once (one
//            atomic flag per request). A hedger thread looks every deadline / 4 at the batches
//            on the device or being submitted, and at batches still waiting for a job slot;
//            `threads` host threads answer them, oldest first, racing the device. A batch
//            still waiting is taken for the host alone (never submitted) only while the host
//            queue holds fewer than `max_queued` units, so the host never owes more than it
//            finishes quickly; a device stall under heavy load costs at most `threads` cores
//            and the rest waits for the device as before. Why: the primary verifies on its one
//            Core task (primary/src/core.rs:338-346), so a device job that stalls for 10-40 ms
//            (the box's host-memory access episodes) stalls the primary, while
//            one certificate costs a host core well under a millisecond.
// Batches are recycled; a batch is never freed before the service (a request that loaded a
// batch just before it was taken only touches its cursor and writer count, and fails).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "narwhal_amd.h"
#include "nw_host.h"
#include "nw_runtime.h"

namespace {

using nw::rt::set_err;
using Clock = std::chrono::steady_clock;

enum Kind { K_CERT = 0, K_HEADER, K_VOTE, K_STRICT, K_BATCH, K_COUNT };

struct Req {
  nw_verdict_fn fn;
  void* arg;
};

template <class T>
void append(std::vector<T>& v, const void* src, size_t count) {
  const size_t o = v.size();
  v.resize(o + count);
  if (count) memcpy(v.data() + o, src, count * sizeof(T));
}

// Cursor of a batch: requests (bits 0..19), var1 = header bytes (bits 20..43), var2 = votes
// or verify_batch items (bits 44..62), sealed (bit 63).
constexpr uint64_t kReqBits = 20, kVar1Bits = 24, kVar2Bits = 19;
constexpr uint64_t kMaxReq = (1ull << kReqBits) - 1, kMaxVar1 = (1ull << kVar1Bits) - 1,
                   kMaxVar2 = (1ull << kVar2Bits) - 1;
constexpr uint64_t kSealed = 1ull << 63;
inline uint64_t c_req(uint64_t c) { return c & kMaxReq; }
inline uint64_t c_v1(uint64_t c) { return (c >> kReqBits) & kMaxVar1; }
inline uint64_t c_v2(uint64_t c) { return (c >> (kReqBits + kVar1Bits)) & kMaxVar2; }
inline uint64_t c_pack(uint64_t r, uint64_t v1, uint64_t v2) {
  return r | (v1 << kReqBits) | (v2 << (kReqBits + kVar1Bits));
}

// A fixed-capacity array (not zeroed: allocating one must not stall the producers waiting
// for a fresh batch; its pages fault in on the first copies instead).
struct Arr {
  uint8_t* p = nullptr;
  size_t cap = 0;
  Arr() = default;
  Arr(const Arr&) = delete;
  Arr& operator=(const Arr&) = delete;
  ~Arr() { free(p); }
  bool ensure(size_t c) {
    if (cap >= c) return true;
    free(p);
    p = static_cast<uint8_t*>(malloc(c));
    cap = p ? c : 0;
    return p != nullptr;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

// Room of a batch: requests, header bytes, votes / items.
struct Caps {
  uint64_t req, v1, v2;
};

// One kind's requests in the SoA form of its nw_submit_* entry point.
struct Batch {
  Kind kind;
  std::atomic<uint64_t> cursor{kSealed};   // sealed until installed as the open batch
  std::atomic<int> writers{0};             // requests copying into the batch
  std::atomic<int64_t> first_ns{0};        // arrival of request 0 (0: not yet stamped)
  Caps caps{0, 0, 0};
  uint64_t n = 0, nv1 = 0, nv2 = 0;        // final counts (from the cursor when taken)
  int64_t t_taken = 0, t_sub0 = 0, t_sub1 = 0;   // NW_SERVICE_DEBUG: taken, submit start / end
  int how = 0;                                     // NW_SERVICE_DEBUG: see JobRec
  Arr reqs;
  // Header / Certificate (nw_certificates)
  Arr header_bytes, header_offsets, payload_counts, ids, header_sigs, vote_offsets, vote_pks,
      vote_sigs;
  // Vote: ids and signatures reuse ids / header_sigs
  Arr rounds, origins, authors;
  // Signature::verify / verify_batch: digests (n x 32), keys, signatures, batch offsets
  Arr digests, pks, sigs, batch_offsets;
  // outputs and the job
  std::vector<int32_t> status;
  std::vector<uint64_t> index;
  nw_job* job = nullptr;
  int rc = 0;
  // hedge: answered[i] = 1 once request i's callback has been claimed (device or host)
  std::vector<uint8_t> answered;
  bool hedged = false;             // queued for the hedge threads (guarded by the hedge mutex)
  bool host_only = false;          // taken for the host alone, never submitted
  std::atomic<size_t> hnext{0};    // next request a hedge thread claims
  std::atomic<size_t> hdone{0};    // requests the hedge threads have finished with
  std::atomic<int> hrefs{0};       // hedge threads inside the batch

  explicit Batch(Kind k) : kind(k) {}

  // the callback of request i is ours to call (exactly one caller wins)
  bool claim(size_t i) { return __atomic_exchange_n(&answered[i], (uint8_t)1, __ATOMIC_ACQ_REL) == 0; }
  bool is_answered(size_t i) const { return __atomic_load_n(&answered[i], __ATOMIC_ACQUIRE) != 0; }
  // fresh per-request flags once the final count n is known (before anyone can claim)
  void reset_answers() {
    answered.assign(n, 0);
    hedged = host_only = false;
    hnext.store(0, std::memory_order_relaxed);
    hdone.store(0, std::memory_order_relaxed);
    hrefs.store(0, std::memory_order_relaxed);
  }

  // arrays for caps c (only the ones this kind uses)
  bool reserve(const Caps& c) {
    const uint64_t r = c.req, r1 = c.req + 1;
    bool ok = reqs.ensure(sizeof(Req) * r);
    switch (kind) {
      case K_CERT:
        ok = ok && vote_offsets.ensure(8 * r1) && vote_pks.ensure(32 * c.v2) &&
             vote_sigs.ensure(64 * c.v2);
        [[fallthrough]];
      case K_HEADER:
        ok = ok && header_bytes.ensure(c.v1) && header_offsets.ensure(8 * r1) &&
             payload_counts.ensure(4 * r) && ids.ensure(32 * r) && header_sigs.ensure(64 * r);
        break;
      case K_VOTE:
        ok = ok && ids.ensure(32 * r) && rounds.ensure(8 * r) && origins.ensure(32 * r) &&
             authors.ensure(32 * r) && header_sigs.ensure(64 * r);
        break;
      case K_STRICT:
        ok = ok && digests.ensure(32 * r) && pks.ensure(32 * r) && sigs.ensure(64 * r);
        break;
      case K_BATCH:
        ok = ok && digests.ensure(32 * r) && batch_offsets.ensure(8 * r1) &&
             pks.ensure(32 * c.v2) && sigs.ensure(64 * c.v2);
        break;
      default:
        break;
    }
    if (!ok) return false;
    caps = c;
    return true;
  }
  // an empty open batch (under the service mutex; the cursor is published last)
  void open_empty() {
    n = nv1 = nv2 = 0;
    job = nullptr;
    rc = 0;
    first_ns.store(0, std::memory_order_relaxed);
    if (header_offsets.p) header_offsets.as<uint64_t>()[0] = 0;
    if (vote_offsets.p) vote_offsets.as<uint64_t>()[0] = 0;
    if (batch_offsets.p) batch_offsets.as<uint64_t>()[0] = 0;
    cursor.store(0, std::memory_order_release);
  }
  // a batch taken for submission: every request that reserved a range has filled it
  void wait_writers() const {
    while (writers.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }
  uint64_t units() const { return units_of(kind, n, nv2); }
  static uint64_t units_of(Kind k, uint64_t r, uint64_t v2) {
    return (k == K_CERT || k == K_BATCH) ? r + v2 : r;
  }
};

uint8_t g_dummy[64];

// The completer polls a job this long before it blocks on it.
constexpr int kSpinUs = 2000;
// Largest batch (units) a request's own thread submits on an idle device (a few
// certificates): anything bigger is the flusher's.
constexpr size_t kInlineUnits = 256;
const uint8_t* nz(const Arr& a, uint64_t count) { return count ? a.p : g_dummy; }
template <class T>
const T* nz(const std::vector<T>& v) {
  return v.empty() ? reinterpret_cast<const T*>(g_dummy) : v.data();
}
// Timed condition waits. -DNW_SERVICE_SYSTEM_CLOCK_WAIT (the ThreadSanitizer build of
// tools/service_stress): on the system clock, because libstdc++ waits on the steady clock
// with pthread_cond_clockwait, which this image's libtsan does not intercept (it then misses
// the mutex release inside the wait and reports races under the mutex).
void wait_ns(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, int64_t ns) {
#ifdef NW_SERVICE_SYSTEM_CLOCK_WAIT
  cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::nanoseconds(ns));
#else
  cv.wait_for(lk, std::chrono::nanoseconds(ns));
#endif
}
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch())
      .count();
}

}  // namespace

struct nw_service {
  int device = 0;   // the creating thread's nw_set_device value (NW_ALL_DEVICES = fan out)
  bool has_committee = false;
  std::vector<uint8_t> com_pks;
  std::vector<uint32_t> com_stakes;
  std::vector<uint64_t> com_wo;
  std::vector<uint32_t> com_wi;
  nw_committee com{};
  size_t max_items = 1 << 16;
  Clock::duration delay{};
  size_t max_inflight = 4;

  std::mutex m;
  std::condition_variable cv_flush;     // flusher: new batch / full / flush / stop
  std::condition_variable cv_inflight;  // completer: a job was submitted
  std::condition_variable cv_space;     // flusher: in-flight count dropped
  std::condition_variable cv_idle;      // drain: requests completed
  // open[k] (owned, guarded by m) and cur[k] (its pointer, read lock-free by producers)
  std::unique_ptr<Batch> open[K_COUNT];
  std::atomic<Batch*> cur[K_COUNT];
  Caps caps[K_COUNT];                   // room of the next batch of each kind (grows)
  // per kind: batches sealed full (no room, or max_items reached) waiting for the flusher
  std::deque<std::unique_ptr<Batch>> sealed[K_COUNT];
  size_t nsealed = 0;
  int last_kind = K_COUNT - 1;          // the flusher's round-robin position
  std::vector<std::unique_ptr<Batch>> spare[K_COUNT];
  std::deque<std::unique_ptr<Batch>> inflight;
  std::atomic<bool> stop{false};
  bool force = false, flusher_done = false;
  std::atomic<uint64_t> accepted{0};
  std::atomic<uint64_t> completed{0};   // callbacks delivered (completer and hedge threads)
  uint64_t jobs = 0;
  // NW_SERVICE_DEBUG: seconds the flusher spent submitting / blocked on max_inflight, the
  // completer waiting for jobs / running callbacks, caller-thread submits and full batches
  // (printed at destroy)
  double t_submit = 0, t_backpressure = 0, t_wait = 0, t_callbacks = 0;
  uint64_t n_inline = 0, n_full = 0;
  // NW_SERVICE_DEBUG: per job, microseconds from its first request to: taken, submit start,
  // submitted, done seen by the completer, callbacks delivered (medians printed at destroy)
  bool debug = false;
  std::vector<float> d_taken, d_sub0, d_sub1, d_done, d_cb;
  // NW_SERVICE_DEBUG=<path containing '/'>: one CSV row per job written there at destroy
  // (kind, requests, votes, how it was submitted, ns timestamps), the per-job timeline the
  // medians above summarise
  std::string debug_path;
  struct JobRec {
    int kind, how;   // how: 0 flusher (timer / eager), 1 caller's thread, 2 sealed full
    uint64_t n, nv2;
    int64_t first, taken, sub0, sub1, done, cb;
  };
  std::vector<JobRec> d_jobs;
  size_t open_jobs = 0;   // submitted (or being submitted), callbacks not yet delivered
  size_t submitting = 0;  // submits in progress outside the lock
  bool inline_submit = true;   // NW_SERVICE_INLINE=0: only the flusher submits
  // A batch goes at once (no max_delay wait) while fewer than eager_jobs jobs are open: one
  // small-job launch only reads the shared tables, so a second one runs beside the first
  // instead of after it (NW_SERVICE_EAGER; 1 = only on an idle device). A/B with the
  // service leg (profiles/r04b/service_eager_ab.txt): p50 at N = 4 and 10^5..10^6 certs/s
  // 0.09-0.10 vs 0.11-0.12 ms, N = 50 at 10^4 0.16 vs 0.22 ms; N = 50 at 10^5 0.26 vs
  // 0.18 ms (smaller jobs, each paying the header digest's serial chain)
  size_t eager_jobs = 2;
  std::thread flusher, completer;

  // ---- hedge (nw_service_set_hedge) ----
  int64_t hedge_ns = 1000000;          // deadline after a batch's first request; 0 = off
  uint32_t hedge_threads = 6;
  uint64_t hedge_max_queued = 512;     // units a batch taken for the host alone may join
  // NW_SERVICE_TEST_DELAY_US (test hook): the completer holds every device verdict until this
  // long after its batch's first request, so the hedge answers first
  int64_t test_delay_ns = 0;
  nw::host::Committee* hc = nullptr;   // the committee's host tables (built in the background)
  std::atomic<bool> hc_ready{false};
  std::thread hc_builder;
  std::mutex hm;                       // hedge queue (lock order: m before hm)
  std::condition_variable cv_hw;       // hedge threads: work queued / stop
  std::condition_variable cv_hedger;   // hedger: stop
  std::deque<Batch*> hq;               // batches the hedge threads answer, oldest first
  std::vector<std::unique_ptr<Batch>> hostonly;   // taken for the host alone (owned here)
  std::vector<std::unique_ptr<Batch>> retired;    // device-done hedged batches still entered
  std::vector<Batch*> submitting_b;    // batches inside launch() (under m)
  bool hworkers_stop = false;          // under hm
  std::atomic<bool> hedger_stop{false};
  std::thread hedger;
  std::vector<std::thread> hworkers;
  std::atomic<uint64_t> n_hedged{0}, n_host_first{0}, n_host_only{0};

  // One request of kind k with v1 header bytes and v2 votes / items: reserve its ranges in
  // the open batch (write(b, i, v1_off, v2_off) fills them), then wake the flusher or submit.
  template <class Write>
  int add(Kind k, uint64_t v1, uint64_t v2, nw_verdict_fn fn, void* arg, Write write) {
    if (!fn) return set_err(NW_E_INVALID_ARG, "null verdict callback");
    if (v1 > kMaxVar1 / 2 || v2 > kMaxVar2 / 2)
      return set_err(NW_E_INVALID_ARG, "request too large for the service");
    Batch* b;
    uint64_t c;
    for (;;) {
      if (stop.load(std::memory_order_acquire))
        return set_err(NW_E_INVALID_ARG, "service is shutting down");
      b = cur[k].load(std::memory_order_acquire);
      b->writers.fetch_add(1, std::memory_order_seq_cst);
      c = b->cursor.load(std::memory_order_seq_cst);
      bool retry = false, room = true;
      for (;;) {
        if (c & kSealed) {
          retry = true;
          break;
        }
        const uint64_t r = c_req(c), a = c_v1(c), z = c_v2(c);
        if (r + 1 > b->caps.req || a + v1 > b->caps.v1 || z + v2 > b->caps.v2) {
          room = false;
          break;
        }
        if (b->cursor.compare_exchange_weak(c, c_pack(r + 1, a + v1, z + v2),
                                            std::memory_order_seq_cst))
          break;
      }
      if (!retry && room) break;
      b->writers.fetch_sub(1, std::memory_order_release);
      if (retry) {   // taken meanwhile: the next batch is (about to be) installed
        std::this_thread::yield();
        continue;
      }
      const int rc = make_room(k, b, v1, v2);   // full: seal it, install a bigger one
      if (rc) return rc;
    }
    const uint64_t i = c_req(c);
    write(*b, i, c_v1(c), c_v2(c));
    b->reqs.as<Req>()[i] = {fn, arg};
    if (i == 0) b->first_ns.store(now_ns(), std::memory_order_relaxed);
    const uint64_t before = Batch::units_of(k, i, c_v2(c));
    const uint64_t after = Batch::units_of(k, i + 1, c_v2(c) + v2);
    b->writers.fetch_sub(1, std::memory_order_release);
    accepted.fetch_add(1, std::memory_order_relaxed);
    if (i == 0) return first_request(k, b);
    if (before < max_items && after >= max_items) seal_full(k, b);   // the batch is done
    return 0;
  }

  // b reached max_items: if it is still the open batch, seal it for the flusher and open the
  // next (a job never holds much more than max_items units, however fast requests arrive).
  void seal_full(Kind k, Batch* b) {
    std::unique_lock<std::mutex> lk(m);
    if (open[k].get() == b) {
      std::unique_ptr<Batch> old = take_open(k);
      if (old) {
        ++n_full;
        old->how = 2;
        sealed[k].push_back(std::move(old));
        ++nsealed;
      }
    }
    lk.unlock();
    cv_flush.notify_one();
  }

  // The first request of batch b: the flusher arms its timer for it, or, with a job slot
  // free (fewer than eager_jobs open, none being submitted), the caller's thread submits the oldest
  // non-empty batch itself — a lone request reaches the device without waking the flusher
  // (a futex wake-up is tens of microseconds, a third of a small job).
  int first_request(Kind k, Batch* b) {
    std::unique_lock<std::mutex> lk(m);
    (void)k;
    (void)b;
    if (inline_submit && open_jobs < eager_jobs && submitting == 0 &&
        inflight.size() < max_inflight &&
        nsealed == 0 && !stop.load(std::memory_order_relaxed)) {
      int pick = -1;
      int64_t oldest = 0;
      for (int j = 0; j < K_COUNT; ++j) {
        const uint64_t cj = open[j]->cursor.load(std::memory_order_acquire);
        if (c_req(cj) == 0) continue;
        int64_t f = open[j]->first_ns.load(std::memory_order_relaxed);
        if (f == 0) f = now_ns();
        if (pick < 0 || f < oldest) {
          pick = j;
          oldest = f;
        }
      }
      if (pick >= 0) {
        const uint64_t cp = open[pick]->cursor.load(std::memory_order_acquire);
        if (Batch::units_of(static_cast<Kind>(pick), c_req(cp), c_v2(cp)) <= kInlineUnits) {
          std::unique_ptr<Batch> own = take_open(static_cast<Kind>(pick));
          if (own) {
            ++n_inline;
            own->how = 1;
            launch(lk, std::move(own));
            return 0;
          }
        }
      }
    }
    lk.unlock();
    cv_flush.notify_one();
    return 0;
  }

  // b (kind k) has no room for a request of v1 / v2: if it is still the open batch, seal it
  // as full (the flusher submits it next) and install the next batch — of the same room
  // (a spare, no allocation) unless the request alone would not fit an empty batch, in
  // which case the kind's room grows to hold it.
  int make_room(Kind k, Batch* b, uint64_t v1, uint64_t v2) {
    std::unique_lock<std::mutex> lk(m);
    if (open[k].get() != b) return 0;   // someone else did (retry on the new batch)
    Caps& c = caps[k];
    if (1 > c.req) c.req = 64;
    if (v1 > c.v1) c.v1 = std::min<uint64_t>(kMaxVar1, std::max<uint64_t>(2 * c.v1, 2 * v1 + 4096));
    if (v2 > c.v2) c.v2 = std::min<uint64_t>(kMaxVar2, std::max<uint64_t>(2 * c.v2, 2 * v2 + 64));
    std::unique_ptr<Batch> old = take_open(k);
    if (!old) return set_err(NW_E_OUT_OF_MEMORY, "service batch");
    if (old->n == 0) {   // empty and too small for this request: recycle it
      spare[k].push_back(std::move(old));
      return 0;
    }
    ++n_full;
    old->how = 2;
    sealed[k].push_back(std::move(old));
    ++nsealed;
    lk.unlock();
    cv_flush.notify_one();
    return 0;
  }

  // Seals the open batch of kind k and installs a fresh one (under m); nullptr when no
  // fresh batch could be made (the open batch stays). The sealed batch's final counts are
  // taken from its cursor; its writers may still be copying (launch waits for them).
  std::unique_ptr<Batch> take_open(Kind k) {
    std::unique_ptr<Batch> fresh = take_spare(k);
    if (!fresh) return nullptr;
    std::unique_ptr<Batch> b = std::move(open[k]);
    const uint64_t c = b->cursor.fetch_or(kSealed, std::memory_order_seq_cst);
    b->n = c_req(c);
    b->nv1 = c_v1(c);
    b->nv2 = c_v2(c);
    fresh->open_empty();
    open[k] = std::move(fresh);
    cur[k].store(open[k].get(), std::memory_order_release);
    return b;
  }

  std::unique_ptr<Batch> take_spare(Kind k) {
    std::unique_ptr<Batch> b;
    if (!spare[k].empty()) {
      b = std::move(spare[k].back());
      spare[k].pop_back();
    } else {
      b.reset(new (std::nothrow) Batch(k));
      if (!b) return b;
    }
    if (!b->reserve(caps[k])) {
      spare[k].push_back(std::move(b));
      return nullptr;
    }
    return b;
  }

  // Submits b as one device job outside the lock (held on entry and on return) and queues it
  // for the completer. The flusher and idle-device requests both come through here.
  void launch(std::unique_lock<std::mutex>& lk, std::unique_ptr<Batch> b) {
    ++open_jobs;
    ++submitting;
    b->reset_answers();
    Batch* const raw = b.get();
    submitting_b.push_back(raw);   // the hedger may hedge it while the submit is slow
    lk.unlock();
    if (debug) b->t_taken = now_ns();
    b->wait_writers();
    const Clock::time_point s0 = Clock::now();
    if (debug) b->t_sub0 = now_ns();
    // the service's device choice, also when a producer's thread submits (restored after)
    const int prev = nw_get_device();
    if (prev != device) nw_set_device(device);
    b->rc = submit(*b);
    if (prev != device) nw_set_device(prev);
    const double ds = std::chrono::duration<double>(Clock::now() - s0).count();
    if (debug) b->t_sub1 = now_ns();
    lk.lock();
    submitting_b.erase(std::find(submitting_b.begin(), submitting_b.end(), raw));
    --submitting;
    t_submit += ds;
    ++jobs;
    inflight.push_back(std::move(b));
    cv_inflight.notify_one();
  }

  int submit(Batch& b) {
    const size_t n = b.n;
    b.status.assign(n, 0);
    b.index.assign(n, 0);
    switch (b.kind) {
      case K_CERT:
      case K_HEADER: {
        nw_certificates c{};
        c.n = n;
        c.header_bytes = nz(b.header_bytes, b.nv1);
        c.header_offsets = b.header_offsets.as<uint64_t>();
        c.payload_counts = b.payload_counts.as<uint32_t>();
        c.ids = b.ids.p;
        c.header_sigs = b.header_sigs.p;
        if (b.kind == K_CERT) {
          c.vote_offsets = b.vote_offsets.as<uint64_t>();
          c.vote_pks = nz(b.vote_pks, b.nv2);
          c.vote_sigs = nz(b.vote_sigs, b.nv2);
          return nw_submit_certificates_verify_many(&com, &c, nullptr, b.status.data(),
                                                    b.index.data(), &b.job);
        }
        return nw_submit_headers_verify_many(&com, &c, b.status.data(), b.index.data(), &b.job);
      }
      case K_VOTE:
        return nw_submit_votes_verify_many(&com, b.ids.p, b.rounds.as<uint64_t>(), b.origins.p,
                                           b.authors.p, b.header_sigs.p, n, b.status.data(),
                                           &b.job);
      case K_STRICT:
        return nw_submit_verify_strict(b.digests.p, 32, b.pks.p, b.sigs.p, n, b.status.data(),
                                       nullptr, &b.job);
      case K_BATCH:
        return nw_submit_verify_batch_many(b.digests.p, nz(b.pks, b.nv2), nz(b.sigs, b.nv2),
                                           b.batch_offsets.as<uint64_t>(), n, nullptr,
                                           b.status.data(), b.index.data(), &b.job);
      default:
        return set_err(NW_E_INVALID_ARG, "bad request kind");
    }
  }

  // Flusher thread: one device job per batch.
  void flusher_main() {
    nw_set_device(device);
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
      const int64_t tnow = now_ns();
      const int64_t dns = std::chrono::duration_cast<std::chrono::nanoseconds>(delay).count();
      int64_t wake = INT64_MAX;
      int pick = -1;
      // Per kind: a sealed batch (full, or at max_items) is ready; an open one when its
      // delay is over, the device is idle, or on flush / stop. Kinds with ready work take
      // turns (round-robin): under a flood of one kind (sealed batches queueing faster than
      // the device takes them) a trickle of another still goes within a job or two — the
      // primary's Core interleaves all three (primary/src/core.rs:349-411).
      bool ready[K_COUNT] = {};
      for (int k = 0; k < K_COUNT; ++k) {
        if (!sealed[k].empty()) {
          ready[k] = true;
          continue;
        }
        const Batch& b = *open[k];
        const uint64_t c = b.cursor.load(std::memory_order_acquire);
        if (c_req(c) == 0) continue;
        int64_t f = b.first_ns.load(std::memory_order_relaxed);
        if (f == 0) f = tnow;
        ready[k] = stop.load(std::memory_order_relaxed) || force ||
                   Batch::units_of(static_cast<Kind>(k), c_req(c), c_v2(c)) >= max_items ||
                   tnow >= f + dns || open_jobs < eager_jobs;
        if (!ready[k] && f + dns < wake) wake = f + dns;
      }
      for (int d = 1; d <= K_COUNT && pick < 0; ++d) {
        const int k = (last_kind + d) % K_COUNT;
        if (ready[k]) pick = k;
      }
      if (pick < 0) {
        force = false;
        if (stop.load(std::memory_order_relaxed)) break;
        if (wake == INT64_MAX)
          cv_flush.wait(lk);
        else
          wait_ns(cv_flush, lk, wake - tnow);
        continue;
      }
      // backpressure: at most max_inflight jobs queued; the open batch keeps growing
      if (inflight.size() >= max_inflight) {
        const Clock::time_point w0 = Clock::now();
        cv_space.wait(lk);
        t_backpressure += std::chrono::duration<double>(Clock::now() - w0).count();
        continue;
      }
      std::unique_ptr<Batch> b;
      if (!sealed[pick].empty()) {
        b = std::move(sealed[pick].front());
        sealed[pick].pop_front();
        --nsealed;
      } else {
        b = take_open(static_cast<Kind>(pick));
        if (!b) {   // out of memory: submit nothing new until something completes
          wait_ns(cv_space, lk, 1000000);
          continue;
        }
      }
      last_kind = pick;
      launch(lk, std::move(b));
    }
    flusher_done = true;
    cv_inflight.notify_all();
  }

  void completer_main() {
    nw_set_device(device);
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
      cv_inflight.wait(lk, [&] { return !inflight.empty() || flusher_done; });
      if (inflight.empty()) break;
      // the job stays counted in `inflight` until it has finished (max_inflight jobs on the
      // device at most); deque::push_back keeps references to existing elements valid
      Batch* const b = inflight.front().get();
      lk.unlock();
      int rc = b->rc;
      const Clock::time_point w0 = Clock::now();
      if (test_delay_ns) {   // test hook: a late device verdict
        const int64_t until = b->first_ns.load(std::memory_order_relaxed) + test_delay_ns;
        while (now_ns() < until) std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
      if (b->job) {
        // poll first (a small job finishes in ~0.1 ms; a blocking event wait adds the
        // runtime's wake-up latency to every verdict), then block
        if (!rc) {
          int done = 0;
          const Clock::time_point spin_end = w0 + std::chrono::microseconds(kSpinUs);
          while (!(done = nw_job_poll(b->job)) && Clock::now() < spin_end)
            std::this_thread::yield();
          rc = done < 0 ? done : done ? 0 : nw_job_wait(b->job);
        }
        nw_job_release(b->job);
        b->job = nullptr;
      }
      const Clock::time_point c0 = Clock::now();
      const int64_t tdone = debug ? now_ns() : 0;
      const size_t n = b->n;
      const Req* reqs = b->reqs.as<Req>();
      uint64_t mine = 0;
      for (size_t i = 0; i < n; ++i)
        if (b->claim(i)) {   // not already answered by the hedge
          reqs[i].fn(reqs[i].arg, rc ? rc : b->status[i], rc ? 0 : b->index[i]);
          ++mine;
        }
      completed.fetch_add(mine, std::memory_order_acq_rel);
      const Clock::time_point c1 = Clock::now();
      if (debug && b->n && d_done.size() < (1u << 22)) {
        const int64_t f = b->first_ns.load(std::memory_order_relaxed);
        const int64_t tcb = now_ns();
        auto us = [f](int64_t t) { return (float)((double)(t - f) * 1e-3); };
        d_taken.push_back(us(b->t_taken));
        d_sub0.push_back(us(b->t_sub0));
        d_sub1.push_back(us(b->t_sub1));
        d_done.push_back(us(tdone));
        d_cb.push_back(us(tcb));
        if (!debug_path.empty())
          d_jobs.push_back({b->kind, b->how, b->n, b->nv2, f, b->t_taken, b->t_sub0, b->t_sub1,
                            tdone, tcb});
      }
      lk.lock();
      std::unique_ptr<Batch> own = std::move(inflight.front());
      inflight.pop_front();
      cv_space.notify_one();
      t_wait += std::chrono::duration<double>(c0 - w0).count();
      t_callbacks += std::chrono::duration<double>(c1 - c0).count();
      // a job slot freed below eager_jobs: flush what has queued
      if (--open_jobs < eager_jobs) cv_flush.notify_one();
      own->how = 0;
      recycle(std::move(own));
      cv_idle.notify_all();
    }
  }

  // ---- hedge --------------------------------------------------------------------------
  // A finished device batch back to the spares (under m), unless hedge threads are still
  // inside it: then the hedger recycles it once they have left.
  void recycle(std::unique_ptr<Batch> b) {
    if (b->hedged) {
      std::lock_guard<std::mutex> g(hm);
      auto it = std::find(hq.begin(), hq.end(), b.get());
      if (it != hq.end()) {
        hq.erase(it);
      }
      if (b->hrefs.load(std::memory_order_acquire) > 0) {
        retired.push_back(std::move(b));
        return;
      }
    }
    spare[b->kind].push_back(std::move(b));
  }

  // Queue b for the hedge threads (under m); own != nullptr: b was taken before submission
  // and is owned by the hedge from now on, and must fit the budget (the host answers it
  // alone, so it must not queue more than the hedge threads finish quickly). A late batch on
  // the device is always queued: the threads work oldest first and the device races them.
  bool queue_hedge(std::unique_ptr<Batch>* own, Batch* b) {
    std::lock_guard<std::mutex> g(hm);
    if (hworkers.empty() || (own && host_queued() + b->units() > hedge_max_queued)) return false;
    b->hedged = true;
    hq.push_back(b);
    if (own) {
      b->host_only = true;
      hostonly.push_back(std::move(*own));
      n_host_only.fetch_add(1, std::memory_order_relaxed);
    }
    n_hedged.fetch_add(b->n, std::memory_order_relaxed);
    cv_hw.notify_all();
    return true;
  }

  // units of the hedge queue not yet taken by a hedge thread (under hm)
  uint64_t host_queued() const {
    uint64_t u = 0;
    for (const Batch* b : hq) {
      const size_t next = std::min(b->hnext.load(std::memory_order_relaxed), b->n);
      u += Batch::units_of(b->kind, b->n - next, b->n ? b->nv2 * (b->n - next) / b->n : 0);
    }
    return u;
  }

  bool hedgeable(const Batch& b, int64_t now) const {
    if (b.hedged || b.n == 0) return false;
    const int64_t f = b.first_ns.load(std::memory_order_relaxed);
    if (f == 0 || now - f < hedge_ns) return false;
    // messages need the committee's host tables (built at create, in the background)
    return b.kind == K_STRICT || b.kind == K_BATCH || hc_ready.load(std::memory_order_acquire);
  }

  void hedger_main() {
    std::unique_lock<std::mutex> lk(m);
    while (!hedger_stop.load(std::memory_order_acquire)) {
      const int64_t tick = std::max<int64_t>(50000, std::min<int64_t>(250000, hedge_ns / 4));
      wait_ns(cv_hedger, lk, hedge_ns ? tick : 2000000);
      if (hedger_stop.load(std::memory_order_acquire)) break;
      // hedged batches the hedge threads have left: back to the spares
      {
        std::lock_guard<std::mutex> g(hm);
        for (size_t i = 0; i < retired.size();) {
          if (retired[i]->hrefs.load(std::memory_order_acquire) == 0) {
            spare[retired[i]->kind].push_back(std::move(retired[i]));
            retired[i] = std::move(retired.back());
            retired.pop_back();
          } else {
            ++i;
          }
        }
        for (size_t i = 0; i < hostonly.size();) {
          Batch& b = *hostonly[i];
          if (b.hdone.load(std::memory_order_acquire) == b.n &&
              b.hrefs.load(std::memory_order_acquire) == 0) {
            std::unique_ptr<Batch> own = std::move(hostonly[i]);
            hostonly[i] = std::move(hostonly.back());
            hostonly.pop_back();
            spare[own->kind].push_back(std::move(own));
          } else {
            ++i;
          }
        }
      }
      if (!hedge_ns) continue;
      const int64_t now = now_ns();
      // batches on the device, or inside a submit, whose verdicts are late
      for (auto& u : inflight)
        if (u->rc == 0 && hedgeable(*u, now)) (void)queue_hedge(nullptr, u.get());
      for (Batch* b : submitting_b)
        if (hedgeable(*b, now)) (void)queue_hedge(nullptr, b);
      // batches still waiting for a job slot (backpressure): the host takes them whole
      for (int k = 0; k < K_COUNT; ++k) {
        while (!sealed[k].empty() && hedgeable(*sealed[k].front(), now)) {
          std::unique_ptr<Batch> own = std::move(sealed[k].front());
          Batch* b = own.get();
          b->reset_answers();
          if (!queue_hedge(&own, b)) {
            sealed[k].front() = std::move(own);
            break;
          }
          sealed[k].pop_front();
          --nsealed;
        }
        Batch& ob = *open[k];
        const uint64_t c = ob.cursor.load(std::memory_order_acquire);
        if (c_req(c) == 0 || (c & kSealed)) continue;
        const int64_t f = ob.first_ns.load(std::memory_order_relaxed);
        {
          std::lock_guard<std::mutex> g(hm);
          if (f == 0 || now - f < hedge_ns || hworkers.empty() ||
              host_queued() + Batch::units_of(static_cast<Kind>(k), c_req(c), c_v2(c)) >
                  hedge_max_queued)
            continue;
        }
        if (k != K_STRICT && k != K_BATCH && !hc_ready.load(std::memory_order_acquire)) continue;
        std::unique_ptr<Batch> own = take_open(static_cast<Kind>(k));
        if (!own) continue;
        Batch* b = own.get();
        b->reset_answers();
        if (!queue_hedge(&own, b)) {   // grew past the budget meanwhile: the flusher's again
          sealed[k].push_front(std::move(own));
          ++nsealed;
          cv_flush.notify_one();
        }
      }
    }
  }

  // Request i of b on the host (nw_host.cpp): status and index as the device job returns them.
  int answer(const Batch& b, size_t i, uint64_t* ix) {
    *ix = 0;
    switch (b.kind) {
      case K_CERT:
      case K_HEADER: {
        const uint64_t* ho = b.header_offsets.as<uint64_t>();
        const uint8_t* hb = b.header_bytes.p + ho[i];
        const size_t hl = ho[i + 1] - ho[i];
        const uint32_t np = b.payload_counts.as<uint32_t>()[i];
        if (b.kind == K_HEADER)
          return nw::host::header_verify(*hc, hb, hl, np, b.ids.p + 32 * i, b.header_sigs.p + 64 * i, ix);
        const uint64_t* vo = b.vote_offsets.as<uint64_t>();
        return nw::host::certificate_verify(*hc, hb, hl, np, b.ids.p + 32 * i,
                                            b.header_sigs.p + 64 * i, b.vote_pks.p + 32 * vo[i],
                                            b.vote_sigs.p + 64 * vo[i], vo[i + 1] - vo[i], nullptr,
                                            ix);
      }
      case K_VOTE:
        return nw::host::vote_verify(*hc, b.ids.p + 32 * i, b.rounds.as<uint64_t>()[i],
                                     b.origins.p + 32 * i, b.authors.p + 32 * i,
                                     b.header_sigs.p + 64 * i);
      case K_STRICT:
        return nw::host::verify_strict(b.digests.p + 32 * i, b.pks.p + 32 * i, b.sigs.p + 64 * i);
      case K_BATCH: {
        const uint64_t* bo = b.batch_offsets.as<uint64_t>();
        return nw::host::verify_batch(b.digests.p + 32 * i, b.pks.p + 32 * bo[i],
                                      b.sigs.p + 64 * bo[i], bo[i + 1] - bo[i], nullptr,
                                      hc_ready.load(std::memory_order_acquire) ? hc : nullptr, ix);
      }
      default:
        return NW_E_INVALID_ARG;
    }
  }

  void hedge_worker() {
    for (;;) {
      Batch* b = nullptr;
      size_t i = 0;
      {
        std::unique_lock<std::mutex> g(hm);
        for (;;) {
          if (!hq.empty()) {
            b = hq.front();
            i = b->hnext.fetch_add(1, std::memory_order_acq_rel);
            if (i < b->n) {
              b->hrefs.fetch_add(1, std::memory_order_acq_rel);
              break;
            }
            hq.pop_front();   // every request claimed: the batch leaves the queue
                continue;
          }
          if (hworkers_stop) return;
          cv_hw.wait(g);
        }
      }
      b->wait_writers();
      if (!b->is_answered(i)) {
        uint64_t ix = 0;
        const int st = answer(*b, i, &ix);
        // a host error (no CSPRNG) is left to the device, unless there is no device job
        if ((st >= 0 || b->host_only) && b->claim(i)) {
          const Req& r = b->reqs.as<Req>()[i];
          r.fn(r.arg, st, st >= 0 ? ix : 0);
          n_host_first.fetch_add(1, std::memory_order_relaxed);
          completed.fetch_add(1, std::memory_order_acq_rel);
          { std::lock_guard<std::mutex> g(m); }   // no lost wake-up for a drain
          cv_idle.notify_all();
        }
      }
      b->hdone.fetch_add(1, std::memory_order_acq_rel);
      b->hrefs.fetch_sub(1, std::memory_order_acq_rel);
    }
  }

  // (Re)starts the hedge threads with the current parameters; the old ones first answer
  // every request already queued.
  void restart_hedge() {
    stop_hedge();
    {
      std::lock_guard<std::mutex> g(hm);
      hworkers_stop = false;
    }
    hedger_stop.store(false, std::memory_order_release);
    if (!hedge_ns || !hedge_threads) return;
    for (uint32_t t = 0; t < hedge_threads; ++t) hworkers.emplace_back([this] { hedge_worker(); });
    hedger = std::thread([this] { hedger_main(); });
  }
  void stop_hedge() {
    hedger_stop.store(true, std::memory_order_release);
    {
      std::lock_guard<std::mutex> g(m);
    }
    cv_hedger.notify_all();
    if (hedger.joinable()) hedger.join();
    {
      std::lock_guard<std::mutex> g(hm);
      hworkers_stop = true;
    }
    cv_hw.notify_all();
    for (auto& t : hworkers) t.join();
    std::lock_guard<std::mutex> g(hm);
    hworkers.clear();
  }
};

extern "C" {

int nw_service_create(const nw_committee* committee, size_t max_items, uint32_t max_delay_us,
                      size_t max_inflight, nw_service** out) {
  if (!out) return set_err(NW_E_INVALID_ARG, "null service pointer");
  *out = nullptr;
  int rc = nw::rt::ensure_init();
  if (rc) return rc;
  if (committee) {
    rc = nw::rt::check_committee(committee);
    if (rc) return rc;
  }
  nw_service* s = new (std::nothrow) nw_service;
  if (!s) return set_err(NW_E_OUT_OF_MEMORY, "service allocation");
  s->device = nw_get_device();
  s->max_items = max_items ? max_items : 1;
  s->delay = std::chrono::duration_cast<Clock::duration>(std::chrono::microseconds(max_delay_us));
  s->max_inflight = max_inflight ? max_inflight : 1;
  if (const char* e = getenv("NW_SERVICE_INLINE")) s->inline_submit = atoi(e) != 0;
  s->debug = getenv("NW_SERVICE_DEBUG") != nullptr;
  if (s->debug && strchr(getenv("NW_SERVICE_DEBUG"), '/')) s->debug_path = getenv("NW_SERVICE_DEBUG");
  if (const char* e = getenv("NW_SERVICE_EAGER")) s->eager_jobs = std::max(1, atoi(e));
  if (const char* e = getenv("NW_SERVICE_TEST_DELAY_US")) s->test_delay_ns = 1000ll * atoll(e);
  // NW_SERVICE_HEDGE_US / _THREADS / _QUEUED: the hedge's defaults (nw_service_set_hedge)
  if (const char* e = getenv("NW_SERVICE_HEDGE_US")) s->hedge_ns = 1000ll * atoll(e);
  if (const char* e = getenv("NW_SERVICE_HEDGE_THREADS")) s->hedge_threads = (uint32_t)atoi(e);
  if (const char* e = getenv("NW_SERVICE_HEDGE_QUEUED")) s->hedge_max_queued = strtoull(e, nullptr, 10);
  if (committee) {
    const size_t na = committee->nauth, nwk = na ? committee->worker_offsets[na] : 0;
    s->has_committee = true;
    append(s->com_pks, committee->pks, 32 * na);
    append(s->com_stakes, committee->stakes, na);
    if (na) append(s->com_wo, committee->worker_offsets, na + 1);
    else s->com_wo.assign(1, 0);
    append(s->com_wi, committee->worker_ids, nwk);
    s->com.nauth = na;
    s->com.pks = nz(s->com_pks);
    s->com.stakes = nz(s->com_stakes);
    s->com.worker_offsets = s->com_wo.data();
    s->com.worker_ids = nz(s->com_wi);
  }
  // Initial room per kind (~11 MB for certificates, ~7 MB for verify_batch, ~4 MB for
  // headers, < 1 MB for the others): a 10^6-per-second N = 50 certificate load makes
  // batches of ~250 certificates (~9k votes, ~280 KB of header bytes), so batches grow only
  // under a backlog
  const uint64_t mi = s->max_items;
  const Caps init[K_COUNT] = {
      {std::min<uint64_t>(mi + 1, 4096), 1 << 22, std::min<uint64_t>(mi, 1 << 16)},   // cert
      {std::min<uint64_t>(mi + 1, 4096), 1 << 22, 0},                                 // header
      {std::min<uint64_t>(mi + 1, 4096), 0, 0},                                       // vote
      {std::min<uint64_t>(mi + 1, 4096), 0, 0},                                       // strict
      {std::min<uint64_t>(mi + 1, 1024), 0, std::min<uint64_t>(mi, 1 << 16)}};        // batch
  // the jobs its first burst needs (max_inflight queued + one being submitted + one
  // submitting from a caller's thread), made now rather than on the flusher's path
  if (s->device >= 0) {
    int dev = 0;
    if (nw::rt::select_device(&dev) == 0)
      (void)nw::rt::jobs_prewarm(dev, (int)std::min<size_t>(s->max_inflight + 2, 16), 4 << 20,
                                 4 << 20);
  }
  for (int k = 0; k < K_COUNT; ++k) {
    s->caps[k] = init[k];
    std::unique_ptr<Batch> b = s->take_spare(static_cast<Kind>(k));
    if (!b) {
      delete s;
      return set_err(NW_E_OUT_OF_MEMORY, "service allocation");
    }
    b->open_empty();
    s->open[k] = std::move(b);
    s->cur[k].store(s->open[k].get(), std::memory_order_release);
  }
  try {
    s->flusher = std::thread([s] { s->flusher_main(); });
    s->completer = std::thread([s] { s->completer_main(); });
    // the committee's host tables for the hedge (~2-5 ms of a core per key), off this thread
    if (s->has_committee)
      s->hc_builder = std::thread([s] {
        s->hc = nw::host::committee_new(&s->com);
        s->hc_ready.store(s->hc != nullptr, std::memory_order_release);
      });
    s->restart_hedge();
  } catch (...) {
    {
      std::lock_guard<std::mutex> g(s->m);
      s->stop = true;
    }
    s->cv_flush.notify_all();
    if (s->flusher.joinable()) s->flusher.join();
    if (s->completer.joinable()) s->completer.join();
    s->stop_hedge();
    if (s->hc_builder.joinable()) s->hc_builder.join();
    nw::host::committee_free(s->hc);
    delete s;
    return set_err(NW_E_OUT_OF_MEMORY, "service threads");
  }
  *out = s;
  return 0;
}

static int need_committee(nw_service* s) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  if (!s->has_committee) return set_err(NW_E_INVALID_ARG, "service has no committee");
  return 0;
}

static int check_header(const uint8_t* header_bytes, size_t header_len, uint32_t payload_count,
                        const uint8_t* id, const uint8_t* sig) {
  if (!header_bytes || !id || !sig) return set_err(NW_E_INVALID_ARG, "null pointer");
  const uint64_t fixed = 40 + 36 * (uint64_t)payload_count;
  if (header_len < fixed || (header_len - fixed) % 32 != 0)
    return set_err(NW_E_INVALID_ARG, "header bytes do not match payload_count");
  return 0;
}

int nw_service_certificate(nw_service* s, const uint8_t* header_bytes, size_t header_len,
                           uint32_t payload_count, const uint8_t* id, const uint8_t* header_sig,
                           const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t nvotes,
                           nw_verdict_fn fn, void* arg) {
  int rc = need_committee(s);
  if (!rc) rc = check_header(header_bytes, header_len, payload_count, id, header_sig);
  if (rc) return rc;
  if (nvotes && (!vote_pks || !vote_sigs)) return set_err(NW_E_INVALID_ARG, "null votes");
  return s->add(K_CERT, header_len, nvotes, fn, arg,
                [&](Batch& b, uint64_t i, uint64_t h, uint64_t v) {
                  memcpy(b.header_bytes.p + h, header_bytes, header_len);
                  b.header_offsets.as<uint64_t>()[i + 1] = h + header_len;
                  b.payload_counts.as<uint32_t>()[i] = payload_count;
                  memcpy(b.ids.p + 32 * i, id, 32);
                  memcpy(b.header_sigs.p + 64 * i, header_sig, 64);
                  if (nvotes) {
                    memcpy(b.vote_pks.p + 32 * v, vote_pks, 32 * nvotes);
                    memcpy(b.vote_sigs.p + 64 * v, vote_sigs, 64 * nvotes);
                  }
                  b.vote_offsets.as<uint64_t>()[i + 1] = v + nvotes;
                });
}

int nw_service_header(nw_service* s, const uint8_t* header_bytes, size_t header_len,
                      uint32_t payload_count, const uint8_t* id, const uint8_t* sig,
                      nw_verdict_fn fn, void* arg) {
  int rc = need_committee(s);
  if (!rc) rc = check_header(header_bytes, header_len, payload_count, id, sig);
  if (rc) return rc;
  return s->add(K_HEADER, header_len, 0, fn, arg,
                [&](Batch& b, uint64_t i, uint64_t h, uint64_t) {
                  memcpy(b.header_bytes.p + h, header_bytes, header_len);
                  b.header_offsets.as<uint64_t>()[i + 1] = h + header_len;
                  b.payload_counts.as<uint32_t>()[i] = payload_count;
                  memcpy(b.ids.p + 32 * i, id, 32);
                  memcpy(b.header_sigs.p + 64 * i, sig, 64);
                });
}

int nw_service_vote(nw_service* s, const uint8_t* id, uint64_t round, const uint8_t* origin,
                    const uint8_t* author, const uint8_t* sig, nw_verdict_fn fn, void* arg) {
  int rc = need_committee(s);
  if (rc) return rc;
  if (!id || !origin || !author || !sig) return set_err(NW_E_INVALID_ARG, "null pointer");
  return s->add(K_VOTE, 0, 0, fn, arg, [&](Batch& b, uint64_t i, uint64_t, uint64_t) {
    memcpy(b.ids.p + 32 * i, id, 32);
    b.rounds.as<uint64_t>()[i] = round;
    memcpy(b.origins.p + 32 * i, origin, 32);
    memcpy(b.authors.p + 32 * i, author, 32);
    memcpy(b.header_sigs.p + 64 * i, sig, 64);
  });
}

int nw_service_verify(nw_service* s, const uint8_t* digest, const uint8_t* pk,
                      const uint8_t* sig, nw_verdict_fn fn, void* arg) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  if (!digest || !pk || !sig) return set_err(NW_E_INVALID_ARG, "null pointer");
  return s->add(K_STRICT, 0, 0, fn, arg, [&](Batch& b, uint64_t i, uint64_t, uint64_t) {
    memcpy(b.digests.p + 32 * i, digest, 32);
    memcpy(b.pks.p + 32 * i, pk, 32);
    memcpy(b.sigs.p + 64 * i, sig, 64);
  });
}

int nw_service_verify_batch(nw_service* s, const uint8_t* digest, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, nw_verdict_fn fn, void* arg) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  if (!digest || (n && (!pks || !sigs))) return set_err(NW_E_INVALID_ARG, "null pointer");
  return s->add(K_BATCH, 0, n, fn, arg, [&](Batch& b, uint64_t i, uint64_t, uint64_t v) {
    memcpy(b.digests.p + 32 * i, digest, 32);
    if (n) {
      memcpy(b.pks.p + 32 * v, pks, 32 * n);
      memcpy(b.sigs.p + 64 * v, sigs, 64 * n);
    }
    b.batch_offsets.as<uint64_t>()[i + 1] = v + n;
  });
}

int nw_service_flush(nw_service* s) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  {
    std::lock_guard<std::mutex> g(s->m);
    s->force = true;
  }
  s->cv_flush.notify_one();
  return 0;
}

int nw_service_drain(nw_service* s) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  std::unique_lock<std::mutex> lk(s->m);
  const uint64_t target = s->accepted.load(std::memory_order_acquire);
  s->force = true;
  s->cv_flush.notify_one();
  s->cv_idle.wait(lk, [&] { return s->completed >= target; });
  return 0;
}

int nw_service_set_hedge(nw_service* s, uint32_t deadline_us, uint32_t threads,
                         uint64_t max_queued) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  if (threads > 64) return set_err(NW_E_INVALID_ARG, "at most 64 hedge threads");
  s->stop_hedge();
  {
    std::lock_guard<std::mutex> g(s->m);
    s->hedge_ns = 1000ll * deadline_us;
    s->hedge_threads = threads;
    s->hedge_max_queued = max_queued;
  }
  try {
    s->restart_hedge();
  } catch (...) {
    return set_err(NW_E_OUT_OF_MEMORY, "hedge threads");
  }
  return 0;
}

int nw_service_hedge_stats(nw_service* s, uint64_t* hedged, uint64_t* host_first,
                           uint64_t* host_only_batches, int* host_ready) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  if (hedged) *hedged = s->n_hedged.load();
  if (host_first) *host_first = s->n_host_first.load();
  if (host_only_batches) *host_only_batches = s->n_host_only.load();
  if (host_ready) *host_ready = s->hc_ready.load(std::memory_order_acquire) ? 1 : 0;
  return 0;
}

int nw_service_stats(nw_service* s, uint64_t* requests, uint64_t* jobs) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  std::lock_guard<std::mutex> g(s->m);
  if (requests) *requests = s->accepted.load(std::memory_order_acquire);
  if (jobs) *jobs = s->jobs;
  return 0;
}

void nw_service_destroy(nw_service* s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(s->m);
    s->stop = true;
  }
  s->cv_flush.notify_all();
  s->cv_space.notify_all();
  s->flusher.join();
  s->completer.join();
  // the hedge answers whatever it took for the host alone, then stops
  s->stop_hedge();
  if (s->hc_builder.joinable()) s->hc_builder.join();
  nw::host::committee_free(s->hc);
  s->hc = nullptr;
  if (getenv("NW_SERVICE_DEBUG"))
    fprintf(stderr,
            "[narwhal_amd] service: %llu requests, %llu jobs (%llu from callers' threads, "
            "%llu full batches); submit %.3f s, backpressure %.3f s; completer wait %.3f s, "
            "callbacks %.3f s\n",
            (unsigned long long)s->accepted.load(), (unsigned long long)s->jobs,
            (unsigned long long)s->n_inline, (unsigned long long)s->n_full, s->t_submit,
            s->t_backpressure, s->t_wait, s->t_callbacks);
  if (s->debug && !s->d_done.empty()) {
    auto med = [](std::vector<float>& v) {
      std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
      return v[v.size() / 2];
    };
    fprintf(stderr,
            "[narwhal_amd] service job timeline, median us after the job's first request: "
            "taken %.1f, submit start %.1f, submitted %.1f, done seen %.1f, callbacks %.1f "
            "(%zu jobs)\n",
            med(s->d_taken), med(s->d_sub0), med(s->d_sub1), med(s->d_done), med(s->d_cb),
            s->d_done.size());
  }
  if (!s->debug_path.empty() && !s->d_jobs.empty()) {
    // one file per service: <path>.<first job's first-request ns>
    char name[4096];
    snprintf(name, sizeof name, "%s.%lld.csv", s->debug_path.c_str(),
             (long long)s->d_jobs.front().first);
    if (FILE* f = fopen(name, "w")) {
      fprintf(f, "kind,how,n,votes,first_ns,taken_ns,sub0_ns,sub1_ns,done_ns,cb_ns\n");
      for (const auto& j : s->d_jobs)
        fprintf(f, "%d,%d,%llu,%llu,%lld,%lld,%lld,%lld,%lld,%lld\n", j.kind, j.how,
                (unsigned long long)j.n, (unsigned long long)j.nv2, (long long)j.first,
                (long long)j.taken, (long long)j.sub0, (long long)j.sub1, (long long)j.done,
                (long long)j.cb);
      fclose(f);
    }
    // the job staging growths of the process so far (steady-clock ns, as first_ns above)
    std::vector<uint64_t> g(4 * 4096);
    const size_t ng = nw::rt::job_growth_log(g.data(), 4096);
    snprintf(name, sizeof name, "%s.%lld.grow.csv", s->debug_path.c_str(),
             (long long)s->d_jobs.front().first);
    if (FILE* f = fopen(name, "w")) {
      fprintf(f, "t_ns,capacity,us,kind\n");
      for (size_t i = 0; i < ng && i < 4096; ++i)
        fprintf(f, "%llu,%llu,%llu,%llu\n", (unsigned long long)g[4 * i],
                (unsigned long long)g[4 * i + 1], (unsigned long long)g[4 * i + 2],
                (unsigned long long)g[4 * i + 3]);
      fclose(f);
    }
  }
  delete s;
}

}  // extern "C"
