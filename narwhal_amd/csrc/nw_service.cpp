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
// Structure: one service per committee. A request reserves its place in the open batch of
// its kind under the service mutex (offsets and its callback; no allocation in the steady
// state: batches are recycled) and copies its signatures, keys and header bytes there after
// releasing it, so producers copy in parallel (an N = 50 certificate is ~3.4 KB; at 10^6 per
// second copying under the mutex was the service's limit). A batch taken for submission
// waits for its writers to finish. A flusher thread submits a batch as ONE device job
// (nw_submit_*: the committee-aware pipeline with its key tables kept on the device) when it
// holds max_items units, max_delay has passed since its first request, or no job is in
// flight (an idle device gains nothing from a bigger batch, so a lone request goes at once
// and batches grow only while the device is busy); a completer thread
// waits for the jobs in submission order and calls every request's verdict callback. At most
// max_inflight jobs are queued on the device at once (backpressure on the flusher; requests
// keep accumulating into the next, larger batch meanwhile, which is what keeps the device
// efficient under load).
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
#include <thread>
#include <vector>

#include "narwhal_amd.h"
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

// A byte array that grows only while nobody writes into it (under the mutex, no writers):
// requests reserve ranges under the mutex and fill them after releasing it. Not
// zero-initialised (std::vector::resize writes every byte twice).
struct Buf {
  uint8_t* p = nullptr;
  size_t n = 0, cap = 0;
  Buf() = default;
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
  ~Buf() { free(p); }
  bool fits(size_t k) const { return n + k <= cap; }
  bool grow(size_t k) {
    const size_t c = std::max<size_t>({2 * cap, n + k, 4096});
    void* q = realloc(p, c);
    if (!q) return false;
    p = static_cast<uint8_t*>(q);
    cap = c;
    return true;
  }
  uint8_t* take(size_t k) {
    uint8_t* d = p + n;
    n += k;
    return d;
  }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const uint8_t* data() const { return p; }
};

// One kind's requests in the SoA form of its nw_submit_* entry point.
struct Batch {
  Kind kind;
  size_t units = 0;
  Clock::time_point first;
  std::vector<Req> reqs;
  std::atomic<int> writers{0};   // requests copying into the Bufs outside the mutex
  // Header / Certificate (nw_certificates)
  Buf header_bytes;
  std::vector<uint64_t> header_offsets{0};
  std::vector<uint32_t> payload_counts;
  Buf ids, header_sigs;
  std::vector<uint64_t> vote_offsets{0};
  Buf vote_pks, vote_sigs;
  // Vote (nw_submit_votes_verify_many): ids and signatures reuse ids / header_sigs
  std::vector<uint64_t> rounds;
  Buf origins, authors;
  // Signature::verify / verify_batch: digests (n x 32), keys, signatures, batch offsets
  Buf digests, pks, sigs;
  std::vector<uint64_t> batch_offsets{0};
  // outputs and the job
  std::vector<int32_t> status;
  std::vector<uint64_t> index;
  nw_job* job = nullptr;
  int rc = 0;

  explicit Batch(Kind k) : kind(k) {}
  void clear() {
    units = 0;
    reqs.clear();
    for (Buf* b : {&header_bytes, &ids, &header_sigs, &vote_pks, &vote_sigs, &origins, &authors,
                   &digests, &pks, &sigs})
      b->n = 0;
    header_offsets.assign(1, 0);
    payload_counts.clear();
    vote_offsets.assign(1, 0);
    rounds.clear();
    batch_offsets.assign(1, 0);
    job = nullptr;
    rc = 0;
  }
  // a batch taken for submission: every request that reserved a range has filled it
  void wait_writers() const {
    while (writers.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }
};

// One input range of a request: len bytes from src into the batch's Buf `buf`.
struct Piece {
  Buf Batch::*buf;
  const void* src;
  size_t len;
};
constexpr int kMaxPieces = 5;

uint8_t g_dummy[64];

// The completer polls a job this long before it blocks on it.
constexpr int kSpinUs = 2000;
// Largest batch (units) a request's own thread submits on an idle device (a few
// certificates): anything bigger is the flusher's.
constexpr size_t kInlineUnits = 256;
template <class T>
const T* nz(const std::vector<T>& v) {
  return v.empty() ? reinterpret_cast<const T*>(g_dummy) : v.data();
}
const uint8_t* nz(const Buf& v) { return v.empty() ? g_dummy : v.data(); }

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
  std::condition_variable cv_flush;     // flusher: new request / flush / stop
  std::condition_variable cv_inflight;  // completer: a job was submitted
  std::condition_variable cv_space;     // flusher: in-flight count dropped
  std::condition_variable cv_idle;      // drain: requests completed
  std::unique_ptr<Batch> open[K_COUNT];
  std::vector<std::unique_ptr<Batch>> spare[K_COUNT];
  std::deque<std::unique_ptr<Batch>> inflight;
  bool force = false, stop = false, flusher_done = false;
  uint64_t accepted = 0, completed = 0, jobs = 0;
  // NW_SERVICE_DEBUG: seconds the flusher spent submitting / blocked on max_inflight, the
  // completer waiting for jobs / running callbacks (printed at destroy)
  double t_submit = 0, t_backpressure = 0, t_wait = 0, t_callbacks = 0;
  size_t open_jobs = 0;   // submitted (or being submitted), callbacks not yet delivered
  size_t submitting = 0;  // submits in progress outside the lock
  bool inline_submit = true;   // NW_SERVICE_INLINE=0: only the flusher submits
  std::thread flusher, completer;

  // Adds one request to its kind's open batch; 0 or NW_E_*. Under the mutex: room in the
  // batch's Bufs for the request's pieces (growing them waits until no request is still
  // copying into the batch), its callback, and the small per-request fields (fill: offsets,
  // counts, rounds); then, with the mutex released, the pieces are copied in.
  // On an idle device (no job in flight, none being submitted) the caller's thread submits
  // the oldest batch itself: the request reaches the device without waking the flusher
  // thread (a futex wake-up is tens of microseconds, a third of a small job).
  template <class Fill>
  int add(Kind k, size_t units, nw_verdict_fn fn, void* arg, const Piece* pc, int npc,
          Fill fill) {
    if (!fn) return set_err(NW_E_INVALID_ARG, "null verdict callback");
    std::unique_lock<std::mutex> lk(m, std::defer_lock);
    lock_spin(lk);
    if (stop) return set_err(NW_E_INVALID_ARG, "service is shutting down");
    for (;;) {
      Batch& b = *open[k];
      bool fits = true;
      for (int i = 0; i < npc; ++i) fits = fits && (b.*pc[i].buf).fits(pc[i].len);
      if (fits) break;
      if (b.writers.load(std::memory_order_acquire) != 0) {
        lk.unlock();   // let them finish; the batch may be flushed meanwhile
        b.wait_writers();
        lk.lock();
        continue;
      }
      for (int i = 0; i < npc; ++i)
        if (!(b.*pc[i].buf).fits(pc[i].len) && !(b.*pc[i].buf).grow(pc[i].len))
          return set_err(NW_E_OUT_OF_MEMORY, "service batch");
    }
    Batch& b = *open[k];
    const bool first_req = b.reqs.empty();
    if (first_req) b.first = Clock::now();
    uint8_t* dst[kMaxPieces];
    for (int i = 0; i < npc; ++i) dst[i] = (b.*pc[i].buf).take(pc[i].len);
    fill(b);
    b.reqs.push_back({fn, arg});
    b.writers.fetch_add(1, std::memory_order_relaxed);
    const size_t before = b.units;
    b.units += units;
    ++accepted;
    // Only the first request of a batch goes from the caller's thread (a quiet service): a
    // batch that filled while the device was busy is the flusher's (the completer wakes it
    // when the device goes idle), since a submit costs the caller ~0.05-0.1 ms and callers
    // that stall under load fall behind their own arrivals
    const bool idle = inline_submit && first_req && open_jobs == 0 && submitting == 0 &&
                      inflight.size() < max_inflight && b.units <= kInlineUnits;
    // wake the flusher to arm its timer (first request) or because the batch just filled
    const bool wake = !idle && (first_req || (before < max_items && b.units >= max_items));
    lk.unlock();
    if (wake) cv_flush.notify_one();
    for (int i = 0; i < npc; ++i)
      if (pc[i].len) memcpy(dst[i], pc[i].src, pc[i].len);
    b.writers.fetch_sub(1, std::memory_order_release);
    if (!idle) return 0;
    lock_spin(lk);
    if (open_jobs == 0 && submitting == 0 && inflight.size() < max_inflight && !stop) {
      // every non-empty batch is ready on an idle device: the oldest goes, as in the flusher
      // (taking always the caller's own kind let a flood of one kind starve the others)
      int pick = -1;
      for (int j = 0; j < K_COUNT; ++j)
        if (!open[j]->reqs.empty() && (pick < 0 || open[j]->first < open[pick]->first))
          pick = j;
      if (pick >= 0 && open[pick]->units > kInlineUnits) pick = -1;   // the flusher's
      std::unique_ptr<Batch> fresh = pick < 0 ? nullptr : take_spare(static_cast<Kind>(pick));
      if (fresh) {
        std::unique_ptr<Batch> own = std::move(open[pick]);
        open[pick] = std::move(fresh);
        launch(lk, std::move(own));
        if (open[k]->reqs.empty()) return 0;
      }
    }
    lk.unlock();
    cv_flush.notify_one();   // whatever is left waits for the flusher
    return 0;
  }

  // The service mutex is held for well under a microsecond at a time; a producer that finds
  // it taken spins briefly instead of sleeping in the kernel (a futex wait and wake-up costs
  // tens of microseconds, and at 10^6 requests per second producers collide constantly).
  static void lock_spin(std::unique_lock<std::mutex>& lk) {
    for (int i = 0; i < 256; ++i) {
      if (lk.try_lock()) return;
      __builtin_ia32_pause();
    }
    lk.lock();
  }

  // Submits b as one device job outside the lock (held on entry and on return) and queues it
  // for the completer. The flusher and idle-device requests both come through here.
  void launch(std::unique_lock<std::mutex>& lk, std::unique_ptr<Batch> b) {
    ++open_jobs;
    ++submitting;
    lk.unlock();
    b->wait_writers();
    const Clock::time_point s0 = Clock::now();
    // the service's device choice, also when a producer's thread submits (restored after)
    const int prev = nw_get_device();
    if (prev != device) nw_set_device(device);
    b->rc = submit(*b);
    if (prev != device) nw_set_device(prev);
    const double ds = std::chrono::duration<double>(Clock::now() - s0).count();
    lk.lock();
    --submitting;
    t_submit += ds;
    ++jobs;
    inflight.push_back(std::move(b));
    cv_inflight.notify_one();
  }

  std::unique_ptr<Batch> take_spare(Kind k) {
    if (!spare[k].empty()) {
      std::unique_ptr<Batch> b = std::move(spare[k].back());
      spare[k].pop_back();
      return b;
    }
    return std::unique_ptr<Batch>(new (std::nothrow) Batch(k));
  }

  // Flusher thread: one device job per batch.
  int submit(Batch& b) {
    const size_t n = b.reqs.size();
    b.status.assign(n, 0);
    b.index.assign(n, 0);
    switch (b.kind) {
      case K_CERT:
      case K_HEADER: {
        nw_certificates c{};
        c.n = n;
        c.header_bytes = nz(b.header_bytes);
        c.header_offsets = b.header_offsets.data();
        c.payload_counts = b.payload_counts.data();
        c.ids = b.ids.data();
        c.header_sigs = b.header_sigs.data();
        if (b.kind == K_CERT) {
          c.vote_offsets = b.vote_offsets.data();
          c.vote_pks = nz(b.vote_pks);
          c.vote_sigs = nz(b.vote_sigs);
          return nw_submit_certificates_verify_many(&com, &c, nullptr, b.status.data(),
                                                    b.index.data(), &b.job);
        }
        return nw_submit_headers_verify_many(&com, &c, b.status.data(), b.index.data(), &b.job);
      }
      case K_VOTE:
        return nw_submit_votes_verify_many(&com, b.ids.data(), b.rounds.data(), b.origins.data(),
                                           b.authors.data(), b.header_sigs.data(), n,
                                           b.status.data(), &b.job);
      case K_STRICT:
        return nw_submit_verify_strict(b.digests.data(), 32, b.pks.data(), b.sigs.data(), n,
                                       b.status.data(), nullptr, &b.job);
      case K_BATCH:
        return nw_submit_verify_batch_many(b.digests.data(), nz(b.pks), nz(b.sigs),
                                           b.batch_offsets.data(), n, nullptr, b.status.data(),
                                           b.index.data(), &b.job);
      default:
        return set_err(NW_E_INVALID_ARG, "bad request kind");
    }
  }

  void flusher_main() {
    nw_set_device(device);
    std::unique_lock<std::mutex> lk(m);
    for (;;) {
      const Clock::time_point now = Clock::now();
      Clock::time_point wake = Clock::time_point::max();
      int pick = -1;
      for (int k = 0; k < K_COUNT; ++k) {
        const Batch& b = *open[k];
        if (b.reqs.empty()) continue;
        // flush: stopping / forced, full, its delay is over, or the device is idle (no job
        // in flight: waiting would only add latency, nothing is gained by a bigger batch).
        // Among the ready kinds the one whose first request is oldest goes first, so a
        // saturating certificate load cannot starve a trickle of votes or headers (the
        // primary's Core interleaves all three, primary/src/core.rs:349-411).
        if (stop || force || b.units >= max_items || now >= b.first + delay ||
            open_jobs == 0) {
          if (pick < 0 || b.first < open[pick]->first) pick = k;
        } else if (b.first + delay < wake) {
          wake = b.first + delay;
        }
      }
      if (pick < 0) {
        force = false;
        if (stop) break;
        if (wake == Clock::time_point::max())
          cv_flush.wait(lk);
        else
          cv_flush.wait_until(lk, wake);
        continue;
      }
      // backpressure: at most max_inflight jobs queued; the open batch keeps growing
      if (inflight.size() >= max_inflight) {
        const Clock::time_point w0 = Clock::now();
        cv_space.wait(lk);
        t_backpressure += std::chrono::duration<double>(Clock::now() - w0).count();
        continue;
      }
      std::unique_ptr<Batch> fresh = take_spare(static_cast<Kind>(pick));
      if (!fresh) {   // out of memory: submit nothing new until something completes
        cv_space.wait_for(lk, std::chrono::milliseconds(1));
        continue;
      }
      std::unique_ptr<Batch> b = std::move(open[pick]);
      open[pick] = std::move(fresh);
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
      const size_t n = b->reqs.size();
      for (size_t i = 0; i < n; ++i)
        b->reqs[i].fn(b->reqs[i].arg, rc ? rc : b->status[i], rc ? 0 : b->index[i]);
      const Clock::time_point c1 = Clock::now();
      lk.lock();
      std::unique_ptr<Batch> own = std::move(inflight.front());
      inflight.pop_front();
      cv_space.notify_one();
      t_wait += std::chrono::duration<double>(c0 - w0).count();
      t_callbacks += std::chrono::duration<double>(c1 - c0).count();
      completed += n;
      if (--open_jobs == 0) cv_flush.notify_one();   // device idle: flush what has queued
      own->clear();
      spare[own->kind].push_back(std::move(own));
      cv_idle.notify_all();
    }
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
  for (int k = 0; k < K_COUNT; ++k) {
    s->open[k].reset(new (std::nothrow) Batch(static_cast<Kind>(k)));
    if (!s->open[k]) {
      delete s;
      return set_err(NW_E_OUT_OF_MEMORY, "service allocation");
    }
  }
  try {
    s->flusher = std::thread([s] { s->flusher_main(); });
    s->completer = std::thread([s] { s->completer_main(); });
  } catch (...) {
    {
      std::lock_guard<std::mutex> g(s->m);
      s->stop = true;
    }
    s->cv_flush.notify_all();
    if (s->flusher.joinable()) s->flusher.join();
    if (s->completer.joinable()) s->completer.join();
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
  const Piece pc[] = {{&Batch::header_bytes, header_bytes, header_len},
                      {&Batch::ids, id, 32},
                      {&Batch::header_sigs, header_sig, 64},
                      {&Batch::vote_pks, vote_pks, 32 * nvotes},
                      {&Batch::vote_sigs, vote_sigs, 64 * nvotes}};
  return s->add(K_CERT, 1 + nvotes, fn, arg, pc, 5, [&](Batch& b) {
    b.header_offsets.push_back(b.header_bytes.size());
    b.payload_counts.push_back(payload_count);
    b.vote_offsets.push_back(b.vote_offsets.back() + nvotes);
  });
}

int nw_service_header(nw_service* s, const uint8_t* header_bytes, size_t header_len,
                      uint32_t payload_count, const uint8_t* id, const uint8_t* sig,
                      nw_verdict_fn fn, void* arg) {
  int rc = need_committee(s);
  if (!rc) rc = check_header(header_bytes, header_len, payload_count, id, sig);
  if (rc) return rc;
  const Piece pc[] = {{&Batch::header_bytes, header_bytes, header_len},
                      {&Batch::ids, id, 32},
                      {&Batch::header_sigs, sig, 64}};
  return s->add(K_HEADER, 1, fn, arg, pc, 3, [&](Batch& b) {
    b.header_offsets.push_back(b.header_bytes.size());
    b.payload_counts.push_back(payload_count);
  });
}

int nw_service_vote(nw_service* s, const uint8_t* id, uint64_t round, const uint8_t* origin,
                    const uint8_t* author, const uint8_t* sig, nw_verdict_fn fn, void* arg) {
  int rc = need_committee(s);
  if (rc) return rc;
  if (!id || !origin || !author || !sig) return set_err(NW_E_INVALID_ARG, "null pointer");
  const Piece pc[] = {{&Batch::ids, id, 32},
                      {&Batch::origins, origin, 32},
                      {&Batch::authors, author, 32},
                      {&Batch::header_sigs, sig, 64}};
  return s->add(K_VOTE, 1, fn, arg, pc, 4, [&](Batch& b) { b.rounds.push_back(round); });
}

int nw_service_verify(nw_service* s, const uint8_t* digest, const uint8_t* pk,
                      const uint8_t* sig, nw_verdict_fn fn, void* arg) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  if (!digest || !pk || !sig) return set_err(NW_E_INVALID_ARG, "null pointer");
  const Piece pc[] = {{&Batch::digests, digest, 32}, {&Batch::pks, pk, 32},
                      {&Batch::sigs, sig, 64}};
  return s->add(K_STRICT, 1, fn, arg, pc, 3, [](Batch&) {});
}

int nw_service_verify_batch(nw_service* s, const uint8_t* digest, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, nw_verdict_fn fn, void* arg) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  if (!digest || (n && (!pks || !sigs))) return set_err(NW_E_INVALID_ARG, "null pointer");
  const Piece pc[] = {{&Batch::digests, digest, 32}, {&Batch::pks, pks, 32 * n},
                      {&Batch::sigs, sigs, 64 * n}};
  return s->add(K_BATCH, n ? n : 1, fn, arg, pc, 3, [&](Batch& b) {
    b.batch_offsets.push_back(b.batch_offsets.back() + n);
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
  const uint64_t target = s->accepted;
  s->force = true;
  s->cv_flush.notify_one();
  s->cv_idle.wait(lk, [&] { return s->completed >= target; });
  return 0;
}

int nw_service_stats(nw_service* s, uint64_t* requests, uint64_t* jobs) {
  if (!s) return set_err(NW_E_INVALID_ARG, "null service");
  std::lock_guard<std::mutex> g(s->m);
  if (requests) *requests = s->accepted;
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
  if (getenv("NW_SERVICE_DEBUG"))
    fprintf(stderr,
            "[narwhal_amd] service: %llu requests, %llu jobs; flusher submit %.3f s, "
            "backpressure %.3f s; completer wait %.3f s, callbacks %.3f s\n",
            (unsigned long long)s->accepted, (unsigned long long)s->jobs, s->t_submit,
            s->t_backpressure, s->t_wait, s->t_callbacks);
  delete s;
}

}  // extern "C"
