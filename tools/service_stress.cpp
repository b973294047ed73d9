// service_stress.cpp — CPU harness for the aggregation service's host logic
// (narwhal_amd/csrc/nw_service.cpp: lock-free ingest, batch sealing and growth, flusher,
// completer), with the device entry points replaced by test doubles: every nw_submit_* here
// checks the batch's structure-of-arrays (offsets start at 0, are monotone and end at the
// array totals) and answers each request with a fingerprint of exactly the bytes that
// request supplied; jobs complete after a random delay. Producer threads submit random
// certificates, headers, votes, strict and verify_batch requests (sizes from empty to large
// enough to force batch growth), and every verdict must equal the fingerprint the producer
// computed from its own inputs, with exactly one callback per request.
//   service_stress PRODUCERS REQUESTS_PER_PRODUCER [MAX_ITEMS] [BENCH]
// BENCH=1: certificates of 34 votes only, 100 us jobs, no hashing; prints the mean cost of one
// nw_service_certificate call (the ingest path) instead of stressing shapes.
// The hedge (nw_service_set_hedge) runs too: one job in 16 is 3 ms late, past the 1 ms
// deadline, and nw::host::* are doubles that answer with the same fingerprints, so a verdict
// is right whichever side delivers it; exactly one callback per request is still required.
// Built with g++ (-fsanitize=thread in `make service_stress_tsan`); test/bench tooling.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "narwhal_amd.h"
#include "nw_host.h"
#include "nw_runtime.h"

namespace {
using Clock = std::chrono::steady_clock;

uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
  return h;
}
constexpr uint64_t kFnv0 = 0xcbf29ce484222325ull;

std::atomic<uint64_t> g_bad_shape{0}, g_jobs{0};
bool g_no_delay = false;

struct Job {
  Clock::time_point due;
};

nw_job* make_job() {
  thread_local std::mt19937_64 rng(std::hash<std::thread::id>()(std::this_thread::get_id()));
  Job* j = new Job;
  // bench: a fixed 100 us per job (a small-job launch), so batches accumulate as on a device
  // one job in 16 is late (3 ms) so that the hedge answers part of the run
  j->due = Clock::now() + std::chrono::microseconds(g_no_delay ? 100 : rng() % 16 == 0 ? 3000
                                                                                       : rng() % 200);
  g_jobs.fetch_add(1);
  return reinterpret_cast<nw_job*>(j);
}

bool offsets_ok(const uint64_t* o, size_t n) {
  if (o[0] != 0) return false;
  for (size_t i = 0; i < n; ++i)
    if (o[i + 1] < o[i]) return false;
  return true;
}
}  // namespace

// ---- test doubles of the runtime and the device entry points ----------------------------
namespace nw {
namespace rt {
int ensure_init() { return 0; }
int set_err(int code, const char*, hipError_t) { return code; }
int check_committee(const nw_committee*) { return 0; }
int select_device(int* dev) {
  *dev = 0;
  return 0;
}
int jobs_prewarm(int, int, size_t, size_t) { return 0; }
size_t job_growth_log(uint64_t*, size_t) { return 0; }
}  // namespace rt
}  // namespace nw

extern "C" {
int nw_get_device(void) { return 0; }
int nw_set_device(int) { return 0; }

int nw_submit_certificates_verify_many(const nw_committee*, const nw_certificates* c,
                                       const uint8_t*, int32_t* st, uint64_t* ix, nw_job** job) {
  if (!offsets_ok(c->header_offsets, c->n) || !offsets_ok(c->vote_offsets, c->n))
    g_bad_shape.fetch_add(1);
  if (g_no_delay) {   // bench: the ingest path is measured, not the double's hashing
    memset(st, 0, 4 * c->n);
    if (ix) memset(ix, 0, 8 * c->n);
    *job = make_job();
    return 0;
  }
  for (size_t i = 0; i < c->n; ++i) {
    const uint64_t h0 = c->header_offsets[i], h1 = c->header_offsets[i + 1];
    const uint64_t v0 = c->vote_offsets[i], v1 = c->vote_offsets[i + 1];
    uint64_t h = fnv(kFnv0, c->header_bytes + h0, h1 - h0);
    h = fnv(h, &c->payload_counts[i], 4);
    h = fnv(h, c->ids + 32 * i, 32);
    h = fnv(h, c->header_sigs + 64 * i, 64);
    h = fnv(h, c->vote_pks + 32 * v0, 32 * (v1 - v0));
    h = fnv(h, c->vote_sigs + 64 * v0, 64 * (v1 - v0));
    st[i] = (int32_t)(h & 0x7fffffff);
    if (ix) ix[i] = h >> 31;
  }
  *job = make_job();
  return 0;
}
int nw_submit_headers_verify_many(const nw_committee*, const nw_certificates* c, int32_t* st,
                                  uint64_t* ix, nw_job** job) {
  if (!offsets_ok(c->header_offsets, c->n)) g_bad_shape.fetch_add(1);
  for (size_t i = 0; i < c->n; ++i) {
    const uint64_t h0 = c->header_offsets[i], h1 = c->header_offsets[i + 1];
    uint64_t h = fnv(kFnv0, c->header_bytes + h0, h1 - h0);
    h = fnv(h, &c->payload_counts[i], 4);
    h = fnv(h, c->ids + 32 * i, 32);
    h = fnv(h, c->header_sigs + 64 * i, 64);
    st[i] = (int32_t)(h & 0x7fffffff);
    if (ix) ix[i] = h >> 31;
  }
  *job = make_job();
  return 0;
}
int nw_submit_votes_verify_many(const nw_committee*, const uint8_t* ids, const uint64_t* rounds,
                                const uint8_t* origins, const uint8_t* authors,
                                const uint8_t* sigs, size_t n, int32_t* st, nw_job** job) {
  for (size_t i = 0; i < n; ++i) {
    uint64_t h = fnv(kFnv0, ids + 32 * i, 32);
    h = fnv(h, &rounds[i], 8);
    h = fnv(h, origins + 32 * i, 32);
    h = fnv(h, authors + 32 * i, 32);
    h = fnv(h, sigs + 64 * i, 64);
    st[i] = (int32_t)(h & 0x7fffffff);
  }
  *job = make_job();
  return 0;
}
int nw_submit_verify_strict(const uint8_t* digests, size_t, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, int32_t* st, uint8_t*, nw_job** job) {
  for (size_t i = 0; i < n; ++i) {
    uint64_t h = fnv(kFnv0, digests + 32 * i, 32);
    h = fnv(h, pks + 32 * i, 32);
    h = fnv(h, sigs + 64 * i, 64);
    st[i] = (int32_t)(h & 0x7fffffff);
  }
  *job = make_job();
  return 0;
}
int nw_submit_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                                const uint64_t* offsets, size_t nb, const uint8_t*, int32_t* st,
                                uint64_t* ix, nw_job** job) {
  if (!offsets_ok(offsets, nb)) g_bad_shape.fetch_add(1);
  for (size_t i = 0; i < nb; ++i) {
    const uint64_t o0 = offsets[i], o1 = offsets[i + 1];
    uint64_t h = fnv(kFnv0, digests + 32 * i, 32);
    h = fnv(h, pks + 32 * o0, 32 * (o1 - o0));
    h = fnv(h, sigs + 64 * o0, 64 * (o1 - o0));
    st[i] = (int32_t)(h & 0x7fffffff);
    if (ix) ix[i] = h >> 31;
  }
  *job = make_job();
  return 0;
}
}  // extern "C"

// ---- the host path (nw_host.cpp) as doubles: the same fingerprints as the device doubles ----
namespace nw {
namespace host {
struct Committee {
  int unused;
};
Committee* committee_new(const nw_committee*) { return new Committee{0}; }
void committee_free(Committee* c) { delete c; }
std::atomic<uint64_t> g_host_calls{0};
int verify_strict(const uint8_t msg32[32], const uint8_t pk[32], const uint8_t sig[64]) {
  g_host_calls.fetch_add(1);
  uint64_t h = fnv(kFnv0, msg32, 32);
  h = fnv(h, pk, 32);
  h = fnv(h, sig, 64);
  return (int32_t)(h & 0x7fffffff);
}
int verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                 const uint8_t*, const Committee*, uint64_t* fail_index) {
  g_host_calls.fetch_add(1);
  uint64_t h = fnv(kFnv0, digest, 32);
  h = fnv(h, pks, 32 * n);
  h = fnv(h, sigs, 64 * n);
  if (fail_index) *fail_index = h >> 31;
  return (int32_t)(h & 0x7fffffff);
}
int header_verify(const Committee&, const uint8_t* hb, size_t hlen, uint32_t np,
                  const uint8_t id[32], const uint8_t sig[64], uint64_t* index) {
  g_host_calls.fetch_add(1);
  uint64_t h = fnv(kFnv0, hb, hlen);
  h = fnv(h, &np, 4);
  h = fnv(h, id, 32);
  h = fnv(h, sig, 64);
  *index = h >> 31;
  return (int32_t)(h & 0x7fffffff);
}
int vote_verify(const Committee&, const uint8_t id[32], uint64_t round, const uint8_t origin[32],
                const uint8_t author[32], const uint8_t sig[64]) {
  g_host_calls.fetch_add(1);
  uint64_t h = fnv(kFnv0, id, 32);
  h = fnv(h, &round, 8);
  h = fnv(h, origin, 32);
  h = fnv(h, author, 32);
  h = fnv(h, sig, 64);
  return (int32_t)(h & 0x7fffffff);
}
int certificate_verify(const Committee&, const uint8_t* hb, size_t hlen, uint32_t np,
                       const uint8_t id[32], const uint8_t hsig[64], const uint8_t* vote_pks,
                       const uint8_t* vote_sigs, size_t nvotes, const uint8_t*, uint64_t* index) {
  g_host_calls.fetch_add(1);
  uint64_t h = fnv(kFnv0, hb, hlen);
  h = fnv(h, &np, 4);
  h = fnv(h, id, 32);
  h = fnv(h, hsig, 64);
  h = fnv(h, vote_pks, 32 * nvotes);
  h = fnv(h, vote_sigs, 64 * nvotes);
  *index = h >> 31;
  return (int32_t)(h & 0x7fffffff);
}
}  // namespace host
}  // namespace nw

extern "C" {
int nw_job_poll(nw_job* job) {
  return Clock::now() >= reinterpret_cast<Job*>(job)->due ? 1 : 0;
}
int nw_job_wait(nw_job* job) {
  std::this_thread::sleep_until(reinterpret_cast<Job*>(job)->due);
  return 0;
}
void nw_job_release(nw_job* job) { delete reinterpret_cast<Job*>(job); }
}  // extern "C"

// ---- the stress run ------------------------------------------------------------------------
namespace {
struct Expect {
  int32_t st;
  uint64_t ix;
  bool has_ix;
  std::atomic<int> calls{0};
  std::atomic<int> bad{0};
};

void on_verdict(void* arg, int32_t st, uint64_t ix) {
  Expect* e = static_cast<Expect*>(arg);
  if (st != e->st || (e->has_ix && ix != e->ix)) e->bad.fetch_add(1);
  e->calls.fetch_add(1);
}

void fill(std::mt19937_64& rng, std::vector<uint8_t>& v, size_t n) {
  v.resize(n);
  for (auto& x : v) x = (uint8_t)rng();
}
}  // namespace

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 4;
  const int R = argc > 2 ? atoi(argv[2]) : 20000;
  const size_t max_items = argc > 3 ? strtoull(argv[3], nullptr, 10) : 4096;
  const bool bench = argc > 4 && atoi(argv[4]) != 0;
  g_no_delay = bench;
  uint8_t pk[32] = {1};
  uint32_t stake = 1;
  uint64_t wo[2] = {0, 0};
  nw_committee com{1, pk, &stake, wo, nullptr};
  nw_service* s = nullptr;
  if (nw_service_create(&com, max_items, 200, 4, &s)) {
    fprintf(stderr, "create failed\n");
    return 2;
  }
  std::vector<Expect> ex((size_t)P * R);
  std::atomic<int> submit_err{0};
  std::vector<double> call_s(P, 0.0);
  std::vector<std::thread> th;
  for (int p = 0; p < P; ++p)
    th.emplace_back([&, p] {
      std::mt19937_64 rng(1234 + p);
      std::vector<uint8_t> hb, id, sg, vp, vs, dg;
      for (int r = 0; r < R; ++r) {
        Expect& e = ex[(size_t)p * R + r];
        const int kind = bench ? 0 : (int)(rng() % 5);
        int rc = 0;
        if (kind == 0 || kind == 1) {   // certificate / header
          const uint32_t pc = bench ? 0 : (uint32_t)(rng() % 4);
          const size_t parents = bench ? 34 : rng() % 70;
          const size_t hl = 40 + 36 * pc + 32 * parents;
          size_t nv = bench ? 34 : (rng() % 8 == 0 ? rng() % 3000 : rng() % 68);
          fill(rng, hb, hl);
          fill(rng, id, 32);
          fill(rng, sg, 64);
          uint64_t h = fnv(kFnv0, hb.data(), hl);
          h = fnv(h, &pc, 4);
          h = fnv(h, id.data(), 32);
          h = fnv(h, sg.data(), 64);
          if (kind == 0) {
            fill(rng, vp, 32 * nv);
            fill(rng, vs, 64 * nv);
            h = fnv(h, vp.data(), 32 * nv);
            h = fnv(h, vs.data(), 64 * nv);
          }
          e.st = bench ? 0 : (int32_t)(h & 0x7fffffff);
          e.ix = bench ? 0 : h >> 31;
          e.has_ix = true;
          const Clock::time_point t0 = Clock::now();
          if (kind == 0)
            rc = nw_service_certificate(s, hb.data(), hl, pc, id.data(), sg.data(), vp.data(),
                                        vs.data(), nv, on_verdict, &e);
          else
            rc = nw_service_header(s, hb.data(), hl, pc, id.data(), sg.data(), on_verdict, &e);
          call_s[p] += std::chrono::duration<double>(Clock::now() - t0).count();
        } else if (kind == 2) {   // vote
          std::vector<uint8_t> o, a;
          fill(rng, id, 32);
          fill(rng, o, 32);
          fill(rng, a, 32);
          fill(rng, sg, 64);
          const uint64_t round = rng();
          uint64_t h = fnv(kFnv0, id.data(), 32);
          h = fnv(h, &round, 8);
          h = fnv(h, o.data(), 32);
          h = fnv(h, a.data(), 32);
          h = fnv(h, sg.data(), 64);
          e.st = (int32_t)(h & 0x7fffffff);
          e.has_ix = false;
          rc = nw_service_vote(s, id.data(), round, o.data(), a.data(), sg.data(), on_verdict, &e);
        } else if (kind == 3) {   // Signature::verify
          fill(rng, dg, 32);
          fill(rng, vp, 32);
          fill(rng, sg, 64);
          uint64_t h = fnv(kFnv0, dg.data(), 32);
          h = fnv(h, vp.data(), 32);
          h = fnv(h, sg.data(), 64);
          e.st = (int32_t)(h & 0x7fffffff);
          e.has_ix = false;
          rc = nw_service_verify(s, dg.data(), vp.data(), sg.data(), on_verdict, &e);
        } else {   // verify_batch, 0 .. 200 items
          const size_t n = rng() % 201;
          fill(rng, dg, 32);
          fill(rng, vp, 32 * n);
          fill(rng, vs, 64 * n);
          uint64_t h = fnv(kFnv0, dg.data(), 32);
          h = fnv(h, vp.data(), 32 * n);
          h = fnv(h, vs.data(), 64 * n);
          e.st = (int32_t)(h & 0x7fffffff);
          e.ix = h >> 31;
          e.has_ix = true;
          rc = nw_service_verify_batch(s, dg.data(), vp.data(), vs.data(), n, on_verdict, &e);
        }
        if (rc) {
          submit_err.fetch_add(1);
          e.calls.store(1);   // not accepted: no callback will come
        }
      }
    });
  for (auto& t : th) t.join();
  nw_service_drain(s);
  uint64_t reqs = 0, jobs = 0, hedged = 0, host_first = 0, host_only = 0;
  nw_service_stats(s, &reqs, &jobs);
  nw_service_hedge_stats(s, &hedged, &host_first, &host_only, nullptr);
  nw_service_destroy(s);
  size_t missing = 0, dup = 0, bad = 0;
  for (auto& e : ex) {
    const int c = e.calls.load();
    missing += c == 0;
    dup += c > 1;
    bad += e.bad.load() != 0;
  }
  double cs = 0;
  for (double x : call_s) cs += x;
  printf("{\"producers\": %d, \"requests\": %zu, \"accepted\": %llu, \"jobs\": %llu, "
         "\"submit_errors\": %d, \"missing\": %zu, \"duplicate\": %zu, \"wrong\": %zu, "
         "\"bad_shape\": %llu, \"cert_call_mean_us\": %.3f, \"hedged\": %llu, "
         "\"host_first\": %llu, \"host_only_batches\": %llu, \"host_calls\": %llu}\n",
         P, ex.size(), (unsigned long long)reqs, (unsigned long long)jobs, submit_err.load(),
         missing, dup, bad, (unsigned long long)g_bad_shape.load(),
         bench ? cs / ((double)P * R) * 1e6 : -1.0, (unsigned long long)hedged,
         (unsigned long long)host_first, (unsigned long long)host_only,
         (unsigned long long)nw::host::g_host_calls.load());
  return (missing || dup || bad || g_bad_shape.load() || submit_err.load()) ? 1 : 0;
}
