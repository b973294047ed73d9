// nw_loadgen.cpp — open-loop load generator for the native aggregation service (bench
// tooling; bench.py's service_latency leg loads it with ctypes). Built against the public C
// ABI only (include/narwhal_amd.h), as a Rust crypto-gpu crate's tokio tasks would call it.
//
// Certificates arrive at a fixed offered rate: request i is due at t0 + i / rate and goes
// to nw_service_certificate from one of `producers` threads (the primary's Core task is
// one producer; several model several primaries or Core plus the synchronizer). Latency of
// request i = verdict-callback time - scheduled arrival time, so a producer that falls
// behind its schedule shows up as latency, not as a lower offered rate. Every verdict is
// compared with the expected (status, index) of the corpus row it came from.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "narwhal_amd.h"

namespace {
using Clock = std::chrono::steady_clock;

struct Run {
  const int32_t* exp_status;
  const uint64_t* exp_index;
  size_t nuniq;
  double* lat;
  std::atomic<uint64_t> mismatches{0};
  std::atomic<int64_t> last_ns{0};
  Clock::time_point t0;
};

struct Rec {
  Run* run;
  uint64_t i;
  Clock::time_point due;
};

void on_verdict(void* arg, int32_t status, uint64_t index) {
  Rec* r = static_cast<Rec*>(arg);
  const Clock::time_point now = Clock::now();
  Run* run = r->run;
  run->lat[r->i] = std::chrono::duration<double>(now - r->due).count();
  const size_t u = r->i % run->nuniq;
  if (status != run->exp_status[u] || index != run->exp_index[u]) run->mismatches.fetch_add(1);
  const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(now - run->t0).count();
  int64_t prev = run->last_ns.load();
  while (ns > prev && !run->last_ns.compare_exchange_weak(prev, ns)) {
  }
}
int timed_run(nw_service* s, const nw_certificates* corpus, const int32_t* exp_status,
              const uint64_t* exp_index, double rate, uint64_t total, uint32_t producers,
              double* lat_out, double* out);
}  // namespace

extern "C" {

// Returns 0 or the first negative NW_E_* from the service. lat_out: total seconds;
// out (16 doubles — a caller's array must hold all 16): elapsed seconds (t0 .. last
// verdict), jobs, mismatches, and the
// producers' lateness: the largest and the mean (call time - due time) of a submit, seconds
// (a producer that cannot keep its schedule shows here before it shows as latency), then
// the producers' CPU / wall time and their voluntary / involuntary context switches, and
// the nw_service_certificate calls' mean and longest duration and the count above 20 us;
// out[11..12]: jobs that took the small-job launch and the bulk pipeline during the timed
// run (nw_path_stats); out[13..15]: the service's hedge during the timed run: requests
// hedged, requests the host answered first, batches the host took whole
// (nw_service_hedge_stats).
int nw_loadgen_certificates(const nw_committee* com, const nw_certificates* corpus,
                            const int32_t* exp_status, const uint64_t* exp_index, double rate,
                            uint64_t total, size_t max_items, uint32_t max_delay_us,
                            size_t max_inflight, uint32_t producers, double* lat_out,
                            double* out) {
  if (!com || !corpus || !corpus->n || !exp_status || !exp_index || !lat_out || !out ||
      rate <= 0 || !producers)
    return NW_E_INVALID_ARG;
  nw_service* s = nullptr;
  int rc = nw_service_create(com, max_items, max_delay_us, max_inflight, &s);
  if (rc) return rc;
  // warm-up (untimed): the committee's key tables and the job pool
  {
    Run warm;
    std::vector<double> wl(64);
    warm.exp_status = exp_status;
    warm.exp_index = exp_index;
    warm.nuniq = corpus->n;
    warm.lat = wl.data();
    warm.t0 = Clock::now();
    std::vector<Rec> wr(64);
    for (uint64_t i = 0; i < 64 && i < total; ++i) {
      wr[i] = {&warm, i, Clock::now()};
      const size_t u = i % corpus->n;
      const uint64_t h0 = corpus->header_offsets[u], h1 = corpus->header_offsets[u + 1];
      const uint64_t v0 = corpus->vote_offsets[u], v1 = corpus->vote_offsets[u + 1];
      rc = nw_service_certificate(s, corpus->header_bytes + h0, h1 - h0, corpus->payload_counts[u],
                                  corpus->ids + 32 * u, corpus->header_sigs + 64 * u,
                                  corpus->vote_pks + 32 * v0, corpus->vote_sigs + 64 * v0,
                                  v1 - v0, on_verdict, &wr[i]);
      if (rc) break;
    }
    nw_service_drain(s);
    if (rc) {
      nw_service_destroy(s);
      return rc;
    }
    // the hedge's host tables of the committee (built in the background at create)
    for (int t = 0; t < 4000; ++t) {
      int ready = 0;
      nw_service_hedge_stats(s, nullptr, nullptr, nullptr, &ready);
      if (ready) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  rc = timed_run(s, corpus, exp_status, exp_index, rate, total, producers, lat_out, out);
  nw_service_destroy(s);
  return rc;
}

int nw_loadgen_certificates_on(nw_service* s, const nw_certificates* corpus,
                               const int32_t* exp_status, const uint64_t* exp_index, double rate,
                               uint64_t total, uint32_t producers, double* lat_out,
                               double* out) {
  if (!s || !corpus || !corpus->n || !exp_status || !exp_index || !lat_out || !out ||
      rate <= 0 || !producers)
    return NW_E_INVALID_ARG;
  return timed_run(s, corpus, exp_status, exp_index, rate, total, producers, lat_out, out);
}

}  // extern "C"

namespace {
int timed_run(nw_service* s, const nw_certificates* corpus, const int32_t* exp_status,
              const uint64_t* exp_index, double rate, uint64_t total, uint32_t producers,
              double* lat_out, double* out) {
  Run run;
  run.exp_status = exp_status;
  run.exp_index = exp_index;
  run.nuniq = corpus->n;
  run.lat = lat_out;
  std::vector<Rec> recs(total);
  std::atomic<int> first_err{0};
  std::vector<double> call_sum(producers, 0.0), call_max(producers, 0.0);
  std::vector<uint64_t> call_slow(producers, 0);
  auto submit = [&](uint64_t i) {
    const size_t u = i % corpus->n;
    const uint64_t h0 = corpus->header_offsets[u], h1 = corpus->header_offsets[u + 1];
    const uint64_t v0 = corpus->vote_offsets[u], v1 = corpus->vote_offsets[u + 1];
    const int e = nw_service_certificate(s, corpus->header_bytes + h0, h1 - h0,
                                         corpus->payload_counts[u], corpus->ids + 32 * u,
                                         corpus->header_sigs + 64 * u, corpus->vote_pks + 32 * v0,
                                         corpus->vote_sigs + 64 * v0, v1 - v0, on_verdict,
                                         &recs[i]);
    if (e) {
      int z = 0;
      first_err.compare_exchange_strong(z, e);
    }
  };
  uint64_t jobs0 = 0, sm0 = 0, pp0 = 0;
  nw_service_stats(s, nullptr, &jobs0);
  nw_path_stats(&sm0, &pp0);
  uint64_t hq0 = 0, hf0 = 0, ho0 = 0;
  nw_service_hedge_stats(s, &hq0, &hf0, &ho0, nullptr);
  run.t0 = Clock::now() + std::chrono::milliseconds(2);
  const double period = 1.0 / rate;
  for (uint64_t i = 0; i < total; ++i)
    recs[i] = {&run, i,
               run.t0 + std::chrono::duration_cast<Clock::duration>(
                            std::chrono::duration<double>(period * (double)i))};
  // NW_LOADGEN_GAPS=<file>: a monitor thread that only reads the clock records every gap
  // above 0.5 ms (the thread was not running: the whole process, or its CPU, stalled), as
  // steady-clock ns, to set beside the service's per-job timeline (NW_SERVICE_DEBUG)
  std::atomic<bool> mon_stop{false};
  std::vector<std::pair<int64_t, int64_t>> gaps;
  std::thread mon;
  const char* gap_path = getenv("NW_LOADGEN_GAPS");
  if (gap_path && *gap_path)
    mon = std::thread([&] {
      auto prev = Clock::now();
      while (!mon_stop.load(std::memory_order_relaxed)) {
        const auto now = Clock::now();
        if (now - prev > std::chrono::microseconds(500) && gaps.size() < 100000)
          gaps.emplace_back(
              std::chrono::duration_cast<std::chrono::nanoseconds>(prev.time_since_epoch()).count(),
              std::chrono::duration_cast<std::chrono::nanoseconds>(now - prev).count());
        prev = now;
      }
    });
  std::vector<std::thread> th;
  std::vector<double> lag_max(producers, 0.0), lag_sum(producers, 0.0);
  std::vector<double> cpu_s(producers, 0.0), wall_s(producers, 0.0);
  std::vector<long> vcsw(producers, 0), ivcsw(producers, 0);
  for (uint32_t p = 0; p < producers; ++p)
    th.emplace_back([&, p] {
      const Clock::time_point w0 = Clock::now();
      struct rusage r0, r1;
      getrusage(RUSAGE_THREAD, &r0);
      for (uint64_t i = p; i < total; i += producers) {
        const Clock::time_point due = recs[i].due;
        Clock::time_point now = Clock::now();
        // sleep to just before the due time, then spin: a sleep wakes up tens of
        // microseconds late, which would count as the service's latency
        const auto early = std::chrono::microseconds(200);
        if (due - now > early) std::this_thread::sleep_until(due - early);
        while ((now = Clock::now()) < due) {
        }
        const double lag = std::chrono::duration<double>(now - due).count();
        lag_max[p] = std::max(lag_max[p], lag);
        lag_sum[p] += lag;
        submit(i);
        const double c = std::chrono::duration<double>(Clock::now() - now).count();
        call_sum[p] += c;
        call_max[p] = std::max(call_max[p], c);
        call_slow[p] += c > 20e-6;
      }
      getrusage(RUSAGE_THREAD, &r1);
      auto sec = [](const timeval& t) { return (double)t.tv_sec + 1e-6 * (double)t.tv_usec; };
      cpu_s[p] = sec(r1.ru_utime) + sec(r1.ru_stime) - sec(r0.ru_utime) - sec(r0.ru_stime);
      wall_s[p] = std::chrono::duration<double>(Clock::now() - w0).count();
      vcsw[p] = r1.ru_nvcsw - r0.ru_nvcsw;
      ivcsw[p] = r1.ru_nivcsw - r0.ru_nivcsw;
    });
  for (auto& t : th) t.join();
  nw_service_drain(s);
  if (mon.joinable()) {
    mon_stop = true;
    mon.join();
    if (FILE* f = fopen(gap_path, "a")) {
      for (const auto& g : gaps) fprintf(f, "%lld,%lld\n", (long long)g.first, (long long)g.second);
      fclose(f);
    }
  }
  uint64_t jobs1 = 0, sm1 = 0, pp1 = 0;
  nw_service_stats(s, nullptr, &jobs1);
  nw_path_stats(&sm1, &pp1);
  out[0] = (double)run.last_ns.load() * 1e-9;
  out[1] = (double)(jobs1 - jobs0);
  out[2] = (double)run.mismatches.load();
  double lm = 0, ls = 0;
  for (uint32_t p = 0; p < producers; ++p) {
    lm = std::max(lm, lag_max[p]);
    ls += lag_sum[p];
  }
  out[3] = lm;
  out[4] = ls / (double)(total ? total : 1);
  double cs = 0, ws = 0, v = 0, iv = 0;
  for (uint32_t p = 0; p < producers; ++p) {
    cs += cpu_s[p];
    ws += wall_s[p];
    v += (double)vcsw[p];
    iv += (double)ivcsw[p];
  }
  out[5] = ws > 0 ? cs / ws : 0;   // producers' CPU time / wall time (1 = never off-CPU)
  out[6] = v;                      // voluntary context switches (sleeps: futex, nanosleep)
  out[7] = iv;                     // involuntary ones (preempted: CPU contention)
  double cs2 = 0, cm = 0, sl = 0;
  for (uint32_t p = 0; p < producers; ++p) {
    cs2 += call_sum[p];
    cm = std::max(cm, call_max[p]);
    sl += (double)call_slow[p];
  }
  out[8] = cs2 / (double)(total ? total : 1);   // mean nw_service_certificate call, seconds
  out[9] = cm;                                  // longest call
  out[10] = sl;                                 // calls longer than 20 us
  out[11] = (double)(sm1 - sm0);                // small-job launches
  out[12] = (double)(pp1 - pp0);                // bulk-pipeline jobs
  uint64_t hq1 = 0, hf1 = 0, ho1 = 0;
  nw_service_hedge_stats(s, &hq1, &hf1, &ho1, nullptr);
  out[13] = (double)(hq1 - hq0);                // requests hedged
  out[14] = (double)(hf1 - hf0);                // answered by the host first
  out[15] = (double)(ho1 - ho0);                // batches the host took whole
  return first_err.load();
}
}  // namespace
