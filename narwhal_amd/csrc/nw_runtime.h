// nw_runtime.h — internal runtime helpers shared by nw_api.cpp and nw_jobs.cpp (not part of
// the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "narwhal_amd.h"
#include "nw_kernels.h"

namespace nw {
namespace rt {

// Initialise the library (idempotent): 0, or a negative NW_E_* with the error text set.
int ensure_init();
// Make the calling thread's selected device (nw_set_device) current for HIP; returns 0 and
// the library device index, or a negative NW_E_*.
int select_device(int* dev_index);
// Make library device dev_index current for HIP on this thread (0 or NW_E_*).
int use_device(int dev_index);
// The calling thread's nw_set_device value (NW_ALL_DEVICES = fan out), and setting it.
int thread_device();
void set_thread_device(int dev_index);
int device_count();
// With nw_set_device(NW_ALL_DEVICES): the device index of every part a host-buffer call is
// split into (one per device, or NW_FANOUT_PARTS parts round-robin); empty otherwise.
std::vector<int> fanout_devices();
// Record the calling thread's last error (nw_last_error) and return `code`.
int set_err(int code, const char* what, hipError_t e = hipSuccess);
// Fill buf from the OS CSPRNG (getrandom).
int os_random(void* buf, size_t n);
// count pooled jobs on library device dev, made now with hbytes / dbytes of staging
// (nw_jobs.cpp; the aggregation service's start-up).
int jobs_prewarm(int dev, int count, size_t hbytes, size_t dbytes);
// Diagnostics (NW_SERVICE_DEBUG): job staging growths so far — pinned (kind 0), device
// (kind 1), small-job counters (kind 2), NW_SMALL_VRAM input buffers (kind 3) — with their time (steady-clock ns), new capacity and
// duration in us. Copies up to `max` of them into `out` (4 words each) and returns the count.
size_t job_growth_log(uint64_t* out, size_t max);

// ---- primary messages (nw_api.cpp), shared by the blocking, job and device entry points ----
// Host-side argument checks of a host-memory committee / certificate stream (0 or
// NW_E_INVALID_ARG with the error text set); *nvotes = vote_offsets[n] (0 for headers).
int check_committee(const nw_committee* com);
int check_certificates(const nw_certificates* cs, int headers_only, size_t* nvotes);
// Device bytes of the Header / Certificate pipeline's scratch, and the pipeline itself on
// library device dev (current for HIP): every pointer inside dcom / dcs and the buffers are
// device pointers, host_vote_offsets the vote offsets in host memory (read during the call
// only). Queues the whole check on `s` and returns without waiting.
size_t cert_workspace_bytes(size_t n, size_t nvotes);
// committee_tag: identifies the committee for the failure-rate policy (committee_hash of
// the host keys; 0 = unknown, the policy is then kept per committee size). host_pks
// (optional): the committee's keys in host memory; the key tables built by this call are
// then marked as theirs, for small jobs (ReadLease).
// fork (optional): a second stream and two events of the caller's; the header checks then
// run on fork->s2 concurrently with the vote checks on s (joined before the call returns).
struct Fork {
  hipStream_t s2;
  hipEvent_t ev_fork, ev_join;
};
int cert_pipeline(int dev, const nw_committee& dcom, const nw_certificates& dcs,
                  const uint64_t* host_vote_offsets, int headers_only, const void* z16,
                  const uint8_t zkey32[32], void* workspace, int32_t* status, uint64_t* index,
                  hipStream_t s, uint64_t committee_tag = 0, const Fork* fork = nullptr,
                  const uint8_t* host_pks = nullptr);
// FNV-1a over a host committee's keys (never 0).
uint64_t committee_hash(const nw_committee* com);
// Vote::verify for n votes (device pointers), scratch = votes_workspace_bytes(n).
size_t votes_workspace_bytes(size_t n);
int votes_pipeline(int dev, const nw_committee& dcom, size_t n, const uint8_t* ids,
                   const uint64_t* rounds, const uint8_t* origins, const uint8_t* authors,
                   const uint8_t* sigs, void* workspace, int32_t* status, hipStream_t s,
                   const uint8_t* host_pks = nullptr);

// Per-device buffers shared by every caller of the library (host-buffer jobs, blocking
// calls and nw_dev_* calls on caller streams): the strict kernel's per-lane table workspace
// and the committee key tables. A launch sequence that uses them holds a Lease on the
// device: acquire() locks the device's lease and makes `stream` wait for the previous
// holder's last launch (an event chain), so launches on different streams never overlap on
// these buffers; release() (or the destructor) records a new event on `stream` and unlocks.
// Growing the key tables first waits for that event: every earlier user is ordered before
// it, so no queued launch still reads the old buffer when it is freed.
class Lease {
 public:
  Lease() = default;
  Lease(const Lease&) = delete;
  Lease& operator=(const Lease&) = delete;
  ~Lease() { (void)release(); }
  int acquire(int dev_index, hipStream_t stream);
  // The device's strict workspace (nw::strict_workspace_bytes(), allocated once).
  int strict_ws(void** out);
  // Key tables for nkeys keys (grow-only at one comb width, nw_api.cpp key_width): tabs
  // (nw::key_tables_bytes) and ok words, their layout (ks), plus the reuse state of
  // nw::launch_key_tables: the device copy of the keys they were last built from, the
  // rebuild flag word, and whether a rebuild is forced (new size / width / buffers).
  int key_tables(size_t nkeys, void** tabs, uint32_t** ok, nw::keyspec* ks,
                 uint32_t** saved = nullptr, uint32_t** flag = nullptr, bool* force = nullptr);
  // After a successful launch_key_tables: the saved keys now describe the tables; host_pks
  // (nkeys x 32 bytes, optional) are those keys in host memory (small jobs compare them).
  void keys_built(size_t nkeys, const uint8_t* host_pks = nullptr);
  // After keys_built: when the committee's tables are wider than 16 bits, also a 16-bit set
  // of the same keys for the small-job kernel (ReadLease hands it out): lone requests read
  // 67 MB per key instead of 940 MB (profiles/r06p: the 20-bit tables made ~3.5 % of N = 50
  // single-certificate jobs take > 1 ms at low rates). dpks: the keys on the device. Skipped
  // (small jobs keep the wide tables) without host keys, without memory, or with
  // NW_SMALL_KEYW16=0.
  int small_tables(const uint32_t* dpks, size_t nkeys, const uint8_t* host_pks);
  // Record the chain event on the stream and unlock (idempotent). 0 or NW_E_DEVICE.
  int release();

 private:
  int dev_ = -1;
  hipStream_t stream_ = nullptr;
  bool held_ = false;
};

// Read-only use of the key tables by a small job (nw_small.hip), which writes none of the
// shared buffers: readers do not wait for each other, only for the last Lease holder (whose
// launches may have built the tables), and every Lease holder waits for the readers queued
// before it (their completion events). acquire() returns 0 with the tables when they hold
// exactly the nkeys keys pks (host memory), 1 when they do not (the caller then
// runs the ordinary pipeline, which builds them), or a negative NW_E_*. The device stays
// locked between acquire() and release() (a launch's host time).
class ReadLease {
 public:
  ReadLease() = default;
  ReadLease(const ReadLease&) = delete;
  ReadLease& operator=(const ReadLease&) = delete;
  ~ReadLease() { (void)release(); }
  int acquire(int dev_index, hipStream_t stream, const uint8_t* pks, size_t nkeys,
              const void** tabs, const uint32_t** ok, nw::keyspec* ks);
  int release();

 private:
  int dev_ = -1;
  hipStream_t stream_ = nullptr;
  bool held_ = false;
};

}  // namespace rt
}  // namespace nw
