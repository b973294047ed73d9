// bar_probe.hip — diagnostics (GPU box; not product code): does the box's host-memory stall
// episode (the GPU's reads of pinned host memory stall for 10-45 ms at times)
// also hit inputs that the CPU writes straight into device memory? Fine-grained device memory
// (hipExtMallocWithFlags(hipDeviceMallocFinegrained)) is CPU-visible when the BAR maps VRAM;
// then a request's bytes can travel as the CPU's posted writes, and the kernel reads device
// memory only. Modes, interleaved every ~100 us for SECONDS, each completion polled:
//   pinned  CPU writes 64 KB into pinned host memory, a kernel reads it across the bus
//   bar     CPU writes 64 KB into fine-grained VRAM through its host mapping, a kernel reads it
//   device  a kernel reads 64 KB of ordinary device memory (no CPU write)
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/bar_probe.hip -o tools/ubench/bar_probe
//   ./tools/ubench/bar_probe [SECONDS]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <setjmp.h>
#include <signal.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr size_t kBytes = 1 << 16;

__global__ void k_sum(const uint4* __restrict__ in, uint32_t* __restrict__ out) {
  const uint4 v = in[blockIdx.x * blockDim.x + threadIdx.x];
  uint32_t s = v.x ^ v.y ^ v.z ^ v.w;
  for (int o = 32; o > 0; o >>= 1) s ^= __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

using Clock = std::chrono::steady_clock;

// Is a device pointer mapped into the CPU's address space? The /proc/self/maps line that
// holds it, then one guarded read and write through it (SIGSEGV / SIGBUS caught).
static sigjmp_buf g_jb;
static void on_fault(int) { siglongjmp(g_jb, 1); }
static bool cpu_touch(volatile uint8_t* p) {
  struct sigaction sa{}, o1{}, o2{};
  sa.sa_handler = on_fault;
  sigaction(SIGSEGV, &sa, &o1);
  sigaction(SIGBUS, &sa, &o2);
  bool ok = false;
  if (sigsetjmp(g_jb, 1) == 0) {
    const uint8_t v = p[0];
    p[0] = (uint8_t)(v ^ 0x5a);
    ok = p[0] == (uint8_t)(v ^ 0x5a);
  }
  sigaction(SIGSEGV, &o1, nullptr);
  sigaction(SIGBUS, &o2, nullptr);
  return ok;
}
static void maps_line(const void* p) {
  FILE* f = fopen("/proc/self/maps", "r");
  char line[512];
  const uintptr_t a = (uintptr_t)p;
  bool found = false;
  while (f && fgets(line, sizeof line, f)) {
    unsigned long lo = 0, hi = 0;
    if (sscanf(line, "%lx-%lx", &lo, &hi) == 2 && a >= lo && a < hi) {
      line[strcspn(line, "\n")] = 0;
      printf("{\"maps\": \"%s\"}\n", line);
      found = true;
    }
  }
  if (f) fclose(f);
  if (!found) printf("{\"maps\": null}\n");
  fflush(stdout);
}

int main(int argc, char** argv) {
  const double secs = argc > 1 ? atof(argv[1]) : 20.0;
  void* bar = nullptr;
  CK(hipExtMallocWithFlags(&bar, kBytes, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, bar));
  printf("{\"finegrained_vram\": {\"type\": %d, \"device\": %p, \"host\": %p}}\n", (int)at.type,
         at.devicePointer, at.hostPointer);
  fflush(stdout);
  uint8_t* bar_host = static_cast<uint8_t*>(at.hostPointer);
  maps_line(bar);
  if (!bar_host) {   // no host mapping reported: is the device address itself CPU-mapped?
    const bool ok = cpu_touch(static_cast<volatile uint8_t*>(bar));
    printf("{\"cpu_access_via_device_pointer\": %s}\n", ok ? "true" : "false");
    fflush(stdout);
    if (ok) bar_host = static_cast<uint8_t*>(bar);
  }
  uint8_t* pinned = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pinned), kBytes, hipHostMallocMapped | hipHostMallocCoherent));
  void* pinned_dev = nullptr;
  CK(hipHostGetDevicePointer(&pinned_dev, pinned, 0));
  void* dmem = nullptr;
  CK(hipMalloc(&dmem, kBytes));
  CK(hipMemset(dmem, 0, kBytes));
  uint32_t* out = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&out), 4096));
  std::vector<uint8_t> src(kBytes);
  for (size_t i = 0; i < kBytes; ++i) src[i] = (uint8_t)(i * 131 + 7);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const char* names[3] = {"pinned", "bar", "device"};
  const int nmodes = bar_host ? 3 : 2;
  std::vector<double> lat[3], wr[3];
  std::vector<std::pair<double, double>> slow[3];
  const int blocks = kBytes / 16 / 256;
  // the CPU's write into the BAR mapping, checked once through the kernel's view
  if (bar_host) {
    memcpy(bar_host, src.data(), kBytes);
    std::vector<uint8_t> back(kBytes);
    CK(hipMemcpy(back.data(), bar, kBytes, hipMemcpyDeviceToHost));
    printf("{\"bar_write_visible_to_device\": %s}\n", memcmp(back.data(), src.data(), kBytes) ? "false" : "true");
    fflush(stdout);
  }
  const Clock::time_point t_start = Clock::now();
  int it = 0;
  while (std::chrono::duration<double>(Clock::now() - t_start).count() < secs) {
    for (int m = 0; m < nmodes; ++m) {
      const int mode = m == 1 && !bar_host ? 2 : m;
      const Clock::time_point t0 = Clock::now();
      const void* in = dmem;
      if (mode == 0) {
        src[it % kBytes] ^= 1;
        memcpy(pinned, src.data(), kBytes);
        in = pinned_dev;
      } else if (mode == 1) {
        src[it % kBytes] ^= 1;
        memcpy(bar_host, src.data(), kBytes);
        in = bar;
      }
      const Clock::time_point t1 = Clock::now();
      hipLaunchKernelGGL(k_sum, dim3(blocks), dim3(256), 0, s, static_cast<const uint4*>(in), out);
      CK(hipEventRecord(ev, s));
      while (hipEventQuery(ev) == hipErrorNotReady) {
      }
      const Clock::time_point t2 = Clock::now();
      const double dt = std::chrono::duration<double>(t2 - t0).count() * 1e3;
      lat[mode].push_back(dt);
      wr[mode].push_back(std::chrono::duration<double>(t1 - t0).count() * 1e3);
      if (dt > 1.0)
        slow[mode].push_back({std::chrono::duration<double>(t0 - t_start).count(), dt});
      while (std::chrono::duration<double>(Clock::now() - t0).count() < 1e-4) {
      }
    }
    ++it;
  }
  for (int m = 0; m < 3; ++m) {
    if (lat[m].empty()) continue;
    std::vector<double> a = lat[m], w = wr[m];
    std::sort(a.begin(), a.end());
    std::sort(w.begin(), w.end());
    printf("{\"mode\": \"%s\", \"iterations\": %zu, \"p50_ms\": %.4f, \"p99_ms\": %.4f, "
           "\"max_ms\": %.3f, \"cpu_write_p50_ms\": %.4f, \"cpu_write_max_ms\": %.3f, "
           "\"over_1ms\": [",
           names[m], a.size(), a[a.size() / 2], a[a.size() * 99 / 100], a.back(),
           w[w.size() / 2], w.back());
    for (size_t i = 0; i < slow[m].size() && i < 200; ++i)
      printf("%s[%.4f, %.3f]", i ? ", " : "", slow[m][i].first, slow[m][i].second);
    printf("]}\n");
  }
  return 0;
}
