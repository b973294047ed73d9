// ubench_h2d.hip — host-side costs of a one-call verify_batch (config 1) on this box:
// memcpy of the inputs into pinned coherent staging, one H2D of them, an empty kernel's
// launch-to-completion, and an empty kernel reading the same bytes straight from the pinned
// buffer (zero-copy). Median of `reps` runs each, microseconds. Bench tooling.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void k_empty(uint32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] = 1;
}

// every lane reads 96 bytes (one vote's key and signature) and folds them into one word
__global__ void k_read(const uint32_t* __restrict__ in, size_t nvotes, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvotes) return;
  uint32_t a = 0;
#pragma unroll
  for (int j = 0; j < 24; ++j) a ^= in[24 * i + j];
  out[i] = a;
}

using Clock = std::chrono::steady_clock;
static double us(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}
static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const size_t nvotes = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000;
  const int reps = argc > 2 ? atoi(argv[2]) : 200;
  const size_t bytes = 96 * nvotes;
  std::vector<uint8_t> src(bytes);
  for (size_t i = 0; i < bytes; ++i) src[i] = (uint8_t)(i * 131 + 7);
  uint8_t* h = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h), bytes, hipHostMallocMapped | hipHostMallocCoherent));
  void* hd = nullptr;
  CK(hipHostGetDevicePointer(&hd, h, 0));
  uint8_t* d = nullptr;
  uint32_t* o = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&d), bytes));
  CK(hipMalloc(reinterpret_cast<void**>(&o), 4 * nvotes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const unsigned grid = (unsigned)((nvotes + 255) / 256);
  std::vector<double> t_memcpy, t_h2d, t_empty, t_read_dev, t_read_host, t_all;
  for (int r = 0; r < reps + 10; ++r) {
    auto a = Clock::now();
    memcpy(h, src.data(), bytes);
    auto b = Clock::now();
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    auto c = Clock::now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, o);
    CK(hipStreamSynchronize(s));
    auto e = Clock::now();
    hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(d),
                       nvotes, o);
    CK(hipStreamSynchronize(s));
    auto f = Clock::now();
    hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(hd),
                       nvotes, o);
    CK(hipStreamSynchronize(s));
    auto g = Clock::now();
    // the job path: memcpy + H2D + kernel, one sync
    memcpy(h, src.data(), bytes);
    CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(d),
                       nvotes, o);
    CK(hipStreamSynchronize(s));
    auto k = Clock::now();
    if (r < 10) continue;
    t_memcpy.push_back(us(a, b));
    t_h2d.push_back(us(b, c));
    t_empty.push_back(us(c, e));
    t_read_dev.push_back(us(e, f));
    t_read_host.push_back(us(f, g));
    t_all.push_back(us(g, k));
  }
  printf("{\"votes\": %zu, \"bytes\": %zu, \"memcpy_us\": %.1f, \"h2d_sync_us\": %.1f, "
         "\"empty_kernel_sync_us\": %.1f, \"read_device_kernel_sync_us\": %.1f, "
         "\"read_pinned_kernel_sync_us\": %.1f, \"memcpy_h2d_kernel_sync_us\": %.1f}\n",
         nvotes, bytes, med(t_memcpy), med(t_h2d), med(t_empty), med(t_read_dev),
         med(t_read_host), med(t_all));
  return 0;
}
