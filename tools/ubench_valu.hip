// Microbenchmark: issue throughput of the gfx950 integer VALU instructions the
// field arithmetic can be built from. Each kernel runs 16 independent accumulator
// chains per lane (inline asm, so the compiler cannot fold them) over a grid that
// fills all 256 CUs at 8 waves/CU. Prints lane-ops/s per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

// 32-bit two-operand form: d = op(a, d)
#define K32(NAME, INSTR)                                                       \
__global__ void NAME(uint32_t* out, uint32_t seed) {                           \
  uint32_t a = seed + threadIdx.x, b = a * 3u + 1u;                            \
  uint32_t d0=a,d1=a+1,d2=a+2,d3=a+3,d4=a+4,d5=a+5,d6=a+6,d7=a+7,d8=a+8,      \
           d9=a+9,d10=a+10,d11=a+11,d12=a+12,d13=a+13,d14=a+14,d15=a+15;      \
  for (int i = 0; i < ITERS; ++i) {                                            \
    asm volatile(                                                              \
      INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)  \
      INSTR(8) INSTR(9) INSTR(10) INSTR(11) INSTR(12) INSTR(13) INSTR(14) INSTR(15) \
      : "+v"(d0),"+v"(d1),"+v"(d2),"+v"(d3),"+v"(d4),"+v"(d5),"+v"(d6),"+v"(d7),\
        "+v"(d8),"+v"(d9),"+v"(d10),"+v"(d11),"+v"(d12),"+v"(d13),"+v"(d14),"+v"(d15) \
      : "v"(a), "v"(b) : "vcc");                                               \
  }                                                                            \
  out[blockIdx.x * blockDim.x + threadIdx.x] = d0^d1^d2^d3^d4^d5^d6^d7^d8^d9^d10^d11^d12^d13^d14^d15; \
}
#define S(x) #x
#define XS(x) S(x)
#define I_MULLO(k)  "v_mul_lo_u32 %" XS(k) ", %16, %" XS(k) "\n"
#define I_MULHI(k)  "v_mul_hi_u32 %" XS(k) ", %16, %" XS(k) "\n"
#define I_MUL24(k)  "v_mul_u32_u24 %" XS(k) ", %16, %" XS(k) "\n"
#define I_MULHI24(k) "v_mul_hi_u32_u24 %" XS(k) ", %16, %" XS(k) "\n"
#define I_MAD24(k)  "v_mad_u32_u24 %" XS(k) ", %16, %17, %" XS(k) "\n"
#define I_ADD(k)    "v_add_u32 %" XS(k) ", %16, %" XS(k) "\n"
#define I_ADDCO(k)  "v_add_co_u32 %" XS(k) ", vcc, %16, %" XS(k) "\n"
#define I_ADDC(k)   "v_addc_co_u32 %" XS(k) ", vcc, %16, %" XS(k) ", vcc\n"
#define I_ADD3(k)   "v_add3_u32 %" XS(k) ", %16, %17, %" XS(k) "\n"
#define I_ALIGN(k)  "v_alignbit_b32 %" XS(k) ", %16, %" XS(k) ", 7\n"
#define I_BITOP3(k) "v_bitop3_b32 %" XS(k) ", %16, %17, %" XS(k) " bitop3:0x96\n"
#define I_XOR(k)    "v_xor_b32 %" XS(k) ", %16, %" XS(k) "\n"
#define I_CNDMASK(k) "v_cndmask_b32 %" XS(k) ", %16, %" XS(k) ", vcc\n"
K32(k_mullo, I_MULLO)
K32(k_mulhi, I_MULHI)
K32(k_mul24, I_MUL24)
K32(k_mulhi24, I_MULHI24)
K32(k_mad24, I_MAD24)
K32(k_add, I_ADD)
K32(k_addco, I_ADDCO)
K32(k_addc, I_ADDC)
K32(k_add3, I_ADD3)
K32(k_align, I_ALIGN)
K32(k_bitop3, I_BITOP3)
K32(k_xor, I_XOR)
K32(k_cndmask, I_CNDMASK)

// 64-bit accumulator forms: 8 independent 64-bit chains per asm
#define K64(NAME, INSTR)                                                       \
__global__ void NAME(uint64_t* out, uint32_t seed) {                           \
  uint32_t a = seed + threadIdx.x, b = a * 3u + 1u;                            \
  uint64_t a64 = ((uint64_t)b << 32) | a;                                      \
  uint64_t d0=a64,d1=a64+1,d2=a64+2,d3=a64+3,d4=a64+4,d5=a64+5,d6=a64+6,d7=a64+7; \
  uint64_t d8=a64+8,d9=a64+9,d10=a64+10,d11=a64+11,d12=a64+12,d13=a64+13,d14=a64+14,d15=a64+15; \
  for (int i = 0; i < ITERS; ++i) {                                            \
    asm volatile(                                                              \
      INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)  \
      INSTR(8) INSTR(9) INSTR(10) INSTR(11) INSTR(12) INSTR(13) INSTR(14) INSTR(15) \
      : "+v"(d0),"+v"(d1),"+v"(d2),"+v"(d3),"+v"(d4),"+v"(d5),"+v"(d6),"+v"(d7),\
        "+v"(d8),"+v"(d9),"+v"(d10),"+v"(d11),"+v"(d12),"+v"(d13),"+v"(d14),"+v"(d15) \
      : "v"(a), "v"(b), "v"(a64) : "vcc");                                     \
  }                                                                            \
  out[blockIdx.x * blockDim.x + threadIdx.x] = d0^d1^d2^d3^d4^d5^d6^d7^d8^d9^d10^d11^d12^d13^d14^d15; \
}
#define I_MAD64(k)  "v_mad_u64_u32 %" XS(k) ", vcc, %16, %17, %" XS(k) "\n"
#define I_LSHLADD64(k) "v_lshl_add_u64 %" XS(k) ", %" XS(k) ", 0, %18\n"
#define I_FMA64(k)  "v_fma_f64 %" XS(k) ", %18, %18, %" XS(k) "\n"
#define I_LSHR64(k) "v_lshrrev_b64 %" XS(k) ", 3, %" XS(k) "\n"
K64(k_mad64, I_MAD64)
K64(k_lshladd64, I_LSHLADD64)
K64(k_fma64, I_FMA64)
K64(k_lshr64, I_LSHR64)

template <typename T>
static int run(const char* name, void (*kern)(T*, uint32_t), T* buf, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, 1u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, 1u);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
  double lane_ops = 5.0 * blocks * threads * (double)ITERS * 16;
  double rate = lane_ops / (ms * 1e-3);
  printf("%-14s %8.3f ms  %7.2f T lane-ops/s  (%.3f of 78.64T = 256CU*4SIMD*32lanes*2.4GHz)\n",
         name, ms, rate / 1e12, rate / 78.6432e12);
  return 0;
}

int main(int argc, char** argv) {
  int waves_per_simd = argc > 1 ? atoi(argv[1]) : 2;
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d clock=%d kHz waves/SIMD=%d\n", p.gcnArchName, p.multiProcessorCount, p.clockRate, waves_per_simd);
  int threads = 256; int blocks = p.multiProcessorCount * waves_per_simd;  // 256 thr = 4 waves = 1 per SIMD
  uint32_t* b32; uint64_t* b64;
  CHK(hipMalloc(&b32, sizeof(uint32_t) * blocks * threads));
  CHK(hipMalloc(&b64, sizeof(uint64_t) * blocks * threads));
  run("mul_lo_u32", k_mullo, b32, blocks, threads);
  run("mul_hi_u32", k_mulhi, b32, blocks, threads);
  run("mul_u32_u24", k_mul24, b32, blocks, threads);
  run("mul_hi_u32_u24", k_mulhi24, b32, blocks, threads);
  run("mad_u32_u24", k_mad24, b32, blocks, threads);
  run("add_u32", k_add, b32, blocks, threads);
  run("add_co_u32", k_addco, b32, blocks, threads);
  run("addc_co_u32", k_addc, b32, blocks, threads);
  run("add3_u32", k_add3, b32, blocks, threads);
  run("alignbit_b32", k_align, b32, blocks, threads);
  run("bitop3_b32", k_bitop3, b32, blocks, threads);
  run("xor_b32", k_xor, b32, blocks, threads);
  run("cndmask_b32", k_cndmask, b32, blocks, threads);
  run("mad_u64_u32", k_mad64, b64, blocks, threads);
  run("lshl_add_u64", k_lshladd64, b64, blocks, threads);
  run("fma_f64", k_fma64, b64, blocks, threads);
  run("lshrrev_b64", k_lshr64, b64, blocks, threads);
  return 0;
}
