// permlane_probe.hip — prints the lane mapping of gfx950's v_permlane16_swap /
// v_permlane32_swap and of DPP row_shr / row_shl (bound_ctrl) for nw_lp.hpp's row moves.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(unsigned* o) {
  const unsigned x = threadIdx.x;
  const unsigned y = 100 + threadIdx.x;
  auto a = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  auto b = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  o[0 * 64 + x] = a[0];
  o[1 * 64 + x] = a[1];
  o[2 * 64 + x] = b[0];
  o[3 * 64 + x] = b[1];
  o[4 * 64 + x] = (unsigned)__builtin_amdgcn_mov_dpp((int)y, 0x113, 0xf, 0xf, true);  // row_shr:3
  o[5 * 64 + x] = (unsigned)__builtin_amdgcn_mov_dpp((int)y, 0x103, 0xf, 0xf, true);  // row_shl:3
}

int main() {
  unsigned* d;
  if (hipMalloc(&d, 6 * 64 * 4) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[6 * 64];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* names[6] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]", "shr3", "shl3"};
  for (int r = 0; r < 6; ++r) {
    printf("%s:", names[r]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[r * 64 + l]);
    printf("\n");
  }
  (void)hipFree(d);
  return 0;
}
