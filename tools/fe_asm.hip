// fe_asm.hip — isolated field-arithmetic kernels for reading the gfx950 instruction mix
// (hipcc --cuda-device-only -S, then tools/asm_mix.py). Not part of the product.
#include "nw_field.hpp"
using namespace nw;
__global__ void k_mul(const fe* a, const fe* b, fe* o) {
  int i = threadIdx.x;
  fe r;
  fe_mul(r, a[i], b[i]);
  o[i] = r;
}
__global__ void k_sq(const fe* a, fe* o) {
  int i = threadIdx.x;
  fe r;
  fe_sq(r, a[i]);
  o[i] = r;
}
