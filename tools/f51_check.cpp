// f51_check.cpp — test shim (not product code): the host path's five-51-bit-limb field
// (narwhal_amd/csrc/nw_host_f51.hpp) exported over a C ABI so tests/test_host_f51.py can
// check it against Python integers mod p, at the limb bounds the header states.
//   g++ -O2 -shared -fPIC -Inarwhal_amd/csrc tools/f51_check.cpp -o tools/libnw_f51check.so
#include "nw_host_f51.hpp"

using namespace nw::host::f51;

extern "C" {
// raw limbs in, canonical bytes out
void f51_mul(const uint64_t* a, const uint64_t* b, uint8_t* out) {
  fe x, y, r;
  memcpy(x.v, a, 40);
  memcpy(y.v, b, 40);
  mul(r, x, y);
  tobytes(out, r);
}
void f51_mul_limbs(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  fe x, y, r;
  memcpy(x.v, a, 40);
  memcpy(y.v, b, 40);
  mul(r, x, y);
  memcpy(out, r.v, 40);
}
void f51_sq(const uint64_t* a, uint8_t* out) {
  fe x, r;
  memcpy(x.v, a, 40);
  sq(r, x);
  tobytes(out, r);
}
void f51_sub(const uint64_t* a, const uint64_t* b, uint64_t* out) {
  fe x, y, r;
  memcpy(x.v, a, 40);
  memcpy(y.v, b, 40);
  sub(r, x, y);
  memcpy(out, r.v, 40);
}
void f51_tobytes(const uint64_t* a, uint8_t* out) {
  fe x;
  memcpy(x.v, a, 40);
  tobytes(out, x);
}
void f51_frombytes(const uint8_t* s, uint64_t* out) {
  fe x;
  frombytes(x, s);
  memcpy(out, x.v, 40);
}
void f51_invert(const uint8_t* s, uint8_t* out) {
  fe x, r;
  frombytes(x, s);
  invert(r, x);
  tobytes(out, r);
}
int f51_eq(const uint64_t* a, const uint64_t* b) {
  fe x, y;
  memcpy(x.v, a, 40);
  memcpy(y.v, b, 40);
  return eq(x, y) ? 1 : 0;
}
}
