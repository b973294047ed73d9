// nw_runtime.h — internal runtime helpers shared by nw_api.cpp and nw_jobs.cpp (not part of
// the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace nw {
namespace rt {

// Initialise the library (idempotent): 0, or a negative NW_E_* with the error text set.
int ensure_init();
// Make the calling thread's selected device (nw_set_device) current for HIP; returns 0 and
// the library device index, or a negative NW_E_*.
int select_device(int* dev_index);
// Record the calling thread's last error (nw_last_error) and return `code`.
int set_err(int code, const char* what, hipError_t e = hipSuccess);
// Fill buf from the OS CSPRNG (getrandom).
int os_random(void* buf, size_t n);

}  // namespace rt
}  // namespace nw
