// nw_kernels.h — launchers for the gfx950 kernels (host side of nw_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "narwhal_amd.h"

namespace nw {

struct z_key_t {
  uint32_t key[8];
  uint64_t nonce;
};

// Computes the curve constants and the B table on the host (from their definitions) and
// copies them to the current device's constant memory.
hipError_t upload_consts();

hipError_t launch_sha512_digest32(const uint8_t* data, const uint64_t* offsets,
                                  const uint64_t* lengths, uint64_t n, uint32_t* out,
                                  hipStream_t stream);

hipError_t launch_verify_strict(const uint32_t* msgs, uint32_t msg_stride_words,
                                const uint32_t* pks, const uint32_t* sigs, uint64_t n,
                                int32_t* status, uint64_t* bitmap, hipStream_t stream);

hipError_t launch_keypair(const uint32_t* seeds, uint64_t n, uint32_t* pks, hipStream_t stream);

hipError_t launch_sign(const uint32_t* sks, uint32_t sk_stride_words, const uint32_t* msgs,
                       uint32_t msg_stride_words, uint64_t n, uint32_t* sigs,
                       hipStream_t stream);

size_t batch_workspace_bytes(uint64_t nitems);

hipError_t launch_verify_batch(const uint32_t* digests, const uint64_t* offsets,
                               uint64_t nbatches, const uint32_t* pks, const uint32_t* sigs,
                               uint64_t nitems, const uint32_t* z16, const z_key_t& zkey,
                               void* workspace, int32_t* status, uint64_t* fail_index,
                               hipStream_t stream);

}  // namespace nw
