// nw_host.h — the engine's host verification path (nw_host.cpp): the kernels' own NW_HD
// arithmetic (nw_field / nw_point / nw_scalar / nw_strict / nw_ladder.hpp) compiled for the
// CPU, behind the same semantics as the device entry points. Used by the aggregation
// service's hedge (nw_service.cpp): a request whose device job has not answered within the
// service's deadline is verified here as well, and the first verdict wins. Never chosen
// implicitly by a device entry point (those fail with NW_E_NO_DEVICE without a GPU).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "narwhal_amd.h"

namespace nw {
namespace host {

// A committee prepared for host verification: config::Committee (config/src/lib.rs:139-173)
// plus, per key, its decompression flags (nw_strict.hpp kKeyDecoded / kKeySmall / lambda)
// and its 8-bit comb tables j * 2^(8 t) A (t < 32, j <= 128, affine niels: 495 KB per key),
// so a keyed check is 64 mixed additions with no doublings.
struct Committee;
// Builds it (about 2-5 ms of one core per key); nullptr on allocation failure.
Committee* committee_new(const nw_committee* c);
void committee_free(Committee* c);

// crypto::Signature::verify (crypto/src/lib.rs:200-204) of a 32-byte digest: NW_OK or the
// NW_ERR_* of the first failing check (the kernels' strict ladder, nw_strict.hpp).
int verify_strict(const uint8_t msg32[32], const uint8_t pk[32], const uint8_t sig[64]);
// crypto::Signature::verify_batch (crypto/src/lib.rs:206-219): status, *fail_index (item or
// n for the equation). z16: n x 16-byte coefficients, or nullptr for ChaCha20 keyed from the
// OS CSPRNG. com (optional): votes whose key is a committee member take the keyed check.
int verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                 const uint8_t* z16, const Committee* com, uint64_t* fail_index);
// Header::verify / Vote::verify / Certificate::verify (primary/src/messages.rs:48-67,
// 131-142, 189-215): NW_DAG_* status and index exactly as nw_certificates_verify_many.
int header_verify(const Committee& c, const uint8_t* hb, size_t hlen, uint32_t np,
                  const uint8_t id[32], const uint8_t sig[64], uint64_t* index);
int vote_verify(const Committee& c, const uint8_t id[32], uint64_t round,
                const uint8_t origin[32], const uint8_t author[32], const uint8_t sig[64]);
int certificate_verify(const Committee& c, const uint8_t* hb, size_t hlen, uint32_t np,
                       const uint8_t id[32], const uint8_t hsig[64], const uint8_t* vote_pks,
                       const uint8_t* vote_sigs, size_t nvotes, const uint8_t* z16,
                       uint64_t* index);

}  // namespace host
}  // namespace nw
