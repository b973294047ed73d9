/*
 * nw_dalek.h — TEST INFRASTRUCTURE ONLY: the timed CPU baseline, a dalek-equivalent
 * restatement of the reference's verify / verify_batch (nw_dalek.c). Same signatures and
 * status codes as the checker's nwo_* entries in nw_oracle.h; built into libnw_oracle.so.
 */
#ifndef NW_DALEK_H
#define NW_DALEK_H
#include <stddef.h>
#include <stdint.h>
#include "nw_oracle.h"
#ifdef __cplusplus
extern "C" {
#endif

int nwd_verify_strict(const uint8_t* msg, size_t len, const uint8_t pk[32],
                      const uint8_t sig[64]);
void nwd_verify_strict_many(const uint8_t* msgs, size_t msg_stride, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, int32_t* status, int nthreads);
int nwd_verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs,
                     size_t n, const uint8_t* z16, size_t* fail_index);
void nwd_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                           const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                           int32_t* status, int nthreads);
/* encode([a]A + [b]B) through vartime_double_scalar_mul_basepoint; 0 if A does not decode */
int nwd_double_base(const uint8_t a[32], const uint8_t A[32], const uint8_t b[32],
                    uint8_t out[32]);
/* Certificate::verify / Header::verify over a packed stream with the message checks of
 * nw_oracle.c and the signature checks above (nwo_certificates_verify_many's layout). */
void nwd_certificates_verify_many(const nwo_committee* c, const uint8_t* header_bytes,
                                  const uint64_t* header_offsets, const uint32_t* payload_counts,
                                  const uint8_t* ids, const uint8_t* header_sigs,
                                  const uint64_t* vote_offsets, const uint8_t* vote_pks,
                                  const uint8_t* vote_sigs, size_t n, const uint8_t* z16,
                                  int headers_only, int32_t* status, uint64_t* index,
                                  int nthreads);

#ifdef __cplusplus
}
#endif
#endif
