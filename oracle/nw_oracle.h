/*
 * nw_oracle.h — CPU restatement of Narwhal's crypto hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity oracle and the CPU baseline for the MI355X engine in
 * narwhal_amd/. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it. The product library (libnarwhal_amd.so) never links or calls it.
 *
 * What it restates (the reference is Rust and cannot be built in this image, see
 * DESIGN.md "Oracle"):
 *   - crypto::Signature::verify        /root/reference/crypto/src/lib.rs:200-204
 *       -> ed25519 1.x Signature::from_bytes (s high-bit check), dalek 1.0.1
 *          PublicKey::from_bytes (decompress A), PublicKey::verify_strict [ext].
 *   - crypto::Signature::verify_batch  /root/reference/crypto/src/lib.rs:206-219
 *       -> per vote from_bytes/decompress (fail fast), dalek 1.0.1 verify_batch [ext]
 *          (cofactorless random linear combination). z_i may be injected.
 *   - Sha512(..)[..32] digests         /root/reference/worker/src/processor.rs:38,
 *                                      /root/reference/primary/src/messages.rs:70-84,145-153,226-234
 *   - fixture generation: rand 0.7 StdRng (ChaCha20) + dalek Keypair::generate and
 *     RFC 8032 signing (/root/reference/crypto/src/lib.rs:167-191,
 *     /root/reference/crypto/src/tests/crypto_tests.rs:26-29).
 * [ext] = third-party crate behaviour (ed25519-dalek 1.0.1 / curve25519-dalek 3.x /
 * sha2 0.9), not vendored in /root/reference; restated from the published algorithm,
 * see SURVEY.md Appendix A.
 *
 * Pinning: tests/test_oracle.py checks this library against hashlib (SHA-512),
 * libsodium 1.0.18 (strict verify, signing, ChaCha20), the SURVEY Appendix B fixture
 * values and the RFC 8032 test vectors committed in tests/golden/.
 */
#ifndef NW_ORACLE_H
#define NW_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Per-item status codes; identical numbering to include/narwhal_amd.h. */
enum {
  NWO_OK = 0,
  NWO_ERR_S_HIGH_BITS = 1,     /* sig[63] & 0xE0 != 0 (ed25519 crate from_bytes)        */
  NWO_ERR_S_NONCANONICAL = 2,  /* s >= l (dalek check_scalar)                            */
  NWO_ERR_A_DECODE = 3,        /* public key does not decompress                         */
  NWO_ERR_R_DECODE = 4,        /* R does not decompress                                  */
  NWO_ERR_A_SMALL_ORDER = 5,   /* strict only                                            */
  NWO_ERR_R_SMALL_ORDER = 6,   /* strict only                                            */
  NWO_ERR_EQUATION = 7         /* [s]B != R + [k]A (strict) / RLC sum != identity (batch) */
};

/* SHA-512 (FIPS 180-4). */
void nwo_sha512(const uint8_t* msg, size_t len, uint8_t out[64]);
/* Digest(Sha512(msg_i)[..32]) for n messages at data+offsets[i], lengths[i]. */
void nwo_sha512_digest32_many(const uint8_t* data, const uint64_t* offsets,
                              const uint64_t* lengths, size_t n, uint8_t* out32,
                              int nthreads);

/* ChaCha20 (DJB: 64-bit counter, 64-bit nonce) keystream = rand_chacha 0.2 StdRng. */
void nwo_chacha20_keystream(const uint8_t key[32], const uint8_t nonce[8],
                            uint64_t counter, uint8_t* out, size_t len);

/* dalek Keypair from a 32-byte seed: pk = encode([clamp(H(seed)[0..32])]B). */
void nwo_keypair_from_seed(const uint8_t seed[32], uint8_t pk[32], uint8_t sk[64]);
/* RFC 8032 / dalek ExpandedSecretKey::sign; sk = seed || pk (crypto::SecretKey). */
void nwo_sign(const uint8_t sk[64], const uint8_t* msg, size_t len, uint8_t sig[64]);
/* Signing with an explicit secret scalar a, nonce prefix and public-key BYTES (used to
 * build mixed-order / non-canonical key fixtures). */
void nwo_sign_raw(const uint8_t a[32], const uint8_t prefix[32], const uint8_t A[32],
                  const uint8_t* msg, size_t len, uint8_t sig[64]);

/* crypto::Signature::verify semantics; returns NWO_* status. */
int nwo_verify_strict(const uint8_t* msg, size_t len, const uint8_t pk[32],
                      const uint8_t sig[64]);
/* Many 32-byte-message strict verifies; msg_stride 0 = one shared digest. */
void nwo_verify_strict_many(const uint8_t* msgs, size_t msg_stride, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, int32_t* status,
                            int nthreads);

/* crypto::Signature::verify_batch(digest, votes). z16 = n x 16-byte LE 128-bit
 * coefficients (NULL: fresh random from getrandom + ChaCha20). Returns NWO_* status of
 * the first failure in reference order; *fail_index (may be NULL) gets the item index
 * for per-item failures, or n for the equation. Empty input -> NWO_OK. */
int nwo_verify_batch(const uint8_t digest[32], const uint8_t* pks, const uint8_t* sigs,
                     size_t n, const uint8_t* z16, size_t* fail_index);
/* Same, over many independent batches (one per thread). */
void nwo_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                           const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                           int32_t* status, int nthreads);

/* ---- point / scalar helpers for building fixtures and checking kernels ---- */
/* Decompress with curve25519-dalek 3 semantics: 1 ok, 0 fail. out = canonical re-encoding. */
int nwo_decompress(const uint8_t in[32], uint8_t out_canonical[32]);
/* 1 if decompresses and 8*P == identity. -1 if it does not decompress. */
int nwo_is_small_order(const uint8_t in[32]);
/* k = SHA512(R||A||M) mod l. */
void nwo_hram(const uint8_t R[32], const uint8_t A[32], const uint8_t* msg, size_t len,
              uint8_t k[32]);
/* 64-byte LE -> mod l. */
void nwo_scalar_reduce64(const uint8_t in[64], uint8_t out[32]);
/* (a*b) mod l, (a+b) mod l, for 32-byte LE inputs (< 2^256). */
void nwo_scalar_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]);
void nwo_scalar_add(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]);
/* out = encode([s]B) (s any 256-bit LE). */
void nwo_scalarmult_base(const uint8_t s[32], uint8_t out[32]);
/* out = encode([s]P); returns 0 if P fails to decompress. */
int nwo_scalarmult(const uint8_t s[32], const uint8_t P[32], uint8_t out[32]);
/* out = encode(P + Q); returns 0 if either fails to decompress. */
int nwo_point_add(const uint8_t P[32], const uint8_t Q[32], uint8_t out[32]);
/* Multi-scalar mult sum s_i P_i over n points (compressed); 0 if any fails to decode.
 * The result is encoded in out; *is_identity set. */
int nwo_msm(const uint8_t* scalars, const uint8_t* points, size_t n, uint8_t out[32],
            int* is_identity);

/* ---- primary messages (primary/src/messages.rs:48-67, 131-153, 189-234) ---- */
/* DagError codes; identical numbering to include/narwhal_amd.h (NW_DAG_*). */
enum {
  NWO_DAG_INVALID_HEADER_ID = 16,
  NWO_DAG_UNKNOWN_AUTHORITY = 17,
  NWO_DAG_MALFORMED_HEADER = 18,
  NWO_DAG_AUTHORITY_REUSE = 19,
  NWO_DAG_REQUIRES_QUORUM = 20,
  NWO_DAG_INVALID_SIGNATURE = 32,   /* + NWO_ERR_* of the message's own signature    */
  NWO_DAG_INVALID_VOTES = 48        /* + NWO_ERR_* of verify_batch over the votes      */
};
/* config::Committee (config/src/lib.rs:139-173), keys sorted by bytes. */
typedef struct {
  size_t nauth;
  const uint8_t* pks;
  const uint32_t* stakes;
  const uint64_t* worker_offsets;
  const uint32_t* worker_ids;
} nwo_committee;
void nwo_digest_72(const uint8_t x[32], uint64_t round, const uint8_t y[32], uint8_t out[32]);
int nwo_header_verify(const nwo_committee* c, const uint8_t* hb, size_t hlen, uint32_t np,
                      const uint8_t id[32], const uint8_t sig[64], uint64_t* index);
int nwo_certificate_verify(const nwo_committee* c, const uint8_t* hb, size_t hlen,
                           uint32_t np, const uint8_t id[32], const uint8_t hsig[64],
                           const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t nvotes,
                           const uint8_t* z16, uint64_t* index);
void nwo_certificates_verify_many(const nwo_committee* c, const uint8_t* header_bytes,
                                  const uint64_t* header_offsets, const uint32_t* payload_counts,
                                  const uint8_t* ids, const uint8_t* header_sigs,
                                  const uint64_t* vote_offsets, const uint8_t* vote_pks,
                                  const uint8_t* vote_sigs, size_t n, const uint8_t* z16,
                                  int headers_only, int32_t* status, uint64_t* index,
                                  int nthreads);
void nwo_votes_verify_many(const nwo_committee* c, const uint8_t* ids, const uint64_t* rounds,
                           const uint8_t* origins, const uint8_t* authors, const uint8_t* sigs,
                           size_t n, int32_t* status);

#ifdef __cplusplus
}
#endif
#endif
