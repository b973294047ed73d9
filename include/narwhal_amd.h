/*
 * narwhal_amd.h — C ABI of the MI355X (gfx950) verification engine for Narwhal's `crypto`
 * crate hot path. Plain pointers and sizes only; thread-safe; no exceptions or aborts
 * cross this boundary.
 *
 * Reference interface each entry point replaces (paths under /root/reference):
 *   nw_signature_verify          crypto/src/lib.rs:200-204  Signature::verify(&Digest, &PublicKey)
 *   nw_signature_verify_batch    crypto/src/lib.rs:206-219  Signature::verify_batch(&Digest, votes)
 *   nw_verify_strict_many        crypto/src/lib.rs:200-204  (bulk form of verify, for the
 *                                primary's header/vote stream, primary/src/core.rs:306-336)
 *   nw_verify_batch_many         crypto/src/lib.rs:206-219  (bulk form of verify_batch, one
 *                                batch per certificate, primary/src/messages.rs:214)
 *   nw_sha512_digest32_many      worker/src/processor.rs:38, worker/src/batch_maker.rs:124-128,
 *                                primary/src/messages.rs:70-84,145-153,226-234
 *                                (Digest(Sha512::digest(bytes)[..32]))
 *   nw_dev_*                     the same work on device-resident buffers, asynchronous on a
 *                                caller stream (hipStream_t passed as void*)
 *
 * Return values: 0 (NW_OK) = valid / success; positive NW_ERR_* = the item is invalid
 * (the reference's CryptoError, with the first failing check named); negative NW_E_* =
 * runtime/device error, never conflated with "invalid". There is no CPU fallback: on a
 * host without a usable gfx950 device every call returns NW_E_NO_DEVICE.
 */
#ifndef NARWHAL_AMD_H
#define NARWHAL_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NW_ABI_VERSION 1

/* Per-item verdicts (check order = the reference's, see DESIGN.md "Semantics"). */
#define NW_OK 0
#define NW_ERR_S_HIGH_BITS 1      /* sig[63] & 0xE0 (ed25519::Signature::from_bytes)        */
#define NW_ERR_S_NONCANONICAL 2   /* s >= l (dalek check_scalar)                            */
#define NW_ERR_A_DECODE 3         /* public key does not decompress                         */
#define NW_ERR_R_DECODE 4         /* R does not decompress                                  */
#define NW_ERR_A_SMALL_ORDER 5    /* verify (strict) only                                   */
#define NW_ERR_R_SMALL_ORDER 6    /* verify (strict) only                                   */
#define NW_ERR_EQUATION 7         /* strict: [s]B != R + [k]A; batch: RLC sum != identity   */

/* Message-level verdicts (primary::DagError variants, primary/src/error.rs:26-59), returned
 * per item by the Header / Vote / Certificate entry points below. */
#define NW_DAG_INVALID_HEADER_ID 16      /* DagError::InvalidHeaderId                        */
#define NW_DAG_UNKNOWN_AUTHORITY 17      /* DagError::UnknownAuthority(pk)                   */
#define NW_DAG_MALFORMED_HEADER 18       /* DagError::MalformedHeader(id): unknown worker id */
#define NW_DAG_AUTHORITY_REUSE 19        /* DagError::AuthorityReuse(pk)                     */
#define NW_DAG_REQUIRES_QUORUM 20        /* DagError::CertificateRequiresQuorum              */
#define NW_DAG_SERIALIZATION 21          /* DagError::SerializationError: the frame does not
                                            bincode-decode as a PrimaryMessage             */
/* DagError::InvalidSignature(CryptoError): base + the NW_ERR_* of the first failing check.
 * NW_DAG_INVALID_SIGNATURE: the message's own Signature::verify (header or vote);
 * NW_DAG_INVALID_VOTES: the certificate's Signature::verify_batch over its votes. */
#define NW_DAG_INVALID_SIGNATURE 32
#define NW_DAG_INVALID_VOTES 48

/* Runtime errors. */
#define NW_E_INVALID_ARG (-1)
#define NW_E_NO_DEVICE (-2)
#define NW_E_DEVICE (-3)
#define NW_E_OUT_OF_MEMORY (-4)

/* ---- runtime ----------------------------------------------------------------------- */
/* Initialise every visible gfx950 device (idempotent). Returns the device count (>0) or a
 * negative NW_E_*. All other calls initialise lazily. */
int nw_init(void);
/* Number of usable devices (0 if none). */
int nw_device_count(void);
/* Device used by the calling thread's calls (default 0). NW_ALL_DEVICES: the calling
 * thread's host-buffer calls (nw_submit_*, the blocking calls built on them, and the
 * Header / Vote / Certificate host calls) split their items into contiguous parts, one per
 * device, run them concurrently on per-device streams and merge the outputs in order, so
 * one process (Narwhal's single Core task, primary/src/core.rs:338-346) drives every GPU;
 * the nw_dev_* calls (device pointers) then fail with NW_E_INVALID_ARG. */
#define NW_ALL_DEVICES (-1)
int nw_set_device(int device);
int nw_get_device(void);
/* Human-readable description of the calling thread's last error ("" if none). */
const char* nw_last_error(void);
/* "narwhal_amd <version> gfx950". */
const char* nw_version(void);
/* Wait for all work this thread queued on its device stream. */
int nw_synchronize(void);
/* Build, now, the per-device tables the engine otherwise builds on first use, on the
 * calling thread's device, or on every device under NW_ALL_DEVICES: the strict kernel's B
 * tables (2 x 8,388,609 entries of 128 B = 2.15 GB, ~0.2 s) and the keyed comb's B tables
 * (11 x 8,388,609 entries = 11.8 GB, ~0.7 s). Besides these a device holds, per committee
 * in use, its key tables (committees of up to 64 keys: 20-bit combs, 14 x 524,289 entries
 * = 940 MB per key, 47 GB at 50 authorities; larger ones: 16-bit combs, 16 x 32,769 entries
 * = 67 MB per key, 6.7 GB at 100 authorities; NW_KEY_WIDTH=16 forces the small ones; built
 * by the first Header / Vote / Certificate call with that committee, ~0.4 s at N = 100) and
 * the strict workspace (~1.9 GB): ~22 GB in all at N = 100. Returns 0, or
 * NW_E_OUT_OF_MEMORY when a table does not fit; without the keyed comb or a committee's key
 * tables, Header / Vote / Certificate calls still run, unkeyed (the strict ladder and
 * per-certificate verify_batch: same verdicts, lower throughput). Optional: keeps the first
 * verification's latency low. hipGraph capture: nw_dev_sha512_digest32_many,
 * nw_dev_keypair_from_seed_many and nw_dev_sign_many may be captured (after one
 * uncaptured call on the device); strict / Header / Vote / Certificate launches share
 * per-device tables under an event chain that a graph replay would bypass, so they return
 * NW_E_INVALID_ARG on a capturing stream. */
int nw_prepare(void);

/* ---- host-buffer (blocking) entry points: the drop-in ------------------------------ */

/* Digest(Sha512(m_i)[..32]) for n messages at data + offsets[i], lengths[i] bytes.
 * out32: n x 32 bytes. */
int nw_sha512_digest32_many(const uint8_t* data, const uint64_t* offsets,
                            const uint64_t* lengths, size_t n, uint8_t* out32);

/* crypto::Signature::verify: sig = part1 (R) || part2 (s), 64 bytes; digest 32 bytes;
 * pk 32 bytes. Returns NW_OK, an NW_ERR_* code, or a negative runtime error. */
int nw_signature_verify(const uint8_t sig[64], const uint8_t digest[32], const uint8_t pk[32]);

/* n strict verifications. digests: n x 32 bytes (digest_stride = 32) or one shared digest
 * (digest_stride = 0). status_out (optional): n x int32 verdicts. bitmap_out (optional):
 * ceil(n/8) bytes, bit i (LSB-first) set iff item i is valid. */
int nw_verify_strict_many(const uint8_t* digests, size_t digest_stride, const uint8_t* pks,
                          const uint8_t* sigs, size_t n, int32_t* status_out,
                          uint8_t* bitmap_out);

/* crypto::Signature::verify_batch(digest, votes) over n (pk, sig) pairs sharing one digest.
 * z16: optional n x 16-byte little-endian 128-bit coefficients (deterministic tests); NULL =
 * fresh coefficients from the OS CSPRNG (the reference draws them from thread_rng).
 * Returns NW_OK (also for n == 0), the first failing check in reference order, or a
 * negative runtime error. fail_index (optional): failing item, or n for the equation. */
int nw_signature_verify_batch(const uint8_t digest[32], const uint8_t* pks,
                              const uint8_t* sigs, size_t n, const uint8_t* z16,
                              size_t* fail_index);

/* nbatches independent verify_batch calls. Batch b = items [offsets[b], offsets[b+1]) of
 * pks/sigs (and z16 if given) with digest digests + 32 b. status_out: nbatches x int32. */
int nw_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                         const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                         int32_t* status_out);

/* crypto::generate_keypair given the CSPRNG's 32-byte seeds (crypto/src/lib.rs:167-175:
 * dalek Keypair::generate fills the seed from the RNG): pks_out n x 32 bytes. The
 * crypto::SecretKey bytes are seed || pk. */
int nw_keypair_from_seed_many(const uint8_t* seeds, size_t n, uint8_t* pks_out);

/* crypto::Signature::new(digest, secret) (crypto/src/lib.rs:185-191, RFC 8032). sks: n x 64
 * bytes (seed || pk) or one shared key (sk_stride = 0); digests: n x 32 (digest_stride 32)
 * or shared (0). sigs_out: n x 64 bytes (part1 || part2). */
int nw_sign_many(const uint8_t* sks, size_t sk_stride, const uint8_t* digests,
                 size_t digest_stride, size_t n, uint8_t* sigs_out);

/* ---- asynchronous host-buffer entry points (submit / poll) ------------------------- */
/* The non-blocking form of the calls above, for callers that must not block their event
 * loop (the reference's primary Core and worker Processor are tokio tasks, node/Cargo.toml:8;
 * crypto::SignatureService, crypto/src/lib.rs:222-250, is its own async-service pattern).
 * Submit copies the inputs into pinned staging memory (input buffers may be reused as soon
 * as it returns), queues H2D + kernels + D2H on the job's own stream and returns. The output
 * buffers must stay valid until nw_job_poll returns 1 or nw_job_wait returns: that is when
 * the library writes them. A job is used by one thread at a time; jobs are independent.
 * The blocking calls above are exactly submit + wait + release. */
typedef struct nw_job nw_job;
struct nw_committee;
struct nw_certificates;

/* Signature::verify over n items (as nw_verify_strict_many). */
int nw_submit_verify_strict(const uint8_t* digests, size_t digest_stride, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, int32_t* status_out,
                            uint8_t* bitmap_out, nw_job** job);
/* Signature::verify_batch per batch (as nw_verify_batch_many; fail_index_out optional). */
int nw_submit_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                                const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                                int32_t* status_out, uint64_t* fail_index_out, nw_job** job);
/* Digest(Sha512(m)[..32]) (as nw_sha512_digest32_many). */
int nw_submit_sha512_digest32_many(const uint8_t* data, const uint64_t* offsets,
                                   const uint64_t* lengths, size_t n, uint8_t* out32,
                                   nw_job** job);
/* Header::verify / Vote::verify / Certificate::verify (as nw_headers_verify_many /
 * nw_votes_verify_many / nw_certificates_verify_many below; the committee and every array
 * are copied at submit). The non-blocking form of the primary's sanitize_header /
 * sanitize_vote / sanitize_certificate (primary/src/core.rs:306-346). A job of up to
 * NW_SMALL_MAX_SLOTS (default 65,536) signatures whose committee's key tables are built
 * (1..256 authorities, <= 128 votes per certificate) is ONE kernel launch reading its
 * inputs from the job's pinned buffer, only reading the shared tables, so such jobs run
 * concurrently; larger jobs (or a committee's first) run the bulk pipeline: per-device
 * committee key tables (kept across jobs while the committee is unchanged) and the shared
 * strict workspace, ordered by the device's lease. status_out is required. */
int nw_submit_certificates_verify_many(const struct nw_committee* committee,
                                       const struct nw_certificates* certs, const uint8_t* z16,
                                       int32_t* status_out, uint64_t* index_out, nw_job** job);
int nw_submit_headers_verify_many(const struct nw_committee* committee,
                                  const struct nw_certificates* headers, int32_t* status_out,
                                  uint64_t* index_out, nw_job** job);
int nw_submit_votes_verify_many(const struct nw_committee* committee, const uint8_t* ids,
                                const uint64_t* rounds, const uint8_t* origins,
                                const uint8_t* authors, const uint8_t* sigs, size_t n,
                                int32_t* status_out, nw_job** job);
/* 1 = done (outputs written), 0 = still running, < 0 = runtime error. Never blocks. */
int nw_job_poll(nw_job* job);
/* Block until done (outputs written): 0 or a runtime error. */
int nw_job_wait(nw_job* job);
/* Call fn(arg) once the job's device work has finished (e.g. to wake an async task, which
 * then calls nw_job_poll). fn runs on the library's own watcher thread, which polls a marker
 * event recorded behind the job (the job's stream never waits for fn); the callbacks of all
 * jobs run one after another on that thread, so fn must be short, and must not call into
 * this library. fn runs exactly once whenever this returns 0, and never when it returns an
 * error (on a fanned-out job: one part could not be armed; the parts already armed are
 * disarmed), so the caller may free arg and fall back to nw_job_wait. */
int nw_job_notify(nw_job* job, void (*fn)(void*), void* arg);
/* Return the job's buffers to the pool (waits first if it is still running). */
void nw_job_release(nw_job* job);
/* Diagnostics: Header / Vote / Certificate host-buffer jobs submitted so far by path, the
 * small-job launch (one kernel, no copies) and the bulk pipeline. Either pointer may be NULL. */
int nw_path_stats(uint64_t* small_jobs, uint64_t* pipeline_jobs);

/* ---- aggregation service: one request per message, coalesced into device jobs ------- */
/* The front end a crypto-gpu crate puts behind the primary's per-message checks: Core
 * verifies one Header / Vote / Certificate at a time (primary/src/core.rs:306-346,
 * sanitize_header / sanitize_vote / sanitize_certificate), and a certificate carries only
 * 3..67 signatures, so single calls are coalesced, the same request/reply shape as
 * crypto::SignatureService (crypto/src/lib.rs:222-250). Each request is copied at submit
 * into the open batch of its kind; a service thread submits a batch as ONE job (the
 * nw_submit_* calls above, so the committee's key tables stay on the device across jobs)
 * once it holds max_items units (certificate = 1 + votes, batch = its votes, else 1),
 * max_delay_us after its first request, or at once while no job is in flight (an idle
 * device gains nothing from waiting: the submitting caller's thread then submits the job
 * itself); among ready batches the one whose first request is oldest goes first; at most
 * max_inflight jobs are on the device at once (the next batch keeps filling meanwhile).
 * Small jobs (up to ~64k signatures) are single launches that do not wait for one another
 * (nw_path_stats). A second service thread waits for the jobs in
 * order and calls fn(arg, status, index) once per accepted request (or a hedge thread does,
 * nw_service_set_hedge): status / index as the
 * corresponding bulk call returns them (NW_DAG_* for messages, NW_ERR_* for verify /
 * verify_batch, index = the batch's fail index), or a negative NW_E_* if the job failed.
 * fn runs on that thread; it may submit new requests but must not call nw_service_drain or
 * nw_service_destroy. Submits are thread-safe and never wait for the device. The service
 * runs on the creating thread's nw_set_device() choice (NW_ALL_DEVICES: jobs fan out).
 * committee may be NULL for a service that only takes nw_service_verify / _verify_batch. */
typedef struct nw_service nw_service;
typedef void (*nw_verdict_fn)(void* arg, int32_t status, uint64_t index);
int nw_service_create(const struct nw_committee* committee, size_t max_items,
                      uint32_t max_delay_us, size_t max_inflight, nw_service** out);
/* Certificate::verify (primary/src/messages.rs:189-215): header fields as nw_certificates
 * row i (header_bytes = the bytes `Hash for Header` hashes), votes nvotes x (32 + 64). */
int nw_service_certificate(nw_service* s, const uint8_t* header_bytes, size_t header_len,
                           uint32_t payload_count, const uint8_t* id, const uint8_t* header_sig,
                           const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t nvotes,
                           nw_verdict_fn fn, void* arg);
/* Header::verify (primary/src/messages.rs:48-67). */
int nw_service_header(nw_service* s, const uint8_t* header_bytes, size_t header_len,
                      uint32_t payload_count, const uint8_t* id, const uint8_t* sig,
                      nw_verdict_fn fn, void* arg);
/* Vote::verify (primary/src/messages.rs:131-142). */
int nw_service_vote(nw_service* s, const uint8_t* id, uint64_t round, const uint8_t* origin,
                    const uint8_t* author, const uint8_t* sig, nw_verdict_fn fn, void* arg);
/* crypto::Signature::verify (crypto/src/lib.rs:200-204) of one 32-byte digest. */
int nw_service_verify(nw_service* s, const uint8_t* digest, const uint8_t* pk,
                      const uint8_t* sig, nw_verdict_fn fn, void* arg);
/* crypto::Signature::verify_batch (crypto/src/lib.rs:206-219) over n (pk, sig) pairs. */
int nw_service_verify_batch(nw_service* s, const uint8_t* digest, const uint8_t* pks,
                            const uint8_t* sigs, size_t n, nw_verdict_fn fn, void* arg);
/* Submit every queued request now (does not wait). */
int nw_service_flush(nw_service* s);
/* Flush and wait until the callback of every request accepted before the call returned. */
int nw_service_drain(nw_service* s);
/* Requests accepted and jobs submitted so far (either pointer may be NULL). */
int nw_service_stats(nw_service* s, uint64_t* requests, uint64_t* jobs);
/* Hedge (on by default: 1000 us, 6 threads, 512 units; NW_SERVICE_HEDGE_US / _THREADS /
 * _QUEUED change the defaults). A request whose verdict has not arrived deadline_us after
 * its batch's first request (its device job is late, or its batch still waits for a job
 * slot) is verified on the host as well (the nw_host_* path below: the kernels' arithmetic
 * compiled for the CPU, same statuses and indices, fresh CSPRNG coefficients), and the
 * first verdict is delivered: fn is still called exactly once per request, but then from
 * one of the `threads` hedge threads, possibly before requests accepted earlier. The hedge
 * threads take late requests oldest first while the device races them; a batch still
 * waiting for a job slot is taken for the host alone (never submitted) only while fewer than
 * max_queued units (certificate = 1 + votes, batch = its votes, else 1) wait for the host,
 * so a stall under load costs at most `threads` cores and the host never owes more than it
 * finishes quickly. deadline_us = 0 or threads = 0 turns hedging off. Why: the primary's Core
 * verifies inline on one task (primary/src/core.rs:338-346), so a late device job would
 * stall the primary. Header / vote / certificate requests are hedged once the committee's
 * host tables exist (built in the background at create, ~2-5 ms of a core per key). */
int nw_service_set_hedge(nw_service* s, uint32_t deadline_us, uint32_t threads,
                         uint64_t max_queued);
/* Requests queued for the hedge, requests the host answered first, batches the host took
 * whole before submission, and whether the committee's host tables are built (1) — until
 * then only verify / verify_batch requests are hedged (any pointer may be NULL). */
int nw_service_hedge_stats(nw_service* s, uint64_t* hedged, uint64_t* host_first,
                           uint64_t* host_only_batches, int* host_ready);
/* Drain, stop the service threads and free the service. */
void nw_service_destroy(nw_service* s);

/* ---- primary messages: Header / Vote / Certificate verification -------------------- */
/* config::Committee (config/src/lib.rs:139-173): authorities sorted by public-key bytes
 * (BTreeMap order), their stake (config::Stake = u32) and worker ids (WorkerId = u32). */
typedef struct nw_committee {
  size_t nauth;
  const uint8_t* pks;              /* nauth x 32, strictly increasing                     */
  const uint32_t* stakes;          /* nauth                                               */
  const uint64_t* worker_offsets;  /* nauth + 1: authority a owns worker_ids[wo[a]..wo[a+1]) */
  const uint32_t* worker_ids;
} nw_committee;

/* A stream of n primary::Certificate (or Header) values in structure-of-arrays form.
 * header_bytes holds, per header, exactly the bytes `Hash for Header` feeds SHA-512
 * (primary/src/messages.rs:70-84): author 32 || round u64 LE || payload_counts[i] x
 * (digest 32 || worker id u32 LE) in BTreeMap order || parents x 32 in BTreeSet order. */
typedef struct nw_certificates {
  size_t n;
  const uint8_t* header_bytes;
  const uint64_t* header_offsets;  /* n + 1; header i = header_bytes[ho[i]..ho[i+1])      */
  const uint32_t* payload_counts;  /* n                                                   */
  const uint8_t* ids;              /* n x 32: header.id as received                       */
  const uint8_t* header_sigs;      /* n x 64: header.signature (part1 || part2)           */
  const uint64_t* vote_offsets;    /* n + 1 (certificates only; NULL for headers)          */
  const uint8_t* vote_pks;         /* vote_offsets[n] x 32: certificate.votes[j].0         */
  const uint8_t* vote_sigs;        /* vote_offsets[n] x 64: certificate.votes[j].1         */
  size_t header_bytes_len;         /* total bytes of header_bytes (device entry points)    */
  size_t nvotes;                   /* vote_offsets[n] (device entry points)                */
  const uint64_t* host_vote_offsets; /* device entry points: host copy of vote_offsets
                                        (optional; NULL = read back, blocking)             */
} nw_certificates;

/* n x Certificate::verify(committee) (primary/src/messages.rs:189-215, with
 * Header::verify 48-67 and Signature::verify_batch over Certificate::digest 226-234).
 * status_out: n x int32 (0 = Ok, else NW_DAG_*), first failure in the reference's order.
 * index_out (optional): n x uint64 — the vote index for UNKNOWN_AUTHORITY (UINT64_MAX =
 * the header author) / AUTHORITY_REUSE / INVALID_VOTES (nvotes for the equation), the
 * payload entry for MALFORMED_HEADER, else 0. z16 (optional): vote_offsets[n] x 16-byte
 * batch coefficients (deterministic tests); NULL = OS CSPRNG as in the reference. */
int nw_certificates_verify_many(const nw_committee* committee, const nw_certificates* certs,
                                const uint8_t* z16, int32_t* status_out, uint64_t* index_out);

/* n x Header::verify(committee) (primary/src/messages.rs:48-67); vote fields ignored. */
int nw_headers_verify_many(const nw_committee* committee, const nw_certificates* headers,
                           int32_t* status_out, uint64_t* index_out);

/* n x Vote::verify(committee) (primary/src/messages.rs:131-142): stake(author) > 0, then
 * Signature::verify(Vote::digest = Sha512(id || round LE || origin)[..32], author). */
int nw_votes_verify_many(const nw_committee* committee, const uint8_t* ids,
                         const uint64_t* rounds, const uint8_t* origins,
                         const uint8_t* authors, const uint8_t* sigs, size_t n,
                         int32_t* status_out);

/* ---- wire-format ingest ------------------------------------------------------------- */
/* primary::PrimaryMessage variants (primary/src/primary.rs:32-38). */
#define NW_MSG_HEADER 0
#define NW_MSG_VOTE 1
#define NW_MSG_CERTIFICATE 2
#define NW_MSG_CERTIFICATES_REQUEST 3

/* n frames as the primary's receiver gets them (PrimaryReceiverHandler::dispatch,
 * primary/src/primary.rs:224-240): frame i = frames[offsets[i]..offsets[i+1]), each a
 * bincode-serialized PrimaryMessage. Decoded natively (bincode 1.3 fixint LE; PublicKey as a
 * base64 string, crypto/src/lib.rs:94-112; payload/parents re-sorted and de-duplicated as
 * BTreeMap/BTreeSet deserialisation does) and verified with the check each variant gets:
 * Header::verify, Vote::verify, Certificate::verify (primary/src/messages.rs). status_out:
 * n x int32 (0 = Ok, NW_DAG_* as for the calls above, NW_DAG_SERIALIZATION for a frame that
 * does not decode; CertificatesRequest frames are only decoded, status 0). kind_out
 * (optional): n x int32 NW_MSG_* or -1. index_out (optional): as nw_certificates_verify_many
 * (0 for votes). Batch coefficients come from the OS CSPRNG. */
int nw_primary_messages_verify_wire(const nw_committee* committee, const uint8_t* frames,
                                    const uint64_t* offsets, size_t n, int32_t* kind_out,
                                    int32_t* status_out, uint64_t* index_out);
/* Decode only (host code, no device needed): kind_out n x int32 as above; counts_out
 * (optional) n x 3 uint64: payload entries and parents after BTreeMap/BTreeSet
 * de-duplication, and votes (Header/Certificate); digests requested (CertificatesRequest). */
int nw_primary_messages_scan(const uint8_t* frames, const uint64_t* offsets, size_t n,
                             int32_t* kind_out, uint64_t* counts_out);

/* ---- device-pointer (asynchronous) entry points ------------------------------------ */
/* All pointers are device pointers on the current device; work is queued on `stream`
 * (a hipStream_t; NULL = the library's per-thread stream) and the call returns without
 * waiting. */
int nw_dev_sha512_digest32_many(const void* data, const uint64_t* offsets,
                                const uint64_t* lengths, size_t n, void* out32, void* stream);

int nw_dev_verify_strict_many(const void* digests, size_t digest_stride, const void* pks,
                              const void* sigs, size_t n, int32_t* status_out,
                              void* bitmap_out, void* stream);

int nw_dev_keypair_from_seed_many(const void* seeds, size_t n, void* pks_out, void* stream);

int nw_dev_sign_many(const void* sks, size_t sk_stride, const void* digests,
                     size_t digest_stride, size_t n, void* sigs_out, void* stream);

/* Workspace bytes nw_dev_verify_batch_many needs for nbatches batches of nitems votes in
 * total (bounded: large calls are processed in slices of ~4M votes; a single batch may not
 * exceed one slice). */
size_t nw_dev_verify_batch_workspace(size_t nbatches, size_t nitems);
/* offsets: device copy of the nbatches + 1 batch boundaries (offsets[0] = 0,
 * offsets[nbatches] = nitems); host_offsets: the same values in host memory, used to plan
 * the launch (NULL: read back from the device, which blocks until the stream is idle).
 * z16 NULL: coefficients drawn on the device from ChaCha20 keyed by zkey32 (32 bytes from
 * the OS CSPRNG if zkey32 is NULL). fail_index (optional, device): nbatches x uint64. */
int nw_dev_verify_batch_many(const void* digests, const void* pks, const void* sigs,
                             const uint64_t* offsets, const uint64_t* host_offsets,
                             size_t nbatches, size_t nitems, const void* z16,
                             const uint8_t* zkey32, void* workspace, int32_t* status_out,
                             uint64_t* fail_index, void* stream);

/* Device form of nw_certificates_verify_many: every pointer inside *committee and *certs
 * (and z16, status_out, index_out, workspace) is a device pointer; the structs themselves
 * are host memory. header_bytes_len and nvotes must be set. headers_only != 0 runs
 * Header::verify instead of Certificate::verify. */
size_t nw_dev_certificates_workspace(size_t n, size_t nvotes);
int nw_dev_certificates_verify_many(const nw_committee* committee, const nw_certificates* certs,
                                    int headers_only, const void* z16, const uint8_t* zkey32,
                                    void* workspace, int32_t* status_out, uint64_t* index_out,
                                    void* stream);

/* ---- host verification path: the aggregation service's hedge --------------------------
 * The kernels' own arithmetic headers compiled for the CPU (narwhal_amd/csrc/nw_host.cpp),
 * with the same statuses and indices as the device entry points above. The service uses it
 * to answer a request whose device job is late (nw_service_set_hedge); these entries expose
 * it for the parity tests and need no device. No device entry point ever falls back to it.
 * Random coefficients (z16 NULL) come from ChaCha20 keyed by the OS CSPRNG, as on the
 * device. Return 0, or a negative NW_E_* (the verdicts go to status_out / index_out). */
int nw_host_verify_strict_many(const uint8_t* msgs, size_t msg_stride, const uint8_t* pks,
                               const uint8_t* sigs, size_t n, int32_t* status_out);
int nw_host_verify_batch_many(const uint8_t* digests, const uint8_t* pks, const uint8_t* sigs,
                              const uint64_t* offsets, size_t nbatches, const uint8_t* z16,
                              int32_t* status_out, uint64_t* fail_index_out);
int nw_host_certificates_verify_many(const nw_committee* committee, const nw_certificates* certs,
                                     const uint8_t* z16, int headers_only, int32_t* status_out,
                                     uint64_t* index_out);
int nw_host_votes_verify_many(const nw_committee* committee, const uint8_t* ids,
                              const uint64_t* rounds, const uint8_t* origins,
                              const uint8_t* authors, const uint8_t* sigs, size_t n,
                              int32_t* status_out);

#ifdef __cplusplus
}
#endif
#endif /* NARWHAL_AMD_H */
