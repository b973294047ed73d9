"""Deterministic synthetic inputs in the reference's byte layouts.

Host-side plumbing for bench.py and the tests; no verification logic here.

* Worker batches: ``bincode::serialize(&WorkerMessage::Batch(Vec<Vec<u8>>))``
  (/root/reference/worker/src/batch_maker.rs:116-119, worker/src/worker.rs:36-40):
  u32 LE enum variant (0) || u64 LE tx count || per tx (u64 LE length || bytes).
  Transactions follow /root/reference/node/src/benchmark_client.rs:122-130:
  byte 0 in {0 = sample, 1 = standard}, then a u64 BE counter, then padding
  (seeded random bytes here instead of zeros, to avoid constant-input artefacts).
* The 500 KB config: batch_size = 500,000 (config/src/lib.rs:92) seals at >= 500,000
  bytes of 512-byte txs -> 977 txs -> 4 + 8 + 977 * 520 = 508,052 bytes.
"""
from __future__ import annotations

import struct

import numpy as np

BATCH_TXS = 977
TX_SIZE = 512
BATCH_BYTES = 4 + 8 + BATCH_TXS * (8 + TX_SIZE)   # 508,052


def serialize_batch(txs: list[bytes]) -> bytes:
    """bincode 1.x legacy encoding of WorkerMessage::Batch(txs)."""
    out = [struct.pack("<IQ", 0, len(txs))]
    for tx in txs:
        out.append(struct.pack("<Q", len(tx)))
        out.append(bytes(tx))
    return b"".join(out)


def reference_serialized_batch() -> bytes:
    """worker/src/tests/common.rs:86-100 fixture: two 100-byte zero transactions."""
    return serialize_batch([bytes(100), bytes(100)])


def worker_batch(batch_id: int, n_tx: int = BATCH_TXS, tx_size: int = TX_SIZE,
                 seed: int = 0) -> np.ndarray:
    """One serialized worker batch as a uint8 array (length 12 + n_tx*(8+tx_size))."""
    rng = np.random.Generator(np.random.PCG64([seed, batch_id]))
    body = rng.integers(0, 256, size=(n_tx, tx_size), dtype=np.uint8)
    counters = np.arange(batch_id * n_tx, (batch_id + 1) * n_tx, dtype=">u8")
    body[:, 0] = (np.arange(n_tx) % 50 != 0).astype(np.uint8)   # a few sample txs (0)
    body[:, 1:9] = counters.view(np.uint8).reshape(n_tx, 8)
    rec = np.empty((n_tx, 8 + tx_size), dtype=np.uint8)
    rec[:, :8] = np.frombuffer(struct.pack("<Q", tx_size) * n_tx, dtype=np.uint8).reshape(n_tx, 8)
    rec[:, 8:] = body
    head = np.frombuffer(struct.pack("<IQ", 0, n_tx), dtype=np.uint8)
    return np.concatenate([head, rec.reshape(-1)])


def ragged_messages(n: int, max_len: int, seed: int = 1) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """n random messages of lengths in [0, max_len] packed contiguously.
    Returns (data, offsets, lengths) with uint64 offsets/lengths."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = rng.integers(0, max_len + 1, size=n).astype(np.uint64)
    offsets = np.zeros(n, dtype=np.uint64)
    if n:
        offsets[1:] = np.cumsum(lengths)[:-1]
    total = int(lengths.sum())
    data = rng.integers(0, 256, size=max(total, 1), dtype=np.uint8)
    return data, offsets, lengths


# --------------------------------------------------------------------------------------
# Certificate streams (BASELINE config 2): primary/src/messages.rs layouts.
# --------------------------------------------------------------------------------------
def quorum(n_auth: int) -> int:
    """Votes needed at stake 1 each: Committee::quorum_threshold (config/src/lib.rs:167-173)."""
    return 2 * n_auth // 3 + 1


def _sort_digests(d: np.ndarray) -> np.ndarray:
    """Sort [m, k, 32] digests along axis 1 in byte-lexicographic (BTreeSet) order."""
    m, k = d.shape[:2]
    rec = np.ascontiguousarray(d).view([("a", ">u8"), ("b", ">u8"), ("c", ">u8"), ("d", ">u8")])
    return np.sort(rec.reshape(m, k), axis=1).view(np.uint8).reshape(m, k, 32)


def certificate_stream(n_certs: int, keys: list[tuple[bytes, bytes]], sign_many, digest_many,
                       payload: int = 0, seed: int = 0, n_votes: int | None = None) -> dict:
    """n_certs honest certificates over the committee ``keys`` (list of (pk, sk)), stake 1
    each, one worker (id 0) per authority. Certificate i: author = keys[i % N], round =
    1 + i // N, ``payload`` (digest, worker 0) entries, q parents from a seeded stream
    (sorted: BTreeSet order), votes by q distinct authorities (starting at the author) over
    Certificate::digest. ``sign_many(sks[n,64], msgs[n,32]) -> sigs[n,64]`` and
    ``digest_many(data, offsets[n+1]) -> [n,32]`` are supplied by the caller (the GPU
    engine in bench.py, the oracle in tests), so this module computes nothing itself.

    Returns the nw_certificates SoA dict (narwhal_amd.messages.pack_certificates layout)
    plus 'committee' (pack_committee layout) and 'rounds', 'authors'."""
    N = len(keys)
    q = quorum(N) if n_votes is None else n_votes
    rng = np.random.Generator(np.random.PCG64([seed, N, payload]))
    order = sorted(range(N), key=lambda k: keys[k][0])
    pk_sorted = np.array([np.frombuffer(keys[k][0], np.uint8) for k in order])
    sks = np.array([np.frombuffer(keys[k][1], np.uint8) for k in range(N)])
    pks = sks[:, 32:]
    a = np.arange(n_certs) % N
    rounds = (1 + np.arange(n_certs) // N).astype(np.uint64)
    # header preimage: author || round || payload (sorted by digest) || parents (sorted)
    L = 40 + 36 * payload + 32 * q
    hb = np.zeros((n_certs, L), np.uint8)
    hb[:, :32] = pks[a]
    hb[:, 32:40] = rounds.astype("<u8").view(np.uint8).reshape(n_certs, 8)
    if payload:
        ent = np.zeros((n_certs, payload, 36), np.uint8)
        ent[:, :, :32] = _sort_digests(rng.integers(0, 256, size=(n_certs, payload, 32),
                                                    dtype=np.uint8))
        hb[:, 40:40 + 36 * payload] = ent.reshape(n_certs, -1)
    par = _sort_digests(rng.integers(0, 256, size=(n_certs, q, 32), dtype=np.uint8))
    hb[:, 40 + 36 * payload:] = par.reshape(n_certs, -1)
    ho = (np.arange(n_certs + 1) * L).astype(np.uint64)
    ids = digest_many(hb.reshape(-1), ho)
    hsig = sign_many(sks[a], ids)
    cpre = np.zeros((n_certs, 72), np.uint8)
    cpre[:, :32] = ids
    cpre[:, 32:40] = hb[:, 32:40]
    cpre[:, 40:] = pks[a]
    cdig = digest_many(cpre.reshape(-1), (np.arange(n_certs + 1) * 72).astype(np.uint64))
    voters = (a[:, None] + np.arange(q)[None, :]) % N
    vsig = sign_many(sks[voters.reshape(-1)], np.repeat(cdig, q, axis=0))
    return {
        "header_bytes": hb.reshape(-1), "header_offsets": ho,
        "payload_counts": np.full(n_certs, payload, np.uint32), "ids": ids,
        "header_sigs": hsig, "vote_offsets": (np.arange(n_certs + 1) * q).astype(np.uint64),
        "vote_pks": pks[voters.reshape(-1)].copy(), "vote_sigs": vsig,
        "committee": {"pks": pk_sorted, "stakes": np.ones(N, np.uint32),
                      "worker_offsets": np.arange(N + 1, dtype=np.uint64),
                      "worker_ids": np.zeros(N, np.uint32)},
        "rounds": rounds, "cert_digests": cdig, "q": q,
    }


# Certificate::verify statuses of the vote-level mutations below (include/narwhal_amd.h:
# NW_DAG_INVALID_VOTES + the first failing check of Signature::verify_batch,
# crypto/src/lib.rs:206-219): (kind, status, index-or-None for "the equation" = #votes).
VOTE_MUTATIONS = (("s_low_flip", 48 + 7, None),      # equation fails (s changed, s < l kept)
                  ("s_high_bits", 48 + 1, "j"),      # ed25519 Signature::from_bytes, fail-fast
                  ("R_undecodable", 48 + 4, "j"))    # y = 2 is not on the curve


def mutate_votes(s: dict, bad_certs: np.ndarray, seed: int = 0) -> tuple[dict, np.ndarray, np.ndarray]:
    """Copy of certificate stream ``s`` in which one vote of every certificate in
    ``bad_certs`` is invalid (byte edits only; the mutation kind cycles through
    VOTE_MUTATIONS, the vote is chosen at random). Returns (stream, expected status[n],
    expected index[n]) as Certificate::verify (primary/src/messages.rs:189-215) gives them:
    the header and quorum are intact, so the votes' verify_batch decides."""
    rng = np.random.Generator(np.random.PCG64([seed, 77]))
    out = dict(s)
    out["vote_sigs"] = s["vote_sigs"].copy()
    n = len(s["header_offsets"]) - 1
    st = np.zeros(n, np.int32)
    ix = np.zeros(n, np.uint64)
    vo = s["vote_offsets"]
    for k, c in enumerate(np.asarray(bad_certs, np.int64)):
        a, b = int(vo[c]), int(vo[c + 1])
        j = int(rng.integers(0, b - a))
        kind, code, where = VOTE_MUTATIONS[k % len(VOTE_MUTATIONS)]
        sig = out["vote_sigs"][a + j]
        if kind == "s_low_flip":
            sig[32] ^= np.uint8(1 << int(rng.integers(0, 8)))   # s' = s +- 2^i, i < 8: s' < l
        elif kind == "s_high_bits":
            sig[63] |= np.uint8(0x80 >> int(rng.integers(0, 3)))
        else:
            sig[:32] = np.frombuffer((2).to_bytes(32, "little"), np.uint8)
        st[c] = code
        ix[c] = (b - a) if where is None else j
    return out, st, ix


# --------------------------------------------------------------------------------------
# Fixture keys (BASELINE config 1): rand 0.7 StdRng::from_seed([0; 32]) =
# ChaCha20(key = 0^32, nonce = 0) keystream; seed i = bytes [32 i, 32 i + 32)
# (primary/src/tests/common.rs:28-32 keys(), extended to 10,000 keys).
# --------------------------------------------------------------------------------------
def chacha20_keystream(key: bytes, nblocks: int, counter: int = 0) -> bytes:
    """DJB ChaCha20 (64-bit counter, 64-bit nonce = 0) keystream, vectorised over blocks."""
    def rotl(x, n):
        return (x << np.uint32(n)) | (x >> np.uint32(32 - n))
    k = np.frombuffer(key, "<u4")
    ctr = np.arange(counter, counter + nblocks, dtype=np.uint64)
    s = np.zeros((16, nblocks), np.uint32)
    s[0:4] = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], np.uint32)[:, None]
    s[4:12] = k[:, None]
    s[12] = (ctr & 0xFFFFFFFF).astype(np.uint32)
    s[13] = (ctr >> 32).astype(np.uint32)
    x = s.copy()

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7)
    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return (x + s).T.astype("<u4").tobytes()


def fixture_seeds(count: int) -> np.ndarray:
    """[count, 32] seeds of the reference keys() fixture generator (StdRng zero seed)."""
    ks = chacha20_keystream(bytes(32), (32 * count + 63) // 64)
    return np.frombuffer(ks[:32 * count], np.uint8).reshape(count, 32).copy()
