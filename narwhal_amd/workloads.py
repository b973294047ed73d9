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
