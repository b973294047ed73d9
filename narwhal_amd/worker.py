"""The worker's batch-digest path on the engine.

``Processor.spawn`` mirrors ``worker::Processor::spawn`` (worker/src/processor.rs:21-57):
receive a serialized ``WorkerMessage::Batch``, compute ``Digest(Sha512(batch)[..32])``,
``store.write(digest, batch)``, then send
``bincode::serialize(&WorkerPrimaryMessage::{OurBatch, OthersBatch}(digest, id))``
(primary/src/primary.rs:51-56) to the primary. Same names, channel semantics and output
bytes, so the reference's ``hash_and_store`` test (worker/src/tests/processor_tests.rs)
reads the same (tests/test_worker.py).

Where the hash runs (``hash_on``):

* ``"host"`` (the default) — SHA-512 on the calling thread (OpenSSL through ``hashlib``, the
  sha2-equivalent), exactly where the reference hashes (worker/src/processor.rs:38).
* ``"device"`` — every batch is handed to the aggregating ``VerificationService`` as soon as
  it arrives (several batches in flight share one SHA-512 device job), while a writer task
  stores and announces the digests strictly in arrival order.

Crossover (bench.py ``worker_latency``, 508,052-B batches, 1x MI355X,
``profiles/r04b/worker.json``, ``worker_deep.json``): SHA-512 is a serial chain per message,
so a GPU digest is one lane walking the batch's ~3,970 blocks — ~31 ms per batch (p50 at 50
batches/s) against 0.36 ms on one host core (OpenSSL). The device path loses on latency at
EVERY offered rate, and on throughput to the host's cores too: with the default lookahead of
16 batches it sustains ~300-500 batches/s (one host core: ~2,800/s; 16 threads: ~20,000/s),
and even with 1,024 batches in flight ~4,500/s at ~250 ms p50. The device only wins when tens
of thousands of batches are hashed at once (config 3: 65,536 batches in 26 ms, 1.28 TB/s),
which a worker's ``Processor`` never sees. Hence the host default; ``"device"`` is for a
worker whose cores are needed elsewhere and that accepts a ~30 ms digest latency.
"""
from __future__ import annotations

import asyncio
import hashlib
import struct

from .service import VerificationService

__all__ = ["Store", "Processor", "our_batch_message", "others_batch_message"]

_OUR_BATCH, _OTHERS_BATCH = 0, 1


def our_batch_message(digest: bytes, worker_id: int) -> bytes:
    """bincode::serialize(&WorkerPrimaryMessage::OurBatch(digest, id))."""
    return struct.pack("<I", _OUR_BATCH) + bytes(digest) + struct.pack("<I", worker_id)


def others_batch_message(digest: bytes, worker_id: int) -> bytes:
    """bincode::serialize(&WorkerPrimaryMessage::OthersBatch(digest, id))."""
    return struct.pack("<I", _OTHERS_BATCH) + bytes(digest) + struct.pack("<I", worker_id)


class Store:
    """In-memory stand-in for store::Store (store/src/lib.rs: RocksDB behind a channel;
    storage is out of scope here): async write / read of byte keys and values."""

    def __init__(self):
        self._kv: dict[bytes, bytes] = {}

    async def write(self, key: bytes, value: bytes) -> None:
        self._kv[bytes(key)] = bytes(value)

    async def read(self, key: bytes) -> bytes | None:
        return self._kv.get(bytes(key))


class Processor:
    """worker::Processor: hashes and stores batches, then outputs the batch's digest."""

    # Batches hashed ahead of the store write (the reference handles one batch before it
    # receives the next, so rx_batch's bound pushes back on senders; this keeps that
    # backpressure with a bounded lookahead instead of an unbounded queue).
    MAX_IN_FLIGHT = 16

    @staticmethod
    def spawn(worker_id: int, store: Store, rx_batch: asyncio.Queue, tx_digest: asyncio.Queue,
              own_digest: bool, service: VerificationService | None = None,
              max_in_flight: int = MAX_IN_FLIGHT, hash_on: str = "host") -> asyncio.Task:
        """Runs until ``rx_batch`` yields None (the reference's closed channel).
        ``hash_on="host"``: one batch at a time, hashed on this thread, as the reference.
        ``hash_on="device"``: hashed through ``service``; at most ``max_in_flight`` batches
        are hashed ahead of the store write, beyond that the hash loop stops taking batches
        from ``rx_batch``."""
        if hash_on not in ("host", "device"):
            raise ValueError(f"hash_on must be 'host' or 'device', not {hash_on!r}")
        if hash_on == "device" and service is None:
            raise ValueError("hash_on='device' needs a VerificationService")
        make = our_batch_message if own_digest else others_batch_message

        async def host_loop():
            while True:
                batch = await rx_batch.get()
                if batch is None:
                    return
                digest = hashlib.sha512(batch).digest()[:32]
                await store.write(digest, batch)
                await tx_digest.put(make(digest, worker_id))

        if hash_on == "host":
            return asyncio.ensure_future(host_loop())

        pending: asyncio.Queue = asyncio.Queue(maxsize=max(1, max_in_flight))

        async def hash_loop():
            while True:
                batch = await rx_batch.get()
                if batch is None:
                    await pending.put(None)
                    return
                # hashing starts now; results are consumed in arrival order below
                await pending.put((batch, asyncio.ensure_future(service.digest(batch))))

        async def deliver_loop():
            while True:
                item = await pending.get()
                if item is None:
                    return
                batch, fut = item
                digest = await fut
                await store.write(digest, batch)
                await tx_digest.put(make(digest, worker_id))

        async def run():
            await asyncio.gather(hash_loop(), deliver_loop())

        return asyncio.ensure_future(run())
