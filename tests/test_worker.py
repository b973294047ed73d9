"""worker::Processor on the engine (narwhal_amd/worker.py), read like the reference's
worker/src/tests/processor_tests.rs::hash_and_store: send WorkerMessage::Batch(batch()),
expect bincode(WorkerPrimaryMessage::OurBatch(Sha512(serialized)[..32], id)) out and the
batch in the store under its digest. The reference fixture digest is also SURVEY
Appendix B's (JNAPdKB2...). CPU: a test-only oracle backend; GPU: the real jobs."""
import asyncio
import base64
import hashlib
import struct

import pytest

from narwhal_amd import workloads as W
from narwhal_amd.service import VerificationService
from narwhal_amd.worker import Processor, Store, our_batch_message

from test_service import _OracleBackend


def _run(backend, batches, own=True, worker_id=0, hash_on="device"):
    async def main():
        svc = VerificationService(backend=backend, max_delay=0.001)
        store = Store()
        rx, tx = asyncio.Queue(), asyncio.Queue()
        task = Processor.spawn(worker_id, store, rx, tx, own, svc, hash_on=hash_on)
        for b in batches:
            await rx.put(b)
        await rx.put(None)
        await task
        out = []
        while not tx.empty():
            out.append(tx.get_nowait())
        stored = [await store.read(hashlib.sha512(b).digest()[:32]) for b in batches]
        return out, stored, svc.jobs_submitted
    return asyncio.run(main())


def _expect(batches, own=True, worker_id=0):
    return [struct.pack("<I", 0 if own else 1) + hashlib.sha512(b).digest()[:32]
            + struct.pack("<I", worker_id) for b in batches]


APPENDIX_B_BATCH_DIGEST = "JNAPdKB2fnSAjIVGYwkClyhT+iAOB55YK4t73s1zMdg="


def test_hash_and_store_reference_fixture():
    serialized = W.reference_serialized_batch()
    out, stored, _ = _run(_OracleBackend(), [serialized])
    digest = hashlib.sha512(serialized).digest()[:32]
    assert out == [our_batch_message(digest, 0)]
    assert stored == [serialized]
    assert base64.b64encode(digest).decode() == APPENDIX_B_BATCH_DIGEST


def test_order_preserved_and_batches_share_jobs():
    batches = [W.serialize_batch([bytes([i]) * (50 + 13 * j) for j in range(i % 5 + 1)])
               for i in range(40)]
    out, stored, jobs = _run(_OracleBackend(), batches, own=False, worker_id=3)
    assert out == _expect(batches, own=False, worker_id=3)
    assert stored == batches
    assert jobs < len(batches)


@pytest.mark.gpu
def test_processor_on_gpu():
    batches = [W.worker_batch(i, seed=4).tobytes() for i in range(6)] + \
              [W.reference_serialized_batch()]
    out, stored, jobs = _run(None, batches, hash_on="device")
    assert out == _expect(batches)
    assert stored == batches
    assert jobs >= 1


def test_host_default_matches_reference_and_submits_no_jobs():
    """The default hashes on the host, one batch at a time, as processor.rs:38 does: same
    messages, same store contents, and the service is never asked for a digest."""
    batches = [W.serialize_batch([bytes([i]) * (50 + 13 * j) for j in range(i % 5 + 1)])
               for i in range(12)] + [W.reference_serialized_batch()]

    async def main():
        svc = VerificationService(backend=_OracleBackend(), max_delay=0.001)
        store, rx, tx = Store(), asyncio.Queue(), asyncio.Queue()
        task = Processor.spawn(7, store, rx, tx, False, svc)          # default: host
        task2 = Processor.spawn(7, Store(), asyncio.Queue(), asyncio.Queue(), False)  # no svc
        for b in batches:
            await rx.put(b)
        await rx.put(None)
        await task
        task2.cancel()
        out = [tx.get_nowait() for _ in range(tx.qsize())]
        stored = [await store.read(hashlib.sha512(b).digest()[:32]) for b in batches]
        return out, stored, svc.jobs_submitted
    out, stored, jobs = asyncio.run(main())
    assert out == _expect(batches, own=False, worker_id=7)
    assert stored == batches
    assert jobs == 0


def test_hash_on_rejects_bad_modes():
    q = asyncio.Queue
    with pytest.raises(ValueError):
        Processor.spawn(0, Store(), q(), q(), True, None, hash_on="device")
    with pytest.raises(ValueError):
        Processor.spawn(0, Store(), q(), q(), True, None, hash_on="gpu")


def test_backpressure_bounded_in_flight():
    """rx_batch backpressure is kept (processor.rs:36-54 takes one batch at a time): with a
    store that never completes a write, the hash loop stops taking batches once
    max_in_flight are pending, so rx_batch's own bound pushes back on the sender."""
    class StuckStore(Store):
        async def write(self, key, value):
            await asyncio.Event().wait()

    async def main():
        svc = VerificationService(backend=_OracleBackend(), max_delay=0.001)
        rx, tx = asyncio.Queue(maxsize=1), asyncio.Queue()
        task = Processor.spawn(0, StuckStore(), rx, tx, True, svc, max_in_flight=3,
                               hash_on="device")
        sent = 0
        batches = [W.serialize_batch([bytes([i]) * 64]) for i in range(20)]
        for b in batches:
            try:
                await asyncio.wait_for(rx.put(b), timeout=0.2)
            except asyncio.TimeoutError:
                break
            sent += 1
        task.cancel()
        return sent

    sent = asyncio.run(main())
    # 1 batch in the writer, 3 pending, 1 held by the hash loop waiting for room, 1 in rx
    assert 3 <= sent <= 7, sent
