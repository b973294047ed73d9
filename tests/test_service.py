"""The asynchronous boundary: nw_submit_* / nw_job_* (include/narwhal_amd.h) and the
aggregating asyncio service over it (narwhal_amd/service.py).

CPU tests drive the service's aggregation logic through a test-only backend whose jobs are
computed by the oracle (the product service has no CPU path); GPU tests run the real
jobs and check them against the oracle, including several jobs in flight at once and the
copy-on-submit contract (inputs may be reused as soon as submit returns)."""
import asyncio
import hashlib

import numpy as np
import pytest
import torch

from narwhal_amd import _lib
from narwhal_amd import crypto as C
from narwhal_amd import service as S
from oracle import oracle as O


# ------------------------------------------------------------------ shared corpus
def _strict_corpus(n, seed):
    ks = O.keys(8)
    rng = np.random.Generator(np.random.PCG64(seed))
    digs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks = np.array([np.frombuffer(ks[i % 8][0], np.uint8) for i in range(n)])
    sigs = np.array([np.frombuffer(O.sign(ks[i % 8][1], digs[i].tobytes()), np.uint8)
                     for i in range(n)])
    for i in range(0, n, 7):
        sigs[i, 40] ^= 1                      # equation failures
    for i in range(3, n, 11):
        sigs[i, 63] |= 0x40                   # s high bits
    return digs, pks, sigs


class _OracleJob:
    def __init__(self, outputs):
        self.outputs = outputs

    async def done(self):
        await asyncio.sleep(0)
        return self.outputs

    def release(self):
        pass


class _OracleBackend:
    """TEST-ONLY stand-in for GpuBackend: same submit/done contract, oracle results."""

    def __init__(self, fail=False):
        self.submits = []
        self.fail = fail

    def submit_strict(self, d, p, s):
        self.submits.append(("strict", len(p)))
        if self.fail:
            raise _lib.EngineError("injected device failure")
        return _OracleJob({"status": O.verify_strict_many(d, p, s)})

    def submit_batches(self, d, p, s, offs, z16=None):
        self.submits.append(("batch", len(offs) - 1))
        return _OracleJob({"status": O.verify_batch_many(d, p, s, offs)})

    def submit_sha(self, data, offs, lens):
        self.submits.append(("sha", len(lens)))
        return _OracleJob({"digests": O.sha512_digest32_many(data, offs, lens)})


# ------------------------------------------------------------------ CPU: aggregation
def test_service_coalesces_concurrent_requests():
    digs, pks, sigs = _strict_corpus(64, 1)
    exp = O.verify_strict_many(digs, pks, sigs)

    async def main():
        b = _OracleBackend()
        svc = S.VerificationService(backend=b, max_items=1 << 16, max_delay=0.01)
        got = await asyncio.gather(*[svc.verify(digs[i].tobytes(), pks[i].tobytes(),
                                                sigs[i].tobytes()) for i in range(64)])
        return got, b.submits

    got, submits = asyncio.run(main())
    assert got == [int(x) for x in exp]
    assert submits == [("strict", 64)]           # one device job for 64 requests


def test_service_flushes_at_max_items():
    digs, pks, sigs = _strict_corpus(35, 2)

    async def main():
        b = _OracleBackend()
        svc = S.VerificationService(backend=b, max_items=10, max_delay=10.0)
        tasks = [asyncio.ensure_future(svc.verify(digs[i].tobytes(), pks[i].tobytes(),
                                                  sigs[i].tobytes())) for i in range(35)]
        await asyncio.sleep(0)
        await svc.drain()                        # flushes the 5-item remainder
        return [t.result() for t in tasks], b.submits

    got, submits = asyncio.run(main())
    assert [n for _, n in submits] == [10, 10, 10, 5]
    assert got == [int(x) for x in O.verify_strict_many(digs, pks, sigs)]


def test_service_batches_and_digests():
    ks = O.keys(4)
    d = O.digest32(b"certificate")
    votes = [(ks[i][0], O.sign(ks[i][1], d)) for i in range(3)]
    bad = votes[:2] + [(ks[2][0], bytes(64))]      # Signature::default()
    msgs = [b"", b"abc", bytes(range(256)) * 3]

    async def main():
        b = _OracleBackend()
        svc = S.VerificationService(backend=b, max_delay=0.01)
        r = await asyncio.gather(svc.verify_batch(d, votes), svc.verify_batch(d, bad),
                                 svc.verify_batch(d, []),
                                 *[svc.digest(m) for m in msgs])
        return r, b.submits

    r, submits = asyncio.run(main())
    assert r[0] == 0 and r[1] != 0 and r[2] == 0   # empty batch: Ok without a job
    assert r[3:] == [hashlib.sha512(m).digest()[:32] for m in msgs]
    assert sorted(submits) == [("batch", 2), ("sha", 3)]


def test_service_device_failure_reaches_every_waiter():
    digs, pks, sigs = _strict_corpus(5, 3)

    async def main():
        svc = S.VerificationService(backend=_OracleBackend(fail=True), max_delay=0.01)
        return await asyncio.gather(*[svc.verify(digs[i].tobytes(), pks[i].tobytes(),
                                                 sigs[i].tobytes()) for i in range(5)],
                                    return_exceptions=True)

    res = asyncio.run(main())
    assert all(isinstance(e, _lib.EngineError) for e in res)


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only behaviour")
def test_gpu_backend_fails_loudly_without_device():
    with pytest.raises(_lib.EngineError):
        S.GpuBackend()
    import ctypes
    h = ctypes.c_void_p()
    L = _lib.lib()
    assert L.nw_submit_verify_strict(b"\0" * 32, 32, b"\0" * 32, b"\0" * 64, 1, None, None,
                                     ctypes.byref(h)) == -2
    assert h.value is None


# ------------------------------------------------------------------ GPU: real jobs
@pytest.mark.gpu
def test_jobs_in_flight_vs_oracle():
    """Three strict jobs and one batch job in flight together; inputs overwritten right
    after each submit (copy-on-submit); poll never blocks; results == oracle."""
    B = S.GpuBackend()
    corp = [_strict_corpus(n, 10 + n) for n in (1, 300, 4097)]
    exp = [O.verify_strict_many(*c) for c in corp]
    jobs = []
    for d, p, s in corp:
        jobs.append(B.submit_strict(d, p, s))
        d[:] = 0
        s[:] = 0                                  # caller reuses its buffers
    ks = O.keys(4)
    dig = O.digest32(b"batch")
    pk = np.array([np.frombuffer(ks[i % 4][0], np.uint8) for i in range(67)])
    sg = np.array([np.frombuffer(O.sign(ks[i % 4][1], dig), np.uint8) for i in range(67)])
    digs2 = np.stack([np.frombuffer(dig, np.uint8), np.frombuffer(O.digest32(b"x"), np.uint8)])
    pk2 = np.concatenate([pk, pk[:3]])
    sg2 = np.concatenate([sg, sg[:3]])          # batch 1: votes signed over another digest
    bj = B.submit_batches(digs2, pk2, sg2, np.array([0, 67, 70], np.uint64))
    assert all(j.poll() in (True, False) for j in jobs)
    for j, e in zip(jobs, exp):
        assert np.array_equal(j.wait()["status"], e)
        j.release()
    out = bj.wait()
    assert int(out["status"][0]) == 0 and int(out["status"][1]) == 7   # NW_ERR_EQUATION
    bj.release()


@pytest.mark.gpu
def test_service_on_gpu_vs_oracle():
    digs, pks, sigs = _strict_corpus(500, 7)
    exp = O.verify_strict_many(digs, pks, sigs)
    msgs = [bytes([i]) * (i * 37 % 1000) for i in range(50)]

    async def main():
        svc = S.VerificationService(max_delay=0.002)
        r = await asyncio.gather(*[svc.verify(digs[i].tobytes(), pks[i].tobytes(),
                                              sigs[i].tobytes()) for i in range(500)],
                                 *[svc.digest(m) for m in msgs])
        return r, svc.jobs_submitted

    r, jobs = asyncio.run(main())
    assert r[:500] == [int(x) for x in exp]
    assert r[500:] == [hashlib.sha512(m).digest()[:32] for m in msgs]
    assert jobs <= 4


@pytest.mark.gpu
def test_blocking_calls_are_submit_plus_wait():
    """The drop-in blocking entry points agree with the async ones (same code path)."""
    digs, pks, sigs = _strict_corpus(130, 9)
    st, bm = C.verify_strict_many(digs, pks, sigs)
    job = S.GpuBackend.submit_strict(digs, pks, sigs)
    assert np.array_equal(job.wait()["status"], st)
    job.release()
    assert np.array_equal(np.unpackbits(bm, bitorder="little")[:130].astype(bool), st == 0)
