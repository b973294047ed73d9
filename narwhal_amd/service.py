"""Asynchronous verification service over the job ABI (nw_submit_* / nw_job_*).

This is the host layer a Rust ``crypto-gpu`` crate would put behind the reference's
``crypto::Signature::{verify, verify_batch}`` for Narwhal's tokio tasks (SURVEY.md 8(f)
rank 1), written against asyncio because the image has no Rust toolchain:

* Narwhal's primary ``Core`` verifies headers, votes and certificates one message at a time
  (primary/src/core.rs:306-346: sanitize_header / sanitize_vote / sanitize_certificate,
  each calling Header/Vote/Certificate::verify -> Signature::verify / verify_batch), and
  the worker ``Processor`` hashes one batch at a time (worker/src/processor.rs:36-54).
  A single signature or a 3..67-vote certificate is far too little work for a GPU launch,
  so the service **aggregates**: concurrent requests queue up, and a flusher submits them
  as one device job when ``max_items`` is reached or ``max_delay`` has passed since the
  first queued request.
* Submission never blocks the event loop on the device: inputs are staged into pinned
  memory by ``nw_submit_*`` and completion arrives through ``nw_job_notify`` (a callback on
  the library's watcher thread, serialised with every other job's, that only schedules the
  future on the loop; the job's stream never waits for it), the same shape as the reference's
  ``SignatureService`` (crypto/src/lib.rs:222-250: requests over a channel, replies over
  oneshot channels).

Verdicts are the engine's per-item status codes (0 = Ok; NW_ERR_* otherwise); the
``Signature.verify*`` wrappers in ``crypto.py`` turn them into ``CryptoError`` exactly as
the reference's ``Result`` does. There is no CPU path: the default backend is the gfx950
library, and a missing library or device raises ``EngineError``.
"""
from __future__ import annotations

import asyncio
import ctypes
import itertools
import threading
from dataclasses import dataclass
from typing import Callable, Sequence

import numpy as np

from . import _lib
from ._lib import EngineError, check

__all__ = ["Job", "GpuBackend", "VerificationService", "NativeService", "CertRow", "cert_row",
           "vote_row"]

_P = ctypes.c_void_p


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(_P)


class Job:
    """One submitted device job. ``outputs`` (numpy arrays) are filled when it completes;
    they are owned here so they outlive the device work."""

    _callbacks: dict[int, object] = {}
    _ids = itertools.count(1)
    _lock = threading.Lock()

    def __init__(self, handle: _P, outputs: dict[str, np.ndarray]):
        self.handle = handle
        self.outputs = outputs
        self._done = handle.value is None

    def poll(self) -> bool:
        if self._done:
            return True
        self._done = check(_lib.lib().nw_job_poll(self.handle), "nw_job_poll") == 1
        return self._done

    def wait(self) -> dict[str, np.ndarray]:
        if not self._done:
            check(_lib.lib().nw_job_wait(self.handle), "nw_job_wait")
            self._done = True
        return self.outputs

    async def done(self) -> dict[str, np.ndarray]:
        """Await completion without blocking the loop (nw_job_notify wakes it)."""
        if self.poll():
            return self.outputs
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with Job._lock:
            key = next(Job._ids)

        def _finish():
            # loop thread, after the thunk has returned: drop it, wake the waiter
            Job._callbacks.pop(key, None)
            if not fut.done():
                fut.set_result(None)

        def _fire(_arg):
            # the library's watcher thread (shared by every job): only hand the wake-up
            # to the loop
            if not loop.is_closed():
                loop.call_soon_threadsafe(_finish)

        cfn = _lib.NOTIFY_FN(_fire)
        Job._callbacks[key] = cfn   # kept alive until it has fired (even if we are cancelled)
        check(_lib.lib().nw_job_notify(self.handle, cfn, None), "nw_job_notify")
        await fut
        self.wait()                 # already complete: delivers the outputs
        return self.outputs

    def release(self) -> None:
        if self.handle.value is not None:
            _lib.lib().nw_job_release(self.handle)
            self.handle = _P(None)

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class GpuBackend:
    """Submits jobs to the gfx950 library through the C ABI."""

    def __init__(self):
        L = _lib.lib()
        n = L.nw_init()
        if n <= 0:
            raise EngineError(f"nw_init: {_lib.E_NAMES.get(n, n)}: "
                              f"{L.nw_last_error().decode(errors='replace')}")

    @staticmethod
    def submit_strict(digests: np.ndarray, pks: np.ndarray, sigs: np.ndarray) -> Job:
        """digests (n,32) or (32,) shared, pks (n,32), sigs (n,64) -> outputs 'status'."""
        n = len(pks)
        shared = digests.ndim == 1
        d = np.ascontiguousarray(digests, np.uint8)
        p = np.ascontiguousarray(pks, np.uint8)
        s = np.ascontiguousarray(sigs, np.uint8)
        st = np.zeros(n, np.int32)
        h = _P()
        check(_lib.lib().nw_submit_verify_strict(_ptr(d), 0 if shared else 32, _ptr(p), _ptr(s),
                                                 n, _ptr(st), None, ctypes.byref(h)),
              "nw_submit_verify_strict")
        return Job(h, {"status": st})

    @staticmethod
    def submit_batches(digests: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                       offsets: np.ndarray, z16: np.ndarray | None = None) -> Job:
        """digests (nb,32), pks/sigs of all votes, offsets (nb+1,) -> 'status', 'index'."""
        nb = len(offsets) - 1
        d = np.ascontiguousarray(digests, np.uint8)
        p = np.ascontiguousarray(pks, np.uint8)
        s = np.ascontiguousarray(sigs, np.uint8)
        o = np.ascontiguousarray(offsets, np.uint64)
        z = None if z16 is None else np.ascontiguousarray(z16, np.uint8)
        st = np.zeros(nb, np.int32)
        fi = np.zeros(nb, np.uint64)
        h = _P()
        check(_lib.lib().nw_submit_verify_batch_many(_ptr(d), _ptr(p), _ptr(s), _ptr(o), nb,
                                                     _ptr(z), _ptr(st), _ptr(fi),
                                                     ctypes.byref(h)),
              "nw_submit_verify_batch_many")
        return Job(h, {"status": st, "index": fi})

    @staticmethod
    def submit_sha(data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray) -> Job:
        n = len(lengths)
        buf = np.ascontiguousarray(data, np.uint8)
        if buf.size == 0:
            buf = np.zeros(1, np.uint8)
        o = np.ascontiguousarray(offsets, np.uint64)
        ln = np.ascontiguousarray(lengths, np.uint64)
        out = np.zeros((n, 32), np.uint8)
        h = _P()
        check(_lib.lib().nw_submit_sha512_digest32_many(_ptr(buf), _ptr(o), _ptr(ln), n,
                                                        _ptr(out), ctypes.byref(h)),
              "nw_submit_sha512_digest32_many")
        return Job(h, {"digests": out})


    @staticmethod
    def submit_certificates(committee: dict, certs: dict, z16: np.ndarray | None = None,
                            headers_only: bool = False) -> Job:
        """committee: messages.pack_committee arrays; certs: messages.pack_certificates
        arrays -> outputs 'status' (NW_DAG_*), 'index'. Everything is copied at submit."""
        from .messages import certificates_struct, committee_struct
        n = len(certs["header_offsets"]) - 1
        cc, cs = committee_struct(committee), certificates_struct(certs, n)
        st = np.zeros(max(n, 1), np.int32)
        ix = np.zeros(max(n, 1), np.uint64)
        h = _P()
        if headers_only:
            check(_lib.lib().nw_submit_headers_verify_many(ctypes.byref(cc), ctypes.byref(cs),
                                                           _ptr(st), _ptr(ix), ctypes.byref(h)),
                  "nw_submit_headers_verify_many")
        else:
            z = None if z16 is None else np.ascontiguousarray(z16, np.uint8)
            check(_lib.lib().nw_submit_certificates_verify_many(
                ctypes.byref(cc), ctypes.byref(cs), _ptr(z), _ptr(st), _ptr(ix),
                ctypes.byref(h)), "nw_submit_certificates_verify_many")
        return Job(h, {"status": st[:n], "index": ix[:n]})

    @staticmethod
    def submit_votes(committee: dict, votes: dict, n: int) -> Job:
        """votes: messages.pack_votes arrays (n votes) -> outputs 'status' (NW_DAG_*)."""
        from .messages import committee_struct
        cc = committee_struct(committee)
        st = np.zeros(max(n, 1), np.int32)
        h = _P()
        check(_lib.lib().nw_submit_votes_verify_many(
            ctypes.byref(cc), _ptr(votes["ids"]), _ptr(votes["rounds"]), _ptr(votes["origins"]),
            _ptr(votes["authors"]), _ptr(votes["sigs"]), n, _ptr(st), ctypes.byref(h)),
            "nw_submit_votes_verify_many")
        return Job(h, {"status": st[:n]})


# ---- one message, packed (the rows a flush concatenates) ------------------------------
@dataclass
class CertRow:
    """One Header / Certificate in nw_certificates row form: the bytes `Hash for Header`
    hashes (primary/src/messages.rs:70-84), its payload count, id, signature and votes."""
    header_bytes: bytes
    payload_count: int
    id: bytes
    signature: bytes
    vote_pks: bytes = b""
    vote_sigs: bytes = b""
    nvotes: int = 0


def cert_row(msg) -> CertRow:
    """A messages.Certificate (or Header) as a CertRow."""
    from .messages import Certificate
    h = msg.header if isinstance(msg, Certificate) else msg
    votes = msg.votes if isinstance(msg, Certificate) else []
    return CertRow(h.digest_bytes(), len(h.payload), h.id.value, h.signature.flatten(),
                   b"".join(pk.value for pk, _ in votes),
                   b"".join(sg.flatten() for _, sg in votes), len(votes))


def vote_row(v) -> tuple:
    """A messages.Vote as (id, round, origin, author, signature) bytes/ints."""
    return (v.id.value, int(v.round), v.origin.value, v.author.value, v.signature.flatten())


def _pack_rows(rows: list[CertRow]) -> dict[str, np.ndarray]:
    n = len(rows)
    ho = np.zeros(n + 1, np.uint64)
    ho[1:] = np.cumsum([len(r.header_bytes) for r in rows])
    vo = np.zeros(n + 1, np.uint64)
    vo[1:] = np.cumsum([r.nvotes for r in rows])

    def cat(parts, w):
        b = b"".join(parts)
        return np.frombuffer(b or bytes(w), np.uint8).reshape(-1, w)
    return {"header_bytes": np.frombuffer(b"".join(r.header_bytes for r in rows) or b"\0",
                                          np.uint8),
            "header_offsets": ho,
            "payload_counts": np.array([r.payload_count for r in rows], np.uint32),
            "ids": cat([r.id for r in rows], 32),
            "header_sigs": cat([r.signature for r in rows], 64),
            "vote_offsets": vo,
            "vote_pks": cat([r.vote_pks for r in rows], 32),
            "vote_sigs": cat([r.vote_sigs for r in rows], 64)}


@dataclass
class _Pending:
    payload: tuple
    future: asyncio.Future


class _Aggregator:
    """Queue of requests of one kind, flushed as one device job."""

    def __init__(self, flush: Callable[[list], "asyncio.Future"], max_items: int,
                 max_delay: float, size_of: Callable[[tuple], int]):
        self.flush_fn = flush
        self.max_items = max_items
        self.max_delay = max_delay
        self.size_of = size_of
        self.queue: list[_Pending] = []
        self.items = 0
        self.timer: asyncio.TimerHandle | None = None
        self.tasks: set[asyncio.Task] = set()
        self.jobs = 0

    def add(self, payload: tuple) -> asyncio.Future:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self.queue.append(_Pending(payload, fut))
        self.items += self.size_of(payload)
        if self.items >= self.max_items:
            self._flush()
        elif self.timer is None:
            self.timer = loop.call_later(self.max_delay, self._flush)
        return fut

    def _flush(self):
        if self.timer is not None:
            self.timer.cancel()
            self.timer = None
        if not self.queue:
            return
        batch, self.queue, self.items = self.queue, [], 0
        self.jobs += 1
        t = asyncio.get_running_loop().create_task(self._run(batch))
        self.tasks.add(t)
        t.add_done_callback(self.tasks.discard)

    async def _run(self, batch: list[_Pending]):
        try:
            results = await self.flush_fn([p.payload for p in batch])
            for p, r in zip(batch, results):
                if not p.future.done():
                    p.future.set_result(r)
        except Exception as e:  # device/runtime failure: every waiter sees it
            for p in batch:
                if not p.future.done():
                    p.future.set_exception(e)

    async def drain(self):
        self._flush()
        while self.tasks:
            await asyncio.gather(*list(self.tasks))


class VerificationService:
    """Aggregating async front end (one per event loop).

    verify(digest, pk, sig)          -> status of crypto::Signature::verify
    verify_batch(digest, votes)      -> status of crypto::Signature::verify_batch
    digest(message)                  -> 32-byte Digest(Sha512(message)[..32])
    verify_certificate(committee, c) -> Certificate::verify (raises DagError)
    verify_header(committee, h)      -> Header::verify (raises DagError)
    verify_vote(committee, v)        -> Vote::verify (raises DagError)
    certificate_status / header_status / vote_status -> the (NW_DAG_* status, index) pairs

    Requests issued concurrently (e.g. by many Core/Processor tasks) are coalesced: one
    device job per ``max_items`` items or per ``max_delay`` seconds, whichever comes first.
    The message checks run the engine's committee-aware pipeline (primary/src/core.rs:306-346
    sanitize_header / sanitize_vote / sanitize_certificate call these one message at a time
    on the single Core task): requests for the same committee share one job, so the
    committee's key tables, built once on the device, serve every message of it.
    ``backend`` is the device backend (GpuBackend by default).
    """

    def __init__(self, backend=None, max_items: int = 1 << 16, max_delay: float = 0.0005):
        self.backend = backend if backend is not None else GpuBackend()
        self.max_items = max_items
        self.max_delay = max_delay
        self._strict = _Aggregator(self._flush_strict, max_items, max_delay, lambda p: 1)
        self._batch = _Aggregator(self._flush_batch, max_items, max_delay,
                                  lambda p: max(1, len(p[1])))
        self._sha = _Aggregator(self._flush_sha, max_items, max_delay, lambda p: 1)
        self._msg: dict[tuple, _Aggregator] = {}   # (kind, committee) -> aggregator

    @property
    def jobs_submitted(self) -> int:
        return (self._strict.jobs + self._batch.jobs + self._sha.jobs
                + sum(a.jobs for a in self._msg.values()))

    def _msg_aggregator(self, kind: str, committee) -> _Aggregator:
        key = (kind, id(committee))
        a = self._msg.get(key)
        if a is None:
            packed = committee.packed()
            if kind == "vote":
                fn = lambda payloads: self._flush_votes(packed, payloads)   # noqa: E731
                size = lambda p: 1                                        # noqa: E731
            else:
                fn = lambda payloads, h=(kind == "header"): self._flush_certs(  # noqa: E731
                    packed, payloads, h)
                size = lambda p: 1 + p[0].nvotes                          # noqa: E731
            a = _Aggregator(fn, self.max_items, self.max_delay, size)
            a.committee = committee            # keeps id(committee) from being reused
            self._msg[key] = a
        return a

    # ---- primary messages ------------------------------------------------------------
    async def certificate_status(self, committee, cert) -> tuple[int, int]:
        """(status, index) of Certificate::verify; cert: messages.Certificate or CertRow."""
        row = cert if isinstance(cert, CertRow) else cert_row(cert)
        return await self._msg_aggregator("cert", committee).add((row,))

    async def header_status(self, committee, header) -> tuple[int, int]:
        row = header if isinstance(header, CertRow) else cert_row(header)
        return await self._msg_aggregator("header", committee).add((row,))

    async def vote_status(self, committee, vote) -> int:
        row = vote if isinstance(vote, tuple) else vote_row(vote)
        return await self._msg_aggregator("vote", committee).add((row,))

    async def verify_certificate(self, committee, cert) -> None:
        """Core::sanitize_certificate's check (messages.rs:189-215): None or DagError."""
        from .messages import raise_for_status
        st, ix = await self.certificate_status(committee, cert)
        raise_for_status(st, ix, cert.header, None, cert.votes)

    async def verify_header(self, committee, header) -> None:
        from .messages import raise_for_status
        st, ix = await self.header_status(committee, header)
        raise_for_status(st, ix, header, None)

    async def verify_vote(self, committee, vote) -> None:
        from .messages import raise_for_status
        raise_for_status(await self.vote_status(committee, vote), 0, None, vote)

    # ---- requests --------------------------------------------------------------------
    async def verify(self, digest: bytes, pk: bytes, sig: bytes) -> int:
        return await self._strict.add((bytes(digest), bytes(pk), bytes(sig)))

    async def verify_batch(self, digest: bytes, votes: Sequence[tuple[bytes, bytes]]) -> int:
        if not votes:   # crypto/src/lib.rs:206-219: no votes -> Ok
            return 0
        return await self._batch.add((bytes(digest), [(bytes(p), bytes(s)) for p, s in votes]))

    async def digest(self, message: bytes) -> bytes:
        return await self._sha.add((bytes(message),))

    async def drain(self):
        for a in (self._strict, self._batch, self._sha, *self._msg.values()):
            await a.drain()

    # ---- flushes: one device job per aggregated group --------------------------------
    async def _flush_strict(self, payloads: list[tuple]):
        n = len(payloads)
        d = np.frombuffer(b"".join(p[0] for p in payloads), np.uint8).reshape(n, 32)
        pk = np.frombuffer(b"".join(p[1] for p in payloads), np.uint8).reshape(n, 32)
        sg = np.frombuffer(b"".join(p[2] for p in payloads), np.uint8).reshape(n, 64)
        job = self.backend.submit_strict(d, pk, sg)
        out = await job.done()
        job.release()
        return [int(x) for x in out["status"]]

    async def _flush_batch(self, payloads: list[tuple]):
        nb = len(payloads)
        d = np.frombuffer(b"".join(p[0] for p in payloads), np.uint8).reshape(nb, 32)
        votes = [v for p in payloads for v in p[1]]
        pk = np.frombuffer(b"".join(v[0] for v in votes), np.uint8).reshape(-1, 32)
        sg = np.frombuffer(b"".join(v[1] for v in votes), np.uint8).reshape(-1, 64)
        offs = np.zeros(nb + 1, np.uint64)
        offs[1:] = np.cumsum([len(p[1]) for p in payloads])
        job = self.backend.submit_batches(d, pk, sg, offs)
        out = await job.done()
        job.release()
        return [int(x) for x in out["status"]]

    async def _flush_sha(self, payloads: list[tuple]):
        msgs = [p[0] for p in payloads]
        lens = np.array([len(m) for m in msgs], np.uint64)
        offs = np.zeros(len(msgs), np.uint64)
        if len(msgs) > 1:
            offs[1:] = np.cumsum(lens)[:-1]
        data = np.frombuffer(b"".join(msgs), np.uint8)
        job = self.backend.submit_sha(data, offs, lens)
        out = await job.done()
        job.release()
        return [bytes(r) for r in out["digests"]]

    async def _flush_certs(self, committee: dict, payloads: list[tuple], headers_only: bool):
        job = self.backend.submit_certificates(committee, _pack_rows([p[0] for p in payloads]),
                                               headers_only=headers_only)
        out = await job.done()
        job.release()
        return [(int(s), int(i)) for s, i in zip(out["status"], out["index"])]

    async def _flush_votes(self, committee: dict, payloads: list[tuple]):
        rows = [p[0] for p in payloads]
        n = len(rows)
        v = {"ids": np.frombuffer(b"".join(r[0] for r in rows), np.uint8).reshape(n, 32),
             "rounds": np.array([r[1] for r in rows], np.uint64),
             "origins": np.frombuffer(b"".join(r[2] for r in rows), np.uint8).reshape(n, 32),
             "authors": np.frombuffer(b"".join(r[3] for r in rows), np.uint8).reshape(n, 32),
             "sigs": np.frombuffer(b"".join(r[4] for r in rows), np.uint8).reshape(n, 64)}
        job = self.backend.submit_votes(committee, v, n)
        out = await job.done()
        job.release()
        return [int(s) for s in out["status"]]


class NativeService:
    """asyncio front end over the library's native aggregation service (nw_service_*,
    include/narwhal_amd.h): the same coalescing as VerificationService, but the queueing,
    batching and job submission run on the library's own threads, so a request costs one
    copy under a mutex instead of Python-level bookkeeping (this is the layer a Rust
    crypto-gpu crate binds: one request per Header / Vote / Certificate::verify from the
    primary's Core task, primary/src/core.rs:306-346; the verdict callback completes the
    request's future, as SignatureService's oneshot replies do, crypto/src/lib.rs:222-250).

    committee: messages.Committee, a packed committee dict, or None (verify / verify_batch
    only). Verdicts: (status, index) pairs as the bulk calls return them; a device failure
    raises EngineError in every affected waiter. hedge: None keeps the library's hedge
    (late requests also verified on the host, nw_service_set_hedge); 0 turns it off, so that
    every verdict is the device's (the device-parity tests); a float sets its deadline."""

    def __init__(self, committee=None, max_items: int = 1 << 16, max_delay: float = 0.0005,
                 max_inflight: int = 4, hedge: float | None = None):
        from .messages import committee_struct
        L = _lib.lib()
        n = L.nw_init()
        if n <= 0:
            raise EngineError(f"nw_init: {_lib.E_NAMES.get(n, n)}: "
                              f"{L.nw_last_error().decode(errors='replace')}")
        self._cc = None
        if committee is not None:
            self._packed = committee if isinstance(committee, dict) else committee.packed()
            self._cc = committee_struct(self._packed)
        h = _P()
        check(L.nw_service_create(ctypes.byref(self._cc) if self._cc is not None else None,
                                  max_items, int(max_delay * 1e6), max_inflight,
                                  ctypes.byref(h)), "nw_service_create")
        self._h = h
        if hedge is not None:
            self.set_hedge(hedge)
        self._lock = threading.Lock()
        self._pending: dict[int, tuple] = {}
        self._ids = itertools.count(1)
        self._cb = _lib.VERDICT_FN(self._verdict)   # one C callback for every request

    # library thread: hand the verdict to the waiter's loop (or call its plain callback)
    def _verdict(self, key, status, index):
        with self._lock:
            target = self._pending.pop(key)
        if isinstance(target, tuple):
            loop, fut = target
            if not loop.is_closed():
                loop.call_soon_threadsafe(_resolve, fut, int(status), int(index))
        else:
            target(int(status), int(index))

    def _register(self, target) -> int:
        key = next(self._ids)
        with self._lock:
            self._pending[key] = target
        return key

    def _submit(self, call, target) -> None:
        key = self._register(target)
        rc = call(key)
        if rc != 0:
            with self._lock:
                self._pending.pop(key, None)
            check(rc, "nw_service submit")

    def _future(self):
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        return (loop, fut), fut

    # ---- submits (target = (loop, future) or a plain callable(status, index)) ---------
    def submit_certificate(self, cert, target) -> None:
        r = cert if isinstance(cert, CertRow) else cert_row(cert)
        self._submit(lambda key: _lib.lib().nw_service_certificate(
            self._h, r.header_bytes, len(r.header_bytes), r.payload_count, r.id, r.signature,
            r.vote_pks or None, r.vote_sigs or None, r.nvotes, self._cb, key), target)

    def submit_header(self, header, target) -> None:
        r = header if isinstance(header, CertRow) else cert_row(header)
        self._submit(lambda key: _lib.lib().nw_service_header(
            self._h, r.header_bytes, len(r.header_bytes), r.payload_count, r.id, r.signature,
            self._cb, key), target)

    def submit_vote(self, vote, target) -> None:
        r = vote if isinstance(vote, tuple) else vote_row(vote)
        self._submit(lambda key: _lib.lib().nw_service_vote(
            self._h, r[0], r[1], r[2], r[3], r[4], self._cb, key), target)

    def submit_verify(self, digest: bytes, pk: bytes, sig: bytes, target) -> None:
        self._submit(lambda key: _lib.lib().nw_service_verify(
            self._h, bytes(digest), bytes(pk), bytes(sig), self._cb, key), target)

    def submit_verify_batch(self, digest: bytes, votes, target) -> None:
        pks = b"".join(bytes(p) for p, _ in votes)
        sgs = b"".join(bytes(s) for _, s in votes)
        self._submit(lambda key: _lib.lib().nw_service_verify_batch(
            self._h, bytes(digest), pks or None, sgs or None, len(votes), self._cb, key), target)

    # ---- awaitables --------------------------------------------------------------------
    async def certificate_status(self, cert) -> tuple[int, int]:
        t, fut = self._future()
        self.submit_certificate(cert, t)
        return await fut

    async def header_status(self, header) -> tuple[int, int]:
        t, fut = self._future()
        self.submit_header(header, t)
        return await fut

    async def vote_status(self, vote) -> int:
        t, fut = self._future()
        self.submit_vote(vote, t)
        return (await fut)[0]

    async def verify(self, digest: bytes, pk: bytes, sig: bytes) -> int:
        t, fut = self._future()
        self.submit_verify(digest, pk, sig, t)
        return (await fut)[0]

    async def verify_batch(self, digest: bytes, votes) -> int:
        if not votes:   # crypto/src/lib.rs:206-219: no votes -> Ok
            return 0
        t, fut = self._future()
        self.submit_verify_batch(digest, votes, t)
        return (await fut)[0]

    async def verify_certificate(self, cert) -> None:
        """Core::sanitize_certificate's check (messages.rs:189-215): None or DagError."""
        from .messages import raise_for_status
        st, ix = await self.certificate_status(cert)
        raise_for_status(st, ix, cert.header, None, cert.votes)

    # ---- control -----------------------------------------------------------------------
    def flush(self) -> None:
        check(_lib.lib().nw_service_flush(self._h), "nw_service_flush")

    def drain(self) -> None:
        """Block until every accepted request's verdict has been delivered (call it from a
        thread, or after the loop's waiters have been gathered)."""
        check(_lib.lib().nw_service_drain(self._h), "nw_service_drain")

    def stats(self) -> tuple[int, int]:
        req, jobs = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().nw_service_stats(self._h, ctypes.byref(req), ctypes.byref(jobs)),
              "nw_service_stats")
        return req.value, jobs.value

    def set_hedge(self, deadline: float, threads: int = 6, max_queued: int = 512) -> None:
        """Host hedge of late requests (nw_service_set_hedge): deadline in seconds (0 = off)."""
        check(_lib.lib().nw_service_set_hedge(self._h, int(deadline * 1e6), threads, max_queued),
              "nw_service_set_hedge")

    def hedge_stats(self) -> tuple[int, int, int]:
        """(requests hedged, requests the host answered first, batches the host took whole)."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().nw_service_hedge_stats(self._h, ctypes.byref(a), ctypes.byref(b),
                                                ctypes.byref(c), None), "nw_service_hedge_stats")
        return a.value, b.value, c.value

    def close(self) -> None:
        if self._h.value is not None:
            _lib.lib().nw_service_destroy(self._h)   # drains: every callback has run
            self._h = _P(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _resolve(fut: asyncio.Future, status: int, index: int) -> None:
    if fut.done():
        return
    if status < 0:
        fut.set_exception(EngineError(f"device job failed: {_lib.E_NAMES.get(status, status)}"))
    else:
        fut.set_result((status, index))
