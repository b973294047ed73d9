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

    def submit_certificates(self, com, certs, z16=None, headers_only=False):
        n = len(certs["header_offsets"]) - 1
        self.submits.append(("headers" if headers_only else "certs", n))
        st, ix = O.certificates_verify_many(com, certs, z16, headers_only=headers_only)
        return _OracleJob({"status": st, "index": ix})

    def submit_votes(self, com, votes, n):
        self.submits.append(("votes", n))
        return _OracleJob({"status": O.votes_verify_many(com, votes, n)})


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


def _rows(s):
    """A packed certificate stream as one CertRow per certificate."""
    from cert_cases import unpack
    return [S.CertRow(r["hb"], r["np"], r["id"], r["sig"], b"".join(pk for pk, _ in r["votes"]),
                      b"".join(sg for _, sg in r["votes"]), len(r["votes"])) for r in unpack(s)]


class _Committee:
    def __init__(self, packed):
        self._p = packed

    def packed(self):
        return self._p


def test_service_coalesces_certificates_per_committee():
    """Core::sanitize_certificate-style requests (one certificate each, many concurrent) are
    coalesced into one job per committee; (status, index) per certificate == the oracle's
    per-certificate Certificate::verify; votes and headers likewise."""
    from cert_cases import mutated_stream, votes_case
    com4, s4, st4, ix4, _ = mutated_stream(N=4, copies=2, seed=41)
    com10, s10, st10, ix10, _ = mutated_stream(N=10, copies=1, seed=42)
    vcom, vp, vn, vexp = votes_case(N=4, seed=43, count=12)
    c4, c10, cv = _Committee(com4), _Committee(com10), _Committee(vcom)
    r4, r10 = _rows(s4), _rows(s10)
    votes = [(vp["ids"][i].tobytes(), int(vp["rounds"][i]), vp["origins"][i].tobytes(),
              vp["authors"][i].tobytes(), vp["sigs"][i].tobytes()) for i in range(vn)]

    async def main():
        b = _OracleBackend()
        svc = S.VerificationService(backend=b, max_delay=0.01)
        got = await asyncio.gather(*[svc.certificate_status(c4, r) for r in r4],
                                   *[svc.certificate_status(c10, r) for r in r10],
                                   *[svc.header_status(c4, r) for r in r4],
                                   *[svc.vote_status(cv, v) for v in votes])
        return got, b.submits

    got, submits = asyncio.run(main())
    n4, n10 = len(r4), len(r10)
    assert got[:n4] == [(int(a), int(b)) for a, b in zip(st4, ix4)]
    assert got[n4:n4 + n10] == [(int(a), int(b)) for a, b in zip(st10, ix10)]
    hst, hix = O.certificates_verify_many(com4, s4, headers_only=True)
    assert got[n4 + n10:2 * n4 + n10] == [(int(a), int(b)) for a, b in zip(hst, hix)]
    assert got[2 * n4 + n10:] == [int(x) for x in vexp]
    assert sorted(submits) == sorted([("certs", n4), ("certs", n10), ("headers", n4),
                                      ("votes", vn)])


def test_service_verify_certificate_raises_dag_errors():
    """verify_certificate / verify_header / verify_vote raise the reference's DagError
    variants (primary/src/error.rs:26-59) exactly as Certificate/Header/Vote.verify do."""
    from narwhal_amd import messages as M
    from narwhal_amd.crypto import PublicKey, Signature
    ks = O.keys(4)
    com = M.Committee({PublicKey(pk): M.Authority(1) for pk, _ in ks})
    h = M.Header(author=PublicKey(ks[0][0]), round=2)
    h.id = M.Digest(O.digest32(h.digest_bytes()))
    h.signature = Signature.from_bytes(O.sign(ks[0][1], h.id.value))
    cert = M.Certificate(h)
    cd = O.digest_72(h.id.value, h.round, h.author.value)        # Certificate::digest
    cert.votes = [(PublicKey(pk), Signature.from_bytes(O.sign(sk, cd))) for pk, sk in ks[:3]]
    reuse = M.Certificate(h, cert.votes[:2] + [cert.votes[0]])
    short = M.Certificate(h, cert.votes[:2])
    badsig = M.Certificate(h, cert.votes[:2] + [(cert.votes[2][0], Signature())])
    vote = M.Vote(h.id, h.round, h.author, PublicKey(ks[1][0]),
                  Signature.from_bytes(O.sign(ks[1][1], cd)))

    async def main():
        svc = S.VerificationService(backend=_OracleBackend(), max_delay=0.001)
        await svc.verify_certificate(com, cert)
        await svc.verify_header(com, h)
        await svc.verify_vote(com, vote)
        out = []
        for c in (reuse, short, badsig):
            try:
                await svc.verify_certificate(com, c)
                out.append(None)
            except M.DagError as e:
                out.append(type(e))
        return out

    assert asyncio.run(main()) == [M.AuthorityReuse, M.CertificateRequiresQuorum,
                                   M.InvalidSignature]


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


# ------------------------------------------------------------------ GPU: message jobs
def _zeroed(d):
    for a in d.values():
        a[...] = 0


@pytest.mark.gpu
def test_message_jobs_in_flight_vs_oracle():
    """Certificate, Header and Vote jobs (nw_submit_certificates_verify_many /
    nw_submit_headers_verify_many / nw_submit_votes_verify_many) in flight together, on two
    committees, every input array overwritten right after its submit (copy-on-submit):
    statuses and indices equal the oracle's, whichever grouping each job ran."""
    from cert_cases import mutated_stream, oracle_digest_many, votes_case
    from narwhal_amd import workloads as W
    B = S.GpuBackend()
    com4, s4, st4, ix4, _ = mutated_stream(N=4, copies=3, seed=51)
    com10, s10, st10, ix10, _ = mutated_stream(N=10, copies=2, seed=52)
    hst, hix = O.certificates_verify_many(com4, s4, headers_only=True)
    vcom, vp, vn, vexp = votes_case(N=4, seed=53, count=64)
    hon = W.certificate_stream(3000, O.keys(4), lambda sk, m: C.sign_many(sk, m),
                               oracle_digest_many, seed=54)
    m, mst, mix = W.mutate_votes(hon, np.arange(17, 3000, 100), seed=3)
    expect = [(st4, ix4), (st10, ix10), (hst, hix), (vexp, None), (mst, mix)]
    jobs = []
    for com, s, kind in ((com4, s4, "c"), (com10, s10, "c"), (com4, s4, "h"), (vcom, vp, "v"),
                         (m["committee"], m, "c")):
        com = {k: np.array(v) for k, v in com.items()}
        s = {k: np.array(v) for k, v in s.items() if k != "committee"}
        if kind == "v":
            jobs.append(B.submit_votes(com, s, vn))
        else:
            jobs.append(B.submit_certificates(com, s, headers_only=kind == "h"))
        _zeroed(com)
        _zeroed(s)                                   # caller reuses its buffers
    assert all(j.poll() in (True, False) for j in jobs)
    for j, (est, eix) in zip(jobs, expect):
        out = j.wait()
        assert out["status"].tolist() == [int(x) for x in est]
        if eix is not None:
            assert out["index"].tolist() == [int(x) for x in eix]
        j.release()


@pytest.mark.gpu
def test_same_size_committees_switch_key_tables():
    """Committees A, B (same size, other keys), A, A: the per-device key tables are reused
    while the committee is unchanged and rebuilt when a same-size committee differs (the
    device-side compare, k_key_cmp). Certificates, headers and votes of each against the
    oracle with injected coefficients, plus the CSPRNG path against the same statuses."""
    from cert_cases import oracle_digest_many, votes_case
    from narwhal_amd import messages as M
    from narwhal_amd import workloads as W
    ka = [O.keypair_from_seed(bytes([i + 1]) * 32) for i in range(6)]
    kb = [O.keypair_from_seed(bytes([i + 101]) * 32) for i in range(6)]
    other = {id(ka): kb, id(kb): ka}
    for keys, seed in ((ka, 61), (kb, 62), (ka, 63), (ka, 64)):
        s = W.certificate_stream(40, keys, lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                                 seed=seed)
        # a quarter of the certificates carry one invalid vote; the honest ones pass only
        # if this committee's tables (not the previous same-size committee's) are used
        s2, _, _ = W.mutate_votes(s, np.arange(0, 40, 4), seed=seed)
        com = _Committee(s["committee"])
        z16 = np.random.Generator(np.random.PCG64(seed)).integers(
            0, 256, size=(len(s2["vote_pks"]), 16), dtype=np.uint8)
        st, ix = M.verify_certificates_many(com, s2, z16)
        ost, oix = O.certificates_verify_many(s["committee"], s2, z16)
        assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()
        st, ix = M.verify_certificates_many(com, s2, None)
        assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()
        hs, hi = M.verify_headers_many(com, s2)
        ohs, ohi = O.certificates_verify_many(s["committee"], s2, headers_only=True)
        assert hs.tolist() == ohs.tolist() and hi.tolist() == ohi.tolist()
        vcom, vp, vn, vexp = votes_case(N=6, seed=seed, count=40, keys=keys)
        assert M.verify_votes_many(_Committee(vcom), vp).tolist() == vexp.tolist()
        # votes by the OTHER committee's keys: unknown authorities here
        ocom, op, on, _ = votes_case(N=6, seed=seed, count=12, keys=other[id(keys)])
        assert (M.verify_votes_many(_Committee(vcom), op) == 17).all()


@pytest.mark.gpu
def test_service_messages_on_gpu_vs_oracle():
    """The aggregating service's certificate / header / vote paths on the device: many
    concurrent single-message requests become a few jobs; every (status, index) equals the
    oracle's."""
    from cert_cases import mutated_stream, votes_case
    com4, s4, st4, ix4, _ = mutated_stream(N=4, copies=4, seed=71)
    vcom, vp, vn, vexp = votes_case(N=4, seed=72, count=40)
    c4, cv = _Committee(com4), _Committee(vcom)
    rows = _rows(s4)
    votes = [(vp["ids"][i].tobytes(), int(vp["rounds"][i]), vp["origins"][i].tobytes(),
              vp["authors"][i].tobytes(), vp["sigs"][i].tobytes()) for i in range(vn)]

    async def main():
        svc = S.VerificationService(max_delay=0.002)
        got = await asyncio.gather(*[svc.certificate_status(c4, r) for r in rows],
                                   *[svc.vote_status(cv, v) for v in votes])
        return got, svc.jobs_submitted

    got, jobs = asyncio.run(main())
    assert got[:len(rows)] == [(int(a), int(b)) for a, b in zip(st4, ix4)]
    assert got[len(rows):] == [int(x) for x in vexp]
    assert jobs <= 4


# ------------------------------------------------------------------ native aggregation service
@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only behaviour")
def test_native_service_fails_loudly_without_device():
    with pytest.raises(_lib.EngineError):
        S.NativeService()
    import ctypes
    h = ctypes.c_void_p()
    assert _lib.lib().nw_service_create(None, 16, 100, 2, ctypes.byref(h)) == -2
    assert h.value is None


@pytest.mark.gpu
def test_native_service_certificates_from_threads_vs_oracle():
    """nw_service_certificate from four threads at once, single certificates of two
    committees (one service each), 1 in 100 with an invalid vote plus the early-failure
    cases of cert_cases: every verdict callback's (status, index) equals the oracle's,
    every request gets exactly one callback, and the requests were coalesced."""
    import threading
    from cert_cases import mutated_stream, oracle_digest_many
    from narwhal_amd import workloads as W
    com4, s4, st4, ix4, _ = mutated_stream(N=4, copies=3, seed=81)
    hon = W.certificate_stream(2000, O.keys(10), lambda sk, m: C.sign_many(sk, m),
                               oracle_digest_many, seed=82)
    m, mst, mix = W.mutate_votes(hon, np.arange(7, 2000, 100), seed=5)
    cases = [(com4, s4, st4, ix4), (m["committee"], m, mst, mix)]
    for com, s, est, eix in cases:
        svc = S.NativeService(com, max_items=1 << 12, max_delay=0.0005, max_inflight=3,
                                 hedge=0)
        rows = _rows(s)
        got = [None] * len(rows)
        calls = [0] * len(rows)

        def worker(t):
            for i in range(t, len(rows), 4):
                def cb(st, ix, i=i):
                    got[i] = (st, ix)
                    calls[i] += 1
                svc.submit_certificate(rows[i], cb)
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        svc.drain()
        req, jobs = svc.stats()
        svc.close()
        assert calls == [1] * len(rows)
        assert got == [(int(a), int(b)) for a, b in zip(est, eix)]
        assert req == len(rows) and jobs < len(rows) / 4


@pytest.mark.gpu
def test_native_service_all_kinds_asyncio_vs_oracle():
    """Header, Vote, Certificate, Signature::verify and Signature::verify_batch requests
    through the asyncio NativeService, interleaved: each kind's verdicts equal the oracle's."""
    from cert_cases import mutated_stream, votes_case
    com4, s4, st4, ix4, _ = mutated_stream(N=4, copies=2, seed=91)
    hst, hix = O.certificates_verify_many(com4, s4, headers_only=True)
    vcom, vp, vn, vexp = votes_case(N=4, seed=92, count=40, keys=None)
    digs, pks, sigs = _strict_corpus(300, 93)
    sexp = O.verify_strict_many(digs, pks, sigs)
    ks = O.keys(4)
    dig = O.digest32(b"native batch")
    good = [(ks[i % 4][0], O.sign(ks[i % 4][1], dig)) for i in range(7)]
    bad = list(good)
    bad[4] = (bad[4][0], bytes(64))                 # Signature::default() in the batch
    rows = _rows(s4)
    votes = [(vp["ids"][i].tobytes(), int(vp["rounds"][i]), vp["origins"][i].tobytes(),
              vp["authors"][i].tobytes(), vp["sigs"][i].tobytes()) for i in range(vn)]

    async def main():
        svc = S.NativeService(com4, max_delay=0.001, hedge=0)
        vsvc = S.NativeService(vcom, max_delay=0.001, hedge=0)
        got = await asyncio.gather(*[svc.certificate_status(r) for r in rows],
                                   *[svc.header_status(r) for r in rows],
                                   *[vsvc.vote_status(v) for v in votes],
                                   *[svc.verify(digs[i].tobytes(), pks[i].tobytes(),
                                                sigs[i].tobytes()) for i in range(300)],
                                   svc.verify_batch(dig, good), svc.verify_batch(dig, bad),
                                   svc.verify_batch(dig, []))
        svc.close()
        vsvc.close()
        return got

    got = asyncio.run(main())
    n = len(rows)
    assert got[:n] == [(int(a), int(b)) for a, b in zip(st4, ix4)]
    assert got[n:2 * n] == [(int(a), int(b)) for a, b in zip(hst, hix)]
    assert got[2 * n:2 * n + vn] == [int(x) for x in vexp]
    assert got[2 * n + vn:2 * n + vn + 300] == [int(x) for x in sexp]
    bpk = np.array([np.frombuffer(p, np.uint8) for p, _ in bad])
    bsg = np.array([np.frombuffer(q, np.uint8) for _, q in bad])
    assert got[-3:] == [0, int(O.verify_batch(dig, bpk, bsg)[0]), 0]
    assert got[-2] != 0


@pytest.mark.gpu
def test_native_service_votes_not_starved_by_certificates():
    """Fairness of the service flusher (nw_service.cpp): a saturating stream of N = 100
    certificates from the C load generator's threads (tools/nw_loadgen.cpp on this very
    service: no Python, so the flood holds no interpreter lock), one job in flight at a time
    (jobs much longer than max_delay), plus a trickle of votes from Python. The ready batch
    whose first request is oldest goes first, also from an idle-device submit on a
    producer's thread, so every vote's verdict arrives within max_delay plus a few jobs'
    time, not after the flood (enum-order picking, or a producer always submitting its own
    kind, starved them). Every verdict equals the oracle's / the construction."""
    import ctypes
    import os
    import sys
    import threading
    import time
    from cert_cases import oracle_digest_many, votes_case
    from narwhal_amd import workloads as W
    from narwhal_amd.messages import certificates_struct
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import loadgen_lib
    keys = O.keys(100)
    s = W.certificate_stream(1500, keys, lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                             seed=61)
    m, mst, mix = W.mutate_votes(s, np.arange(3, 1500, 100), seed=6)
    mst = np.ascontiguousarray(mst, np.int32)
    mix = np.ascontiguousarray(mix, np.uint64)
    vcom, vp, vn, vexp = votes_case(N=100, seed=62, count=40, keys=keys)
    for k in ("pks", "stakes", "worker_offsets", "worker_ids"):
        assert np.array_equal(vcom[k], m["committee"][k]), k
    svc = S.NativeService(m["committee"], max_items=1 << 16, max_delay=0.0002, max_inflight=1,
                          hedge=0)
    rows = _rows(m)
    for r in rows[:8]:                                # warm: key tables, pools
        svc.submit_certificate(r, lambda st, ix: None)
    svc.drain()
    LG = loadgen_lib()
    cs = certificates_struct(m, len(rows))
    total = 400_000
    lat_c, out3 = np.zeros(total), np.zeros(16)   # nw_loadgen.cpp writes out[0..15]
    res = {}

    def flood():
        res["rc"] = LG.nw_loadgen_certificates_on(
            svc._h, ctypes.byref(cs), mst.ctypes.data, mix.ctypes.data,
            2e6, total, 2, lat_c.ctypes.data, out3.ctypes.data)
    lat, got = [None] * vn, [None] * vn
    th = threading.Thread(target=flood)
    th.start()
    time.sleep(0.1)                                   # the flood is in full swing
    for i in range(vn):
        v = (vp["ids"][i].tobytes(), int(vp["rounds"][i]), vp["origins"][i].tobytes(),
             vp["authors"][i].tobytes(), vp["sigs"][i].tobytes())
        t0 = time.perf_counter()

        def vcb(st, ix, i=i, t0=t0):
            lat[i] = time.perf_counter() - t0
            got[i] = st
        svc.submit_vote(v, vcb)
        time.sleep(0.005)
    th.join()
    svc.drain()
    svc.close()
    assert res["rc"] == 0 and out3[2] == 0, (res, out3)
    flood_s = out3[0]
    assert flood_s > 0.3, flood_s                     # the votes arrived during the flood
    assert got == [int(x) for x in vexp]
    assert max(lat) < 0.05, sorted(lat)[-5:]
