"""In-library fan-out across devices: nw_set_device(NW_ALL_DEVICES) splits every host-buffer
call into contiguous parts, one per device, and merges the outputs in order (SURVEY 8(e):
one Narwhal primary process, primary/src/core.rs:338-346, drives all GPUs). On a one-GPU box
NW_FANOUT_PARTS=k deals k parts round-robin over the devices, so the split and merge logic
(64-aligned strict parts and bitmap bytes, whole batches / messages / certificates per part,
parent jobs over per-part jobs) runs and is checked against the oracle and the single-device
results."""
import ctypes
import hashlib
import threading

import numpy as np
import pytest

from narwhal_amd import _lib
from narwhal_amd import crypto as C
from narwhal_amd import messages as M
from narwhal_amd import workloads as W
from oracle import oracle as O

from cert_cases import mutated_stream, votes_case

pytestmark = pytest.mark.gpu

ALL = -1   # NW_ALL_DEVICES


class _Com:
    def __init__(self, p):
        self._p = p

    def packed(self):
        return self._p


@pytest.fixture(params=[1, 3, 5])
def fanout(request, monkeypatch):
    """Every host-buffer call of this thread fans out over `parts` parts."""
    L = _lib.lib()
    assert L.nw_init() > 0
    monkeypatch.setenv("NW_FANOUT_PARTS", str(request.param))
    assert L.nw_set_device(ALL) == 0
    assert L.nw_get_device() == ALL
    yield request.param
    assert L.nw_set_device(0) == 0


def _strict_corpus(n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    kps = [O.keypair_from_seed(rng.bytes(32)) for _ in range(16)]
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks = np.array([np.frombuffer(kps[i % 16][0], np.uint8) for i in range(n)])
    sigs = np.array([np.frombuffer(O.sign(kps[i % 16][1], msgs[i].tobytes()), np.uint8)
                     for i in range(n)])
    for i in rng.choice(n, n // 6, replace=False):
        sigs[i, rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))
    return msgs, pks, sigs


@pytest.mark.parametrize("n", [1, 63, 200, 1000])
def test_fanout_strict_matches_oracle(fanout, n):
    m, p, s = _strict_corpus(n, n)
    st, bm = C.verify_strict_many(m, p, s)
    ref = O.verify_strict_many(m, p, s)
    assert np.array_equal(st, ref)
    assert np.array_equal(np.unpackbits(bm, bitorder="little")[:n], (ref == 0).astype(np.uint8))


def test_fanout_batches_and_sha(fanout):
    rng = np.random.Generator(np.random.PCG64(4))
    kps = [O.keypair_from_seed(rng.bytes(32)) for _ in range(40)]
    sizes = [0, 3, 7, 34, 67, 1, 600, 5, 12]
    offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    digests = rng.integers(0, 256, size=(len(sizes), 32), dtype=np.uint8)
    pks, sigs = [], []
    for b, k in enumerate(sizes):
        for j in range(k):
            pk, sk = kps[j % 40]
            pks.append(np.frombuffer(pk, np.uint8))
            sigs.append(np.frombuffer(O.sign(sk, digests[b].tobytes()), np.uint8))
    pks, sigs = np.array(pks), np.array(sigs)
    sigs[int(offsets[4]) + 9, 40] ^= 2
    z = rng.integers(0, 256, size=(len(pks), 16), dtype=np.uint8)
    st = C.verify_batch_many(digests, pks, sigs, offsets, z16=z)
    assert np.array_equal(st, O.verify_batch_many(digests, pks, sigs, offsets, z16=z))
    assert st[4] != 0 and (np.delete(st, 4) == 0).all()
    data, offs, lens = W.ragged_messages(300, 2000, seed=3)
    out = C.sha512_digest32_many(data, offs, lens)
    for i in range(300):
        m = data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
        assert out[i].tobytes() == hashlib.sha512(m).digest()[:32]


def test_fanout_messages_vs_oracle(fanout):
    com, s, exp_st, exp_ix, _ = mutated_stream(N=10, copies=2, seed=41)
    st, ix = M.verify_certificates_many(_Com(com), s, None)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    hst, hix = M.verify_headers_many(_Com(com), s)
    ost, oix = O.certificates_verify_many(com, s, headers_only=True)
    assert hst.tolist() == ost.tolist() and hix.tolist() == oix.tolist()
    vcom, p, n, exp = votes_case()
    assert M.verify_votes_many(_Com(vcom), p).tolist() == exp.tolist()


def test_fanout_async_jobs_notify(fanout):
    """Parent jobs: poll until done, notify fires once after every part finished."""
    L = _lib.lib()
    m, p, s = _strict_corpus(700, 9)
    ref = O.verify_strict_many(m, p, s)
    st = np.full(700, -9, np.int32)
    job = ctypes.c_void_p()
    rc = L.nw_submit_verify_strict(m.ctypes.data, 32, p.ctypes.data, s.ctypes.data, 700,
                                   st.ctypes.data, None, ctypes.byref(job))
    assert rc == 0, L.nw_last_error()
    fired = threading.Event()
    count = []
    cb = _lib.NOTIFY_FN(lambda arg: (count.append(1), fired.set()))
    assert L.nw_job_notify(job, cb, None) == 0
    assert fired.wait(30)
    while L.nw_job_poll(job) == 0:
        pass
    L.nw_job_release(job)
    assert np.array_equal(st, ref)
    assert count == [1]


def test_fanout_rejects_device_pointer_calls():
    L = _lib.lib()
    assert L.nw_set_device(ALL) == 0
    try:
        rc = L.nw_dev_sha512_digest32_many(None, None, None, 0, None, None)
        assert rc == -1 and b"one device" in L.nw_last_error()
    finally:
        assert L.nw_set_device(0) == 0


def test_native_service_fans_out(fanout):
    """A native aggregation service created under nw_set_device(NW_ALL_DEVICES) submits its
    jobs fanned out (its threads take the creating thread's device choice): single
    certificates from two threads, verdicts equal the oracle's."""
    from narwhal_amd import service as S
    from cert_cases import oracle_digest_many, oracle_sign_many
    hon = W.certificate_stream(900, O.keys(10), oracle_sign_many, oracle_digest_many, seed=97)
    m, est, eix = W.mutate_votes(hon, np.arange(3, 900, 50), seed=7)
    from cert_cases import unpack
    rows = [S.CertRow(r["hb"], r["np"], r["id"], r["sig"], b"".join(pk for pk, _ in r["votes"]),
                      b"".join(sg for _, sg in r["votes"]), len(r["votes"])) for r in unpack(m)]
    svc = S.NativeService(m["committee"], max_items=2000, max_delay=0.0005, hedge=0)
    got = [None] * len(rows)

    def worker(t):
        for i in range(t, len(rows), 2):
            svc.submit_certificate(rows[i], lambda st, ix, i=i: got.__setitem__(i, (st, ix)))
    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    svc.drain()
    svc.close()
    assert got == [(int(a), int(b)) for a, b in zip(est, eix)]
