"""Stream and thread safety of the device-pointer entry points (nw_dev_*), whose launches
share the device's strict-table workspace and committee key tables (nw::rt::Lease,
narwhal_amd/csrc/nw_runtime.h). Overlapping launches on two caller streams, and concurrent
host calls from two threads with different committees, must each give the oracle's
verdicts (primary/src/core.rs:306-346 calls Header/Vote/Certificate::verify from one task,
but a crypto-gpu crate serving several tokio tasks issues such calls concurrently)."""
import ctypes
import threading

import numpy as np
import pytest
import torch

from narwhal_amd import _lib
from narwhal_amd import messages as M
from narwhal_amd import workloads as W
from oracle import oracle as O

from cert_cases import mutated_stream

pytestmark = pytest.mark.gpu


def _strict_corpus(n_unique: int, seed: int):
    rng = np.random.Generator(np.random.PCG64(seed))
    kps = [O.keypair_from_seed(rng.bytes(32)) for _ in range(32)]
    msgs = rng.integers(0, 256, size=(n_unique, 32), dtype=np.uint8)
    pks = np.zeros((n_unique, 32), np.uint8)
    sigs = np.zeros((n_unique, 64), np.uint8)
    for i in range(n_unique):
        pk, sk = kps[i % 32]
        pks[i] = np.frombuffer(pk, np.uint8)
        sigs[i] = np.frombuffer(O.sign(sk, msgs[i].tobytes()), np.uint8)
    for i in rng.choice(n_unique, n_unique // 5, replace=False):
        sigs[i, rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))
    return msgs, pks, sigs, O.verify_strict_many(msgs, pks, sigs)


def test_two_streams_strict_overlapping():
    """Two nw_dev_verify_strict_many launches on two torch streams, queued back to back so
    they would overlap on the shared per-lane table workspace; both equal the oracle."""
    L = _lib.lib()
    assert L.nw_init() > 0
    dev = torch.device("cuda", 0)
    reps = 64
    runs = []
    for seed in (1, 2):
        m, p, s, exp = _strict_corpus(2048, seed)
        n = len(m) * reps
        t = [torch.from_numpy(a).to(dev).repeat(reps, 1).contiguous() for a in (m, p, s)]
        st = torch.full((n,), -99, dtype=torch.int32, device=dev)
        bm = torch.zeros((n + 63) // 64 * 8, dtype=torch.uint8, device=dev)
        runs.append((t, st, bm, np.tile(exp, reps), torch.cuda.Stream(device=dev)))
    torch.cuda.synchronize()
    for (m, p, s), st, bm, _, stream in runs:
        rc = L.nw_dev_verify_strict_many(ctypes.c_void_p(m.data_ptr()), 32,
                                         ctypes.c_void_p(p.data_ptr()),
                                         ctypes.c_void_p(s.data_ptr()), m.shape[0],
                                         ctypes.c_void_p(st.data_ptr()),
                                         ctypes.c_void_p(bm.data_ptr()),
                                         ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0, L.nw_last_error()
    torch.cuda.synchronize()
    for _, st, bm, exp, _ in runs:
        got = st.cpu().numpy()
        assert np.array_equal(got, exp)
        bits = np.unpackbits(bm.cpu().numpy(), bitorder="little")[:len(exp)]
        assert np.array_equal(bits.astype(bool), exp == 0)


def _dev_certs(com, s, dev):
    n = len(s["header_offsets"]) - 1
    nv = int(s["vote_offsets"][-1])
    keep = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items()
            if isinstance(v, np.ndarray)}
    C = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in com.items()}
    keep.update({"c_" + k: v for k, v in C.items()})
    P = lambda t: t.data_ptr()
    cc = M._CCommittee(len(com["stakes"]), P(C["pks"]), P(C["stakes"]), P(C["worker_offsets"]),
                       P(C["worker_ids"]))
    cs = M._CCertificates(n, P(keep["header_bytes"]), P(keep["header_offsets"]),
                          P(keep["payload_counts"]), P(keep["ids"]), P(keep["header_sigs"]),
                          P(keep["vote_offsets"]), P(keep["vote_pks"]), P(keep["vote_sigs"]),
                          int(s["header_offsets"][-1]), nv, s["vote_offsets"].ctypes.data)
    return cc, cs, keep, n, nv


def test_two_streams_certificates_different_committees():
    """Certificate::verify for two different committees on two streams: each call's
    committee key tables must not be replaced by the other's while it still reads them."""
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    jobs = []
    for N, seed in ((4, 21), (10, 22)):
        com, s, exp_st, exp_ix, _ = mutated_stream(N=N, copies=3, seed=seed)
        cc, cs, keep, n, nv = _dev_certs(com, s, dev)
        z16 = np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size=(nv, 16),
                                                                  dtype=np.uint8)
        keep["z"] = torch.from_numpy(z16).to(dev)
        ws = torch.empty(L.nw_dev_certificates_workspace(n, nv), dtype=torch.uint8, device=dev)
        st = torch.full((n,), -99, dtype=torch.int32, device=dev)
        ix = torch.zeros(n, dtype=torch.int64, device=dev)
        jobs.append((cc, cs, keep, ws, st, ix, exp_st, exp_ix, torch.cuda.Stream(device=dev)))
    torch.cuda.synchronize()
    for _ in range(3):
        for cc, cs, keep, ws, st, ix, _, _, stream in jobs:
            rc = L.nw_dev_certificates_verify_many(
                ctypes.byref(cc), ctypes.byref(cs), 0, ctypes.c_void_p(keep["z"].data_ptr()),
                None, ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(st.data_ptr()),
                ctypes.c_void_p(ix.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
            assert rc == 0, L.nw_last_error()
        torch.cuda.synchronize()
        for *_, st, ix, exp_st, exp_ix, _ in jobs:
            assert st.cpu().numpy().tolist() == exp_st.tolist()
            assert ix.cpu().numpy().astype(np.uint64).tolist() == exp_ix.tolist()


def test_two_threads_host_calls_different_committees():
    """Blocking host calls from two threads at once (ctypes drops the GIL): committees of 4
    and 50 keys, certificates and strict verification interleaved."""
    cases = [mutated_stream(N=4, copies=2, seed=31), mutated_stream(N=50, copies=1, seed=32)]
    m, p, s, exp = _strict_corpus(512, 3)
    errors = []

    class _Com:
        def __init__(self, c):
            self.c = c

        def packed(self):
            return self.c

    def work(k):
        try:
            com, st_in, exp_st, exp_ix, _ = cases[k]
            for _ in range(4):
                st, ix = M.verify_certificates_many(_Com(com), st_in, None)
                assert st.tolist() == exp_st.tolist(), k
                assert ix.tolist() == exp_ix.tolist(), k
                from narwhal_amd import crypto as C
                got, _ = C.verify_strict_many(m, p, s)
                assert np.array_equal(got, exp), k
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=work, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_graph_capture_sha512_replays_and_strict_refuses():
    """hipGraph capture (include/narwhal_amd.h, nw_prepare): nw_dev_sha512_digest32_many
    captured into a torch CUDA graph replays correctly on new inputs written into the same
    buffers; a strict launch (shared tables under the device lease) refuses to be captured
    with NW_E_INVALID_ARG instead of recording an event chain a replay would bypass."""
    import hashlib
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    n, ln = 64, 300
    rng = np.random.Generator(np.random.PCG64(5))
    data = torch.from_numpy(rng.integers(0, 256, size=n * ln, dtype=np.uint8)).to(dev)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * ln
    lens = torch.full((n,), ln, dtype=torch.int64, device=dev)
    out = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):          # one uncaptured call first (module load, constants)
        assert L.nw_dev_sha512_digest32_many(P(data), P(offs), P(lens), n, P(out),
                                             ctypes.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cs = torch.cuda.current_stream()
        assert L.nw_dev_sha512_digest32_many(P(data), P(offs), P(lens), n, P(out),
                                             ctypes.c_void_p(cs.cuda_stream)) == 0
        m = torch.zeros((4, 32), dtype=torch.uint8, device=dev)
        st = torch.zeros(4, dtype=torch.int32, device=dev)
        bm = torch.zeros(8, dtype=torch.uint8, device=dev)
        rc = L.nw_dev_verify_strict_many(P(m), 32, P(m), P(torch.zeros((4, 64), dtype=torch.uint8,
                                                                         device=dev)),
                                         4, P(st), P(bm), ctypes.c_void_p(cs.cuda_stream))
        assert rc == -1                 # NW_E_INVALID_ARG
    for rep in range(3):
        host = rng.integers(0, 256, size=n * ln, dtype=np.uint8)
        data.copy_(torch.from_numpy(host))
        g.replay()
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for i in range(n):
            assert got[i].tobytes() == hashlib.sha512(host[i * ln:(i + 1) * ln].tobytes()).digest()[:32]
