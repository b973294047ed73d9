"""The engine's host verification path (narwhal_amd/csrc/nw_host.cpp: the kernels' NW_HD
arithmetic compiled for the CPU; the certificate service's hedge) against the oracle, on the
CPU container (no device needed): the golden edge corpus and batches, batches with
z-dependent torsion residuals at irregular sizes, the certificate / header / vote streams of
the message tests and the irregular-committee shapes of tests/irregular.py. Injected z:
(status, index) bit-exact; random z: every verdict one the oracle gives for some z.
"""
import ctypes

import numpy as np
import pytest

from narwhal_amd import _lib
from narwhal_amd.messages import certificates_struct, committee_struct
from oracle import oracle as O
from tests import cert_cases as CC
from tests import irregular as IR


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _arr(hexes, width):
    return np.ascontiguousarray(
        np.array([np.frombuffer(bytes.fromhex(h), np.uint8) for h in hexes]).reshape(-1, width))


def host_strict(msgs, pks, sigs):
    n = len(pks)
    st = np.zeros(max(n, 1), np.int32)
    rc = _lib.lib().nw_host_verify_strict_many(_p(msgs), 32, _p(pks), _p(sigs), n, _p(st))
    assert rc == 0
    return st[:n]


def host_batch(digests, pks, sigs, offsets, z16=None):
    nb = len(offsets) - 1
    st = np.zeros(max(nb, 1), np.int32)
    fi = np.zeros(max(nb, 1), np.uint64)
    z = None if z16 is None else np.ascontiguousarray(z16, np.uint8)
    rc = _lib.lib().nw_host_verify_batch_many(_p(digests), _p(pks), _p(sigs), _p(offsets), nb,
                                              None if z is None else _p(z), _p(st), _p(fi))
    assert rc == 0
    return st[:nb], fi[:nb]


def host_certs(com, p, z16=None, headers_only=False):
    n = len(p["header_offsets"]) - 1
    st = np.zeros(max(n, 1), np.int32)
    ix = np.zeros(max(n, 1), np.uint64)
    cc, cs = committee_struct(com), certificates_struct(p, n)
    z = None if z16 is None else np.ascontiguousarray(z16, np.uint8)
    rc = _lib.lib().nw_host_certificates_verify_many(ctypes.byref(cc), ctypes.byref(cs),
                                                     None if z is None else _p(z),
                                                     1 if headers_only else 0, _p(st), _p(ix))
    assert rc == 0
    return st[:n], ix[:n]


def test_edge_corpus(golden):
    items = golden["edge_corpus"]["items"]
    st = host_strict(_arr([i["msg"] for i in items], 32), _arr([i["pk"] for i in items], 32),
                     _arr([i["sig"] for i in items], 64))
    assert [int(x) for x in st] == [i["status"] for i in items]


def test_golden_batches(golden):
    for b in golden["batches"]["batches"]:
        n = len(b["pks"])
        pks = _arr(b["pks"], 32) if n else np.zeros((0, 32), np.uint8)
        sigs = _arr(b["sigs"], 64) if n else np.zeros((0, 64), np.uint8)
        z = np.frombuffer(bytes.fromhex(b["z"]), np.uint8).reshape(n, 16) if n else None
        dg = np.frombuffer(bytes.fromhex(b["digest"]), np.uint8).reshape(1, 32).copy()
        off = np.array([0, n], np.uint64)
        st, fi = host_batch(dg, pks, sigs, off, z)
        assert (int(st[0]), int(fi[0])) == (b["status"], b["index"]), b["name"]
        if not b["name"].startswith("torsion_residual"):
            st, _ = host_batch(dg, pks, sigs, off, None)
            assert int(st[0]) == b["status"], b["name"]


def test_irregular_batches_injected_z():
    """Mixed-order signers (torsion residuals whose verdict depends on z) and damaged votes,
    ragged batch sizes, one call over many batches: equal to the oracle."""
    rng = np.random.Generator(np.random.PCG64(17))
    from tests.test_dalek_restatement import _irregular_batch
    batches = [_irregular_batch(int(k), 500 + i, bad=int(i % 3 == 0))
               for i, k in enumerate(rng.integers(1, 48, 14))]
    dg = np.stack([np.frombuffer(b[0], np.uint8) for b in batches])
    pks = np.concatenate([b[1] for b in batches])
    sigs = np.concatenate([b[2] for b in batches])
    z = np.concatenate([b[3] for b in batches])
    off = np.cumsum([0] + [len(b[1]) for b in batches]).astype(np.uint64)
    st, fi = host_batch(dg, pks, sigs, off, z)
    for j, b in enumerate(batches):
        want = O.verify_batch(b[0], b[1], b[2], b[3])
        assert (int(st[j]), int(fi[j])) == want, j
    assert len(set(st.tolist())) >= 2


def test_random_strict_set():
    from tests.test_dalek_restatement import _random_strict_set
    msgs, pks, sigs = _random_strict_set(600, 23)
    assert np.array_equal(host_strict(msgs, pks, sigs), O.verify_strict_many(msgs, pks, sigs))


@pytest.mark.parametrize("N", [4, 10])
def test_certificates_mutated_stream(N):
    com, p, exp_st, exp_ix, _ = CC.mutated_stream(N=N, copies=1, seed=N + 7)
    z = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(max(len(p["vote_pks"]), 1), 16),
                                                           dtype=np.uint8)
    st, ix = host_certs(com, p, z)
    ost, oix = O.certificates_verify_many(com, p, z)
    assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()
    st, ix = host_certs(com, p, None)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    hs, hx = host_certs(com, p, None, headers_only=True)
    ohs, ohx = O.certificates_verify_many(com, p, headers_only=True)
    assert hs.tolist() == ohs.tolist() and hx.tolist() == ohx.tolist()


@pytest.mark.parametrize("N,seed", [(4, 1), (4, 2), (10, 3), (16, 4)])
def test_certificates_irregular(N, seed):
    """Irregular committees (mixed-order, small-order, y >= p and undecodable members as
    authors and voters at every index): injected z bit-exact, random z within the oracle's
    possible verdicts."""
    com, p, kinds = IR.irregular_stream(N, 24, seed=seed)
    z = np.random.Generator(np.random.PCG64([N, seed])).integers(
        0, 256, size=(len(p["vote_pks"]), 16), dtype=np.uint8)
    st, ix = host_certs(com, p, z)
    ost, oix = O.certificates_verify_many(com, p, z)
    assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()
    st, ix = host_certs(com, p, None)
    poss = IR.possible_verdicts(com, p, 64, seed)
    for i in range(len(st)):
        v = (int(st[i]), int(ix[i]))
        assert v in poss[i] or IR.verdict_possible(com, p, i, v, seed), (i, v, poss[i])


def test_votes():
    vcom, vp, vn, vexp = CC.votes_case(N=8, seed=5, count=64)
    st = np.zeros(vn, np.int32)
    cc = committee_struct(vcom)
    rc = _lib.lib().nw_host_votes_verify_many(ctypes.byref(cc), _p(vp["ids"]), _p(vp["rounds"]),
                                              _p(vp["origins"]), _p(vp["authors"]), _p(vp["sigs"]),
                                              vn, _p(st))
    assert rc == 0 and st.tolist() == vexp.tolist()
