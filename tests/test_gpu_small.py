"""GPU parity of the small-job launch (narwhal_amd/csrc/nw_small.hip: Header / Vote /
Certificate checks of a job in ONE kernel, the aggregation service's latency path) against
the oracle: statuses AND indices bit-exact with injected batch coefficients, equal to the
construction with CSPRNG coefficients; every workgroup size S (slots per workgroup: messages
spanning workgroups go through the arrival counters); certificates whose batch verdict
depends on torsion (a mixed-order committee key; votes whose R carries a torsion point).

NW_SMALL=1 makes every qualifying job take the small path whatever its size; a committee's
first job builds its key tables in the ordinary pipeline, so each check runs its job twice
and requires the second to be a small-job launch (nw_path_stats)."""
import hashlib
import struct

import numpy as np
import pytest

from narwhal_amd import _lib
from narwhal_amd import messages as M
from narwhal_amd import workloads as W
from narwhal_amd.crypto import PublicKey, Signature
from oracle import oracle as O

from cert_cases import mutated_stream, oracle_digest_many, oracle_sign_many, votes_case
from test_gpu_messages import _Com, mixed_order_committee_certs

pytestmark = pytest.mark.gpu

L_ORDER = 2**252 + 27742317777372353535851937790883648493
T8 = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")


def _small(monkeypatch, S=None):
    monkeypatch.setenv("NW_SMALL", "1")
    if S is not None:
        monkeypatch.setenv("NW_SMALL_S", str(S))


def _twice(fn):
    """fn() twice; the second run must be small-job launches only."""
    fn()
    s0, p0 = _lib.path_stats()
    out = fn()
    s1, p1 = _lib.path_stats()
    assert s1 > s0 and p1 == p0, ("small path not taken", s0, s1, p0, p1)
    return out


@pytest.mark.parametrize("N,copies,S", [(4, 3, 4), (4, 3, 64), (10, 2, 8), (50, 1, 4),
                                        (50, 1, 32), (100, 1, 4), (100, 1, 16)])
def test_small_certificates_vs_oracle(monkeypatch, N, copies, S):
    """Every Certificate::verify failure class (cert_cases.mutated_stream: header, quorum,
    vote classes), injected z: status and index == the oracle's; CSPRNG z: == the
    construction (pinned by the oracle in tests/test_messages.py)."""
    _small(monkeypatch, S)
    com, s, exp_st, exp_ix, cls = mutated_stream(N=N, copies=copies, seed=N + 100)
    z16 = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(len(s["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = _twice(lambda: M.verify_certificates_many(_Com(com), s, z16))
    ost, oix = O.certificates_verify_many(com, s, z16)
    bad = [(c, int(a), int(b), int(x), int(y)) for c, a, b, x, y in zip(cls, st, ost, ix, oix)
           if a != b or x != y]
    assert not bad, bad
    st2, ix2 = _twice(lambda: M.verify_certificates_many(_Com(com), s, None))
    assert st2.tolist() == exp_st.tolist() and ix2.tolist() == exp_ix.tolist()


@pytest.mark.parametrize("S", [4, 64])
def test_small_headers_vs_oracle(monkeypatch, S):
    _small(monkeypatch, S)
    com, s, _, _, _ = mutated_stream(N=4, copies=3, seed=17)
    st, ix = _twice(lambda: M.verify_headers_many(_Com(com), s))
    ost, oix = O.certificates_verify_many(com, s, headers_only=True)
    assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()


@pytest.mark.parametrize("N,count,S", [(4, 24, 4), (16, 700, 16), (16, 700, 64)])
def test_small_votes_vs_oracle(monkeypatch, N, count, S):
    _small(monkeypatch, S)
    com, p, n, exp = votes_case(N=N, seed=N + count, count=count)
    st = _twice(lambda: M.verify_votes_many(_Com(com), p))
    assert st.tolist() == exp.tolist() == O.votes_verify_many(com, p, n).tolist()


def test_small_committee_key_classes(monkeypatch):
    """Committee members whose keys are small-order / non-decodable (their votes reach the
    batch with A decode failures, or small-order A with the batch equation checked as
    dalek does), certificates and headers by every member, injected z: == the oracle."""
    _small(monkeypatch)
    keys = O.keys(4)
    small = bytes.fromhex("01" + "00" * 31)
    undec = (2).to_bytes(32, "little")
    members = [pk for pk, _ in keys] + [small, undec]
    sk_of = dict(keys)
    com = M.Committee({PublicKey(pk): M.Authority(1) for pk in members})
    d32 = lambda b: hashlib.sha512(b).digest()[:32]
    certs = []
    for author in members:
        h = M.Header(author=PublicKey(author), round=3)
        h.id = M.Digest(d32(h.digest_bytes()))
        h.signature = Signature.from_bytes(O.sign(sk_of.get(author, keys[0][1]), h.id.value))
        cd = d32(h.id.value + struct.pack("<Q", h.round) + author)
        c = M.Certificate(h)
        c.votes = [(PublicKey(pk), Signature.from_bytes(O.sign(sk_of.get(pk, keys[1][1]), cd)))
                   for pk in members]
        certs.append(c)
        c2 = M.Certificate(h)
        c2.votes = [(PublicKey(pk), Signature.from_bytes(O.sign(sk, cd))) for pk, sk in keys]
        certs.append(c2)
        c3 = M.Certificate(h)   # the small-order member votes with R = [s]B: batch-valid
        sv = int.from_bytes(hashlib.sha512(cd).digest()[:32], "little") % L_ORDER
        sb = sv.to_bytes(32, "little")
        c3.votes = [(PublicKey(pk), Signature.from_bytes(O.sign(sk, cd))) for pk, sk in keys]
        c3.votes.append((PublicKey(small), Signature.from_bytes(O.scalarmult_base(sb) + sb)))
        certs.append(c3)
    p = M.pack_certificates(certs)
    z16 = np.random.Generator(np.random.PCG64(1)).integers(0, 256, size=(len(p["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = _twice(lambda: M.verify_certificates_many(com, p, z16))
    ost, oix = O.certificates_verify_many(com.packed(), p, z16)
    assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()
    assert {int(x) for x in ost} >= {0, 48 + 3}
    hst, hix = _twice(lambda: M.verify_headers_many(com, p))
    ohst, ohix = O.certificates_verify_many(com.packed(), p, headers_only=True)
    assert hst.tolist() == ohst.tolist() and hix.tolist() == ohix.tolist()


def _scalar_a(sk: bytes) -> int:
    h = bytearray(hashlib.sha512(sk[:32]).digest()[:32])
    h[0] &= 248
    h[31] = (h[31] & 127) | 64
    return int.from_bytes(h, "little") % L_ORDER


def torsion_r_certs(count: int = 24, seed: int = 5):
    """Honest N = 4 certificates in which some votes carry R'' = rB + [t]T8 with
    s = r + H(R'' || A || M) a: then [s]B - [k]A = rB and the vote's residual is the pure
    torsion point [t]T8 (strict rejects it: R'' is not [s]B - [k]A; dalek's batch sum is
    [z t]T8 plus the other votes' terms). Returns (Committee, certificates)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    keys = O.keys(4)
    tors = [bytes.fromhex("01" + "00" * 31)]
    for _ in range(7):
        tors.append(O.point_add(tors[-1], T8))
    com = M.Committee({PublicKey(pk): M.Authority(1) for pk, _ in keys})
    d32 = lambda b: hashlib.sha512(b).digest()[:32]
    certs = []
    for i in range(count):
        pk0, sk0 = keys[i % 4]
        h = M.Header(author=PublicKey(pk0), round=9 + i)
        h.id = M.Digest(d32(h.digest_bytes()))
        h.signature = Signature.from_bytes(O.sign(sk0, h.id.value))
        cd = d32(h.id.value + struct.pack("<Q", h.round) + pk0)
        votes = []
        for v, (pk, sk) in enumerate(keys):
            t = (i + v) % 8 if (i + v) % 3 == 0 else 0
            if t:
                r = int.from_bytes(rng.bytes(32), "little") % L_ORDER
                R = O.point_add(O.scalarmult_base(r.to_bytes(32, "little")), tors[t])
                k = int.from_bytes(O.hram(R, pk, cd), "little")
                s = (r + k * _scalar_a(sk)) % L_ORDER
                votes.append((PublicKey(pk), Signature.from_bytes(R + s.to_bytes(32, "little"))))
            else:
                votes.append((PublicKey(pk), Signature.from_bytes(O.sign(sk, cd))))
        c = M.Certificate(h)
        c.votes = votes
        certs.append(c)
    return com, certs


def test_small_torsion_verdicts_vs_oracle(monkeypatch):
    """Certificates whose batch verdict depends on z: votes with torsion residuals
    (torsion_r_certs) and a mixed-order committee key (its strict-valid votes still leave
    [(z k mod l)]T8 in dalek's sum). Six injected coefficient sets: every status and index
    == the oracle's; both verdicts occur."""
    for S in (4, 64):
        _small(monkeypatch, S)
        seen = set()
        for com, certs in (torsion_r_certs(), mixed_order_committee_certs()):
            p = M.pack_certificates(certs)
            for zs in range(6):
                z16 = np.random.Generator(np.random.PCG64(100 + zs)).integers(
                    0, 256, size=(len(p["vote_pks"]), 16), dtype=np.uint8)
                st, ix = _twice(lambda: M.verify_certificates_many(com, p, z16))
                ost, oix = O.certificates_verify_many(com.packed(), p, z16)
                assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist(), (S, zs)
                seen |= {int(x) for x in ost}
        assert seen >= {0, 48 + 7}, seen


@pytest.mark.parametrize("N,n", [(4, 3000), (50, 300)])
def test_small_mixed_validity_random_z(monkeypatch, N, n):
    """About 1% of the certificates carry one invalid vote of every class
    (workloads.mutate_votes), CSPRNG coefficients: the small path's statuses and indices ==
    the construction and == the bulk pipeline's (NW_SMALL=0)."""
    from narwhal_amd import crypto as C
    keys = O.keys(N)
    s = W.certificate_stream(n, keys, lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                             seed=500 + N)
    m, exp_st, exp_ix = W.mutate_votes(s, np.arange(7 % n, n, 97), seed=N + 1)
    com = _Com(s["committee"])
    _small(monkeypatch)
    st, ix = _twice(lambda: M.verify_certificates_many(com, m, None))
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    st, _ = _twice(lambda: M.verify_certificates_many(com, s, None))
    assert (st == 0).all()
    monkeypatch.setenv("NW_SMALL", "0")
    s0, _ = _lib.path_stats()
    stp, ixp = M.verify_certificates_many(com, m, None)
    assert _lib.path_stats()[0] == s0
    assert stp.tolist() == exp_st.tolist() and ixp.tolist() == exp_ix.tolist()


@pytest.mark.parametrize("N,payload,S", [(100, 32, 4), (100, 64, 4), (50, 80, 4), (10, 0, 64)])
def test_small_header_digest_sizes(monkeypatch, N, payload, S):
    """The header digest of the small-job kernel (nw_small.hip header_digest): one owned
    header per wave hashes with its block schedules spread over lanes up to 32 blocks (N =
    100 with 32 payload entries: 27 blocks; N = 50 with 80: exactly 32), a larger header
    (N = 100, 64 entries: 36 blocks) and several owned headers per wave (N = 10, S = 64) on
    one lane each. Honest
    certificates (the construction: Ok) and the same with every header id flipped in one
    byte (InvalidHeaderId) - statuses and indices == the oracle's."""
    _small(monkeypatch, S)
    keys = O.keys(N)
    s = W.certificate_stream(6, keys, oracle_sign_many, oracle_digest_many, payload=payload,
                             seed=N + payload)
    com = _Com(s["committee"])
    st, ix = _twice(lambda: M.verify_certificates_many(com, s, None))
    assert st.tolist() == [0] * 6
    bad = dict(s)
    bad["ids"] = s["ids"].copy()
    bad["ids"][:, 5] ^= 0x10
    z16 = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(len(s["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = _twice(lambda: M.verify_certificates_many(com, bad, z16))
    ost, oix = O.certificates_verify_many(s["committee"], bad, z16)
    assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()
    assert set(st.tolist()) == {16}    # NW_DAG_INVALID_HEADER_ID
