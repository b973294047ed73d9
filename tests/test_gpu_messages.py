"""GPU parity for the primary-message entry points (nw_certificates_verify_many,
nw_headers_verify_many, nw_votes_verify_many, nw_dev_certificates_verify_many) against the
oracle: status codes AND indices bit-exact, with injected batch coefficients; verdicts
equal with random coefficients on the deterministic set."""
import ctypes

import numpy as np
import pytest
import torch

from narwhal_amd import _lib
from narwhal_amd import messages as M
from narwhal_amd import workloads as W
from narwhal_amd.crypto import PublicKey, SecretKey, Signature
from oracle import oracle as O

from cert_cases import mutated_stream, oracle_digest_many, oracle_sign_many, votes_case
from test_messages import HEADER_LEVEL, fixture_header

pytestmark = pytest.mark.gpu


class _Com:
    """Adapter: a packed committee dict as a messages.Committee-like object."""

    def __init__(self, p):
        self._p = p

    def packed(self):
        return self._p


def test_appendix_b_fixture_through_mirror():
    keys, h = fixture_header()
    committee = M.Committee({PublicKey(pk): M.Authority(1) for pk, _ in keys})
    assert h.digest() == h.id                        # GPU SHA-512 over the header layout
    h.verify(committee)
    cert = M.Certificate(h)
    cd = cert.digest()
    cert.votes = [(PublicKey(pk), Signature.from_bytes(O.sign(sk, cd.value))) for pk, sk in keys]
    cert.verify(committee)
    for g in M.Certificate.genesis(committee):       # genesis certificates are always valid
        g.verify(committee)
    v = M.Vote.new(h, PublicKey(keys[0][0]), SecretKey(keys[0][1]))
    v.verify(committee)
    assert v.digest() == cd                          # Vote::digest == Certificate::digest
    bad = M.Certificate(h, cert.votes[:2])
    with pytest.raises(M.CertificateRequiresQuorum):
        bad.verify(committee)
    bad = M.Certificate(h, cert.votes[:2] + [cert.votes[0]])
    with pytest.raises(M.AuthorityReuse):
        bad.verify(committee)


@pytest.mark.parametrize("N,copies", [(4, 3), (10, 2), (50, 1), (100, 1)])
def test_certificates_vs_oracle(N, copies):
    com, s, exp_st, exp_ix, cls = mutated_stream(N=N, copies=copies, seed=N)
    z16 = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(len(s["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = M.verify_certificates_many(_Com(com), s, z16)
    ost, oix = O.certificates_verify_many(com, s, z16)
    assert np.array_equal(ost, exp_st) and np.array_equal(oix, exp_ix)
    bad = [(c, int(a), int(b), int(x), int(y)) for c, a, b, x, y in zip(cls, st, ost, ix, oix)
           if a != b or x != y]
    assert not bad, bad
    st2, ix2 = M.verify_certificates_many(_Com(com), s, None)   # CSPRNG coefficients
    assert np.array_equal(st2, exp_st) and np.array_equal(ix2, exp_ix)


def test_headers_vs_oracle():
    com, s, exp_st, exp_ix, cls = mutated_stream(N=4, copies=2)
    st, ix = M.verify_headers_many(_Com(com), s)
    ost, oix = O.certificates_verify_many(com, s, headers_only=True)
    assert np.array_equal(st, ost) and np.array_equal(ix, oix)
    assert all((a != 0) == (c in HEADER_LEVEL or c.startswith("genesis"))
               for a, c in zip(st, cls))


def test_headers_and_votes_keyed_fast_path_vs_full(monkeypatch):
    """The keyed fast path of the strict launches (compressed-R check, exact verification
    only for the leftovers; NW_STRICT_KEYED_FAST=0 turns it off): header and vote statuses,
    with every header-level failure class mixed into an honest stream, equal the full
    path's and the oracle's."""
    from cert_cases import pack, unpack
    from narwhal_amd import crypto as C
    com, ms, _, _, cls = mutated_stream(N=4, copies=6, seed=41)
    honest = W.certificate_stream(700, O.keys(4), lambda sk, m: C.sign_many(sk, m),
                                  oracle_digest_many, seed=43, n_votes=4)
    hrec, mrec = unpack(honest), unpack(ms)
    p = pack(hrec[:350] + mrec + hrec[350:])
    ost, oix = O.certificates_verify_many(com, p, headers_only=True)
    vcom, vp, vn, vexp = votes_case(N=8, seed=44, count=900)
    for fast in ("1", "0"):
        monkeypatch.setenv("NW_STRICT_KEYED_FAST", fast)
        st, ix = M.verify_headers_many(_Com(com), p)
        assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist(), fast
        assert M.verify_votes_many(_Com(vcom), vp).tolist() == vexp.tolist(), fast


def test_votes_vs_oracle():
    com, p, n, exp = votes_case()
    st = M.verify_votes_many(_Com(com), p)
    assert st.tolist() == exp.tolist() == O.votes_verify_many(com, p, n).tolist()


def test_votes_keyed_comb_many_vs_oracle():
    """Many votes of a 16-key committee through the keyed strict path (comb tables for the
    keys and for B, no ladder): every status equals the oracle's Vote::verify."""
    com, p, n, exp = votes_case(N=16, seed=21, count=3000)
    st = M.verify_votes_many(_Com(com), p)
    assert st.tolist() == exp.tolist() == O.votes_verify_many(com, p, n).tolist()


def test_committee_tables_reused_and_rebuilt():
    """Committee key tables are kept across calls with the same committee and rebuilt when
    it changes (device-side compare): committees A, B (same size, other keys), A again,
    each against the oracle."""
    ka = [O.keypair_from_seed(bytes([i + 1]) * 32) for i in range(6)]
    kb = [O.keypair_from_seed(bytes([i + 101]) * 32) for i in range(6)]
    for keys, seed in ((ka, 31), (kb, 32), (ka, 33), (ka, 34)):
        com, p, n, exp = votes_case(N=6, seed=seed, count=40, keys=keys)
        st = M.verify_votes_many(_Com(com), p)
        assert st.tolist() == exp.tolist() == O.votes_verify_many(com, p, n).tolist()


def test_certificate_stream_large_committee_payload():
    keys = O.keys(50)
    s = W.certificate_stream(40, keys, oracle_sign_many, oracle_digest_many, payload=3, seed=9)
    st, ix = M.verify_certificates_many(_Com(s["committee"]), s)
    assert st.tolist() == [0] * 40


@pytest.mark.parametrize("case_host", [True, False])
def test_device_entry_point_matches_host(case_host):
    """nw_dev_certificates_verify_many on device-resident buffers (the bench path), with and
    without the host copy of the vote offsets."""
    com, s, exp_st, exp_ix, cls = mutated_stream(N=4, copies=2, seed=11)
    n = len(s["header_offsets"]) - 1
    nv = int(s["vote_offsets"][-1])
    z16 = np.random.Generator(np.random.PCG64(2)).integers(0, 256, size=(nv, 16), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    T = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in s.items()}
    C = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in com.items()}
    zt = torch.from_numpy(z16).to(dev)
    L = _lib.lib()
    ws = torch.empty(L.nw_dev_certificates_workspace(n, nv), dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    ix = torch.empty(n, dtype=torch.int64, device=dev)
    P = lambda t: t.data_ptr()
    cc = M._CCommittee(len(com["stakes"]), P(C["pks"]), P(C["stakes"]), P(C["worker_offsets"]),
                       P(C["worker_ids"]))
    cs = M._CCertificates(n, P(T["header_bytes"]), P(T["header_offsets"]), P(T["payload_counts"]),
                          P(T["ids"]), P(T["header_sigs"]), P(T["vote_offsets"]), P(T["vote_pks"]),
                          P(T["vote_sigs"]), int(s["header_offsets"][-1]), nv,
                          s["vote_offsets"].ctypes.data if case_host else None)
    torch.cuda.synchronize()
    rc = L.nw_dev_certificates_verify_many(ctypes.byref(cc), ctypes.byref(cs), 0,
                                           ctypes.c_void_p(P(zt)), None, ctypes.c_void_p(P(ws)),
                                           ctypes.c_void_p(P(st)), ctypes.c_void_p(P(ix)), None)
    assert rc == 0, L.nw_last_error()
    assert L.nw_synchronize() == 0
    assert st.cpu().numpy().tolist() == exp_st.tolist()
    assert ix.cpu().numpy().astype(np.uint64).tolist() == exp_ix.tolist()


def test_committee_key_classes_vs_oracle():
    """Committee members whose keys are small-order / non-decodable: their pre-decompressed
    key tables must give the same Header::verify and Certificate::verify statuses as
    per-message decompression (oracle). Header authored by each member, votes by all."""
    import hashlib
    import struct
    keys = O.keys(4)
    small = bytes.fromhex("01" + "00" * 31)                      # identity: small order
    undec = (2).to_bytes(32, "little")                          # y = 2: not on the curve
    members = [pk for pk, _ in keys] + [small, undec]
    sk_of = dict(keys)
    com = M.Committee({PublicKey(pk): M.Authority(1) for pk in members})
    d32 = lambda b: hashlib.sha512(b).digest()[:32]
    certs = []
    for author in members:
        h = M.Header(author=PublicKey(author), round=3)
        h.id = M.Digest(d32(h.digest_bytes()))
        signer = sk_of.get(author, keys[0][1])                  # no key for small / undec
        h.signature = Signature.from_bytes(O.sign(signer, h.id.value))
        c = M.Certificate(h)
        cd = c.digest().value
        c.votes = [(PublicKey(pk), Signature.from_bytes(O.sign(sk_of.get(pk, keys[1][1]), cd)))
                   for pk in members]
        certs.append(c)
        c2 = M.Certificate(h)                                   # honest members only
        c2.votes = [(PublicKey(pk), Signature.from_bytes(O.sign(sk, cd))) for pk, sk in keys]
        certs.append(c2)
    p = M.pack_certificates(certs)
    z16 = np.random.Generator(np.random.PCG64(1)).integers(0, 256, size=(len(p["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = M.verify_certificates_many(com, p, z16)
    ost, oix = O.certificates_verify_many(com.packed(), p, z16)
    assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist()
    hst, _ = M.verify_headers_many(com, p)
    ohst, _ = O.certificates_verify_many(com.packed(), p, headers_only=True)
    assert hst.tolist() == ohst.tolist()
    assert {int(x) for x in hst} >= {0, 32 + 5, 32 + 3}         # Ok, A small order, A decode


def mixed_order_committee_certs(count: int = 16, seed: int = 77):
    """A committee of the 4 fixture keys plus a MIXED-ORDER member A = aB + T8 (decodes, not
    small order, [l]A = [lambda]T8 != 0). Certificates whose header is by a fixture key or by
    A, with votes by every member; A's signatures are made with its scalar a and a nonce
    chosen so that k = H(R||A||M) is 0 mod 8 (dalek's verify_strict ACCEPTS: R == [s]B - [k]A)
    or not (strict rejects). dalek's verify_batch weights A by (z k mod l), so even A's
    strict-valid votes leave [(z k mod l)]T8 in the batch sum: the certificate's verdict
    depends on z (tested with injected z). Returns (Committee, certificates)."""
    import hashlib
    import struct
    rng = np.random.Generator(np.random.PCG64(seed))
    L = 2**252 + 27742317777372353535851937790883648493
    keys = O.keys(4)
    t8 = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")
    a = (int.from_bytes(rng.bytes(32), "little") % L).to_bytes(32, "little")
    A = O.point_add(O.scalarmult_base(a), t8)
    assert O.is_small_order(A) == 0

    def sign_A(msg: bytes, k_zero: bool) -> bytes:
        for _ in range(200):
            sig = O.sign_raw(a, rng.bytes(32), A, msg)
            k = int.from_bytes(O.hram(sig[:32], A, msg), "little")
            if (k % 8 == 0) == k_zero:
                return sig
        raise AssertionError("no nonce found")

    sk_of = dict(keys)
    members = [pk for pk, _ in keys] + [A]
    com = M.Committee({PublicKey(pk): M.Authority(1) for pk in members})
    d32 = lambda b: hashlib.sha512(b).digest()[:32]
    certs = []
    for i in range(count):
        author = A if i % 3 == 0 else keys[i % 4][0]
        h = M.Header(author=PublicKey(author), round=5 + i)
        h.id = M.Digest(d32(h.digest_bytes()))
        hs = sign_A(h.id.value, i % 2 == 0) if author == A else O.sign(sk_of[author], h.id.value)
        h.signature = Signature.from_bytes(hs)
        c = M.Certificate(h)
        cd = d32(h.id.value + struct.pack("<Q", h.round) + author)   # Certificate::digest
        votes = []
        for pk in members:
            s = sign_A(cd, (i // 2) % 2 == 0) if pk == A else O.sign(sk_of[pk], cd)
            votes.append((PublicKey(pk), Signature.from_bytes(s)))
        c.votes = votes[i % 5:] + votes[:i % 5]            # A's vote at every position
        certs.append(c)
    return com, certs


def test_committee_mixed_order_key_vs_oracle():
    """Certificate::verify with a mixed-order committee key (mixed_order_committee_certs):
    with injected batch coefficients every status and index equals the oracle's dalek
    restatement, including certificates whose only irregular vote passes verify_strict
    (k = 0 mod 8) yet fails the batch equation for most z; Header::verify too."""
    com, certs = mixed_order_committee_certs()
    p = M.pack_certificates(certs)
    seen = set()
    for zs in range(3):
        z16 = np.random.Generator(np.random.PCG64(zs)).integers(
            0, 256, size=(len(p["vote_pks"]), 16), dtype=np.uint8)
        st, ix = M.verify_certificates_many(com, p, z16)
        ost, oix = O.certificates_verify_many(com.packed(), p, z16)
        assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist(), zs
        seen |= {int(x) for x in ost}
    assert seen >= {0, 32 + 7, 48 + 7}
    hst, hix = M.verify_headers_many(com, p)
    ohst, ohix = O.certificates_verify_many(com.packed(), p, headers_only=True)
    assert hst.tolist() == ohst.tolist() and hix.tolist() == ohix.tolist()
    assert {int(x) for x in ohst} >= {0, 32 + 7}


# ---- merged certificate groups (launch_cert_groups) ------------------------------------
def test_certificate_groups_vs_per_certificate(monkeypatch):
    """With random coefficients, Certificate::verify's vote batches are checked as one random
    linear combination per group of certificates and only failing groups are re-verified per
    certificate. Honest groups (including certificates that fail before their votes: header
    or pre-check classes, which contribute nothing) must pass the merged check; groups with a
    bad vote fall back. Statuses and indices equal the expected per-certificate ones, and the
    unmerged path (NW_CERT_MERGE=0)."""
    from cert_cases import pack, unpack
    from narwhal_amd import crypto as C
    com, ms, exp_st, exp_ix, cls = mutated_stream(N=4, copies=12, seed=7)
    honest = W.certificate_stream(3000, O.keys(4), lambda sk, m: C.sign_many(sk, m),
                                  oracle_digest_many, seed=11, n_votes=4)
    hrec, mrec = unpack(honest), unpack(ms)
    early = [i for i, c in enumerate(cls) if c in HEADER_LEVEL or c.startswith("genesis")]
    recs = hrec[:1500] + [mrec[i] for i in early] + hrec[1500:] + mrec
    exp = ([0] * 1500 + [int(exp_st[i]) for i in early] + [0] * 1500 + [int(x) for x in exp_st])
    expi = ([0] * 1500 + [int(exp_ix[i]) for i in early] + [0] * 1500 +
            [int(x) for x in exp_ix])
    p = pack(recs)
    monkeypatch.setenv("NW_CERT_GROUP_VOTES", "1024")
    st, ix = M.verify_certificates_many(_Com(com), p, None)
    assert st.tolist() == exp and ix.tolist() == expi
    monkeypatch.setenv("NW_CERT_MERGE", "0")
    st0, ix0 = M.verify_certificates_many(_Com(com), p, None)
    assert st0.tolist() == exp and ix0.tolist() == expi


@pytest.mark.parametrize("N", [4, 10, 50, 100])
def test_certificate_groups_honest_and_one_bad(monkeypatch, N):
    """Merged groups (NW_CERT_KEYED=0) of the default size over an honest stream (every
    group passes the merged check), then one bad vote signature: only that certificate
    fails (its group falls back); the default keyed checks and the unmerged path agree."""
    from narwhal_amd import crypto as C
    monkeypatch.setenv("NW_CERT_KEYED", "0")
    keys = O.keys(N)
    n = max(2000, 70000 // (2 * N // 3 + 1))
    s = W.certificate_stream(n, keys, lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                             seed=N, n_votes=None)
    com = _Com(s["committee"])
    st, _ = M.verify_certificates_many(com, s, None)
    assert (st == 0).all()
    bad = n // 2
    v = int(s["vote_offsets"][bad]) + 1
    s["vote_sigs"][v, 7] ^= 0x40
    st, ix = M.verify_certificates_many(com, s, None)
    assert st[bad] != 0 and (np.delete(st, bad) == 0).all()
    monkeypatch.delenv("NW_CERT_KEYED")
    stk, ixk = M.verify_certificates_many(com, s, None)
    assert stk.tolist() == st.tolist() and ixk[bad] == ix[bad]
    monkeypatch.setenv("NW_CERT_MERGE", "0")
    st0, ix0 = M.verify_certificates_many(com, s, None)
    assert st0.tolist() == st.tolist() and ix0[bad] == ix[bad]


@pytest.mark.parametrize("N,n", [(4, 6000), (10, 3000), (100, 600)])
def test_certificate_groups_mixed_validity(monkeypatch, N, n):
    """About 1% of the certificates carry one invalid vote (equation, s high bits, R not on
    the curve: workloads.mutate_votes), spread over many merged groups
    (NW_CERT_GROUP_VOTES=4096). Every group with a bad certificate falls back; statuses and
    indices equal the construction (pinned by the oracle in tests/test_messages.py) and
    the unmerged path, with random coefficients as in the reference."""
    from narwhal_amd import crypto as C
    keys = O.keys(N)
    s = W.certificate_stream(n, keys, lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                             seed=100 + N)
    bad = np.arange(37 % n, n, 100)
    m, exp_st, exp_ix = W.mutate_votes(s, bad, seed=N)
    com = _Com(s["committee"])
    monkeypatch.setenv("NW_CERT_GROUP_VOTES", "4096")
    st, ix = M.verify_certificates_many(com, m, None)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    monkeypatch.setenv("NW_CERT_MERGE", "0")
    st0, ix0 = M.verify_certificates_many(com, m, None)
    assert st0.tolist() == exp_st.tolist() and ix0.tolist() == exp_ix.tolist()


@pytest.mark.parametrize("N,n,K", [(4, 6000, 1), (4, 6000, 8), (10, 3000, 5), (100, 600, 3),
                                   (100, 600, 32)])
def test_certificate_small_groups_mixed_validity(monkeypatch, N, n, K):
    """Small groups (launch_cert_sgroups, NW_CERT_SMALL_K = K certificates per keyed Straus
    check, then the per-certificate ladders of failed groups from the same items): about 1%
    of the certificates carry one invalid vote of every class (workloads.mutate_votes);
    statuses and indices equal the construction and the unmerged path."""
    from narwhal_amd import crypto as C
    keys = O.keys(N)
    s = W.certificate_stream(n, keys, lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                             seed=200 + N)
    bad = np.arange(11 % n, n, 97)
    m, exp_st, exp_ix = W.mutate_votes(s, bad, seed=N + K)
    com = _Com(s["committee"])
    monkeypatch.setenv("NW_CERT_SMALL_K", str(K))
    st, ix = M.verify_certificates_many(com, m, None)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    st, _ = M.verify_certificates_many(com, s, None)      # honest: every group passes
    assert (st == 0).all()
    monkeypatch.setenv("NW_BATCH_SLICE_UNITS", "20000")   # several slices of whole groups
    st, ix = M.verify_certificates_many(com, m, None)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    monkeypatch.delenv("NW_BATCH_SLICE_UNITS")
    monkeypatch.setenv("NW_CERT_MERGE", "0")
    st0, ix0 = M.verify_certificates_many(com, m, None)
    assert st0.tolist() == exp_st.tolist() and ix0.tolist() == exp_ix.tolist()


def test_certificate_small_groups_early_failures(monkeypatch):
    """Small groups mixing honest certificates with every header-level and pre-check failure
    class (they contribute no votes) and every vote-level class: statuses and indices equal
    the expected per-certificate ones."""
    from cert_cases import pack, unpack
    from narwhal_amd import crypto as C
    com, ms, exp_st, exp_ix, cls = mutated_stream(N=4, copies=12, seed=9)
    honest = W.certificate_stream(600, O.keys(4), lambda sk, m: C.sign_many(sk, m),
                                  oracle_digest_many, seed=13, n_votes=4)
    hrec, mrec = unpack(honest), unpack(ms)
    recs = hrec[:300] + mrec + hrec[300:]
    exp = [0] * 300 + [int(x) for x in exp_st] + [0] * 300
    expi = [0] * 300 + [int(x) for x in exp_ix] + [0] * 300
    p = pack(recs)
    for K in (2, 7, 32):
        monkeypatch.setenv("NW_CERT_SMALL_K", str(K))
        st, ix = M.verify_certificates_many(_Com(com), p, None)
        assert st.tolist() == exp and ix.tolist() == expi, K


@pytest.mark.parametrize("N,n", [(4, 6000), (10, 3000), (50, 800), (100, 600)])
def test_certificate_keyed_votes_mixed_validity(monkeypatch, N, n):
    """Keyed vote checks (launch_votes_keyed, NW_CERT_KEYED=1: every vote through the keyed
    comb, then verify_batch only for certificates with a failing vote): about 1% of the
    certificates carry one invalid vote of every class (workloads.mutate_votes); statuses
    and indices equal the construction and the unmerged path, with the votes checked in
    certificate order and in key-major order; an honest stream is all Ok."""
    from narwhal_amd import crypto as C
    keys = O.keys(N)
    s = W.certificate_stream(n, keys, lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                             seed=300 + N)
    bad = np.arange(5 % n, n, 89)
    m, exp_st, exp_ix = W.mutate_votes(s, bad, seed=N + 3)
    com = _Com(s["committee"])
    monkeypatch.setenv("NW_CERT_KEYED", "1")
    for order in ("0", "1"):   # cert-major and key-major vote order (k_vk_* counting sort)
        monkeypatch.setenv("NW_VOTES_KEY_MAJOR", order)
        st, ix = M.verify_certificates_many(com, m, None)
        assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist(), order
        st, _ = M.verify_certificates_many(com, s, None)
        assert (st == 0).all(), order
    monkeypatch.delenv("NW_VOTES_KEY_MAJOR")
    monkeypatch.delenv("NW_CERT_KEYED")
    monkeypatch.setenv("NW_CERT_MERGE", "0")
    st0, ix0 = M.verify_certificates_many(com, m, None)
    assert st0.tolist() == exp_st.tolist() and ix0.tolist() == exp_ix.tolist()


def test_certificate_keyed_votes_early_failures(monkeypatch):
    """Keyed vote checks over honest certificates mixed with every header-level, pre-check
    and vote-level failure class (mutated_stream): statuses and indices equal the expected
    per-certificate ones."""
    from cert_cases import pack, unpack
    from narwhal_amd import crypto as C
    com, ms, exp_st, exp_ix, cls = mutated_stream(N=4, copies=12, seed=19)
    honest = W.certificate_stream(600, O.keys(4), lambda sk, m: C.sign_many(sk, m),
                                  oracle_digest_many, seed=23, n_votes=4)
    hrec, mrec = unpack(honest), unpack(ms)
    p = pack(hrec[:300] + mrec + hrec[300:])
    exp = [0] * 300 + [int(x) for x in exp_st] + [0] * 300
    expi = [0] * 300 + [int(x) for x in exp_ix] + [0] * 300
    monkeypatch.setenv("NW_CERT_KEYED", "1")
    for order in ("0", "1"):   # key-major: decided certificates' votes sort into the last bin
        monkeypatch.setenv("NW_VOTES_KEY_MAJOR", order)
        st, ix = M.verify_certificates_many(_Com(com), p, None)
        assert st.tolist() == exp and ix.tolist() == expi, order


def test_certificate_groups_adaptive_repeated_calls(monkeypatch):
    """The merged-group policy (NW_CERT_KEYED=0; nw_api.cpp group_failure_rate): a stream
    with ~1% failing certificates moves from the big merged groups to small groups from the
    next call on (the measured rate makes most big groups fail), and back once an honest
    stream reports no failures; every call's statuses and indices equal the construction,
    whichever path ran. Then the same calls with the default keyed checks."""
    from narwhal_amd import crypto as C
    monkeypatch.setenv("NW_CERT_KEYED", "0")
    N, n = 10, 5200
    s = W.certificate_stream(n, O.keys(N), lambda sk, m: C.sign_many(sk, m), oracle_digest_many,
                             seed=77)
    m, exp_st, exp_ix = W.mutate_votes(s, np.arange(13, n, 100), seed=5)
    com = _Com(s["committee"])
    for _ in range(10):
        st, ix = M.verify_certificates_many(com, m, None)
        assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    for _ in range(3):
        st, ix = M.verify_certificates_many(com, s, None)     # honest again
        assert (st == 0).all()
    monkeypatch.delenv("NW_CERT_KEYED")
    for _ in range(3):
        st, ix = M.verify_certificates_many(com, m, None)
        assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
        st, ix = M.verify_certificates_many(com, s, None)
        assert (st == 0).all()
