"""CPU tests for the primary-message layer: the oracle's Header / Vote / Certificate
restatement pinned against the reference fixtures (SURVEY Appendix B values derived from
primary/src/tests/common.rs:96-112, 136-170) and against hand-written expectations for
every DagError class; the host mirror's digest layouts against hashlib."""
import base64
import hashlib
import struct

import numpy as np
import pytest

from narwhal_amd import workloads as W
from narwhal_amd.crypto import Digest, PublicKey, Signature
from narwhal_amd.messages import Authority, Certificate, Committee, Header
from oracle import oracle as O

from cert_cases import MAX, mutated_stream, oracle_digest_many, oracle_sign_many, votes_case


def d32(b: bytes) -> bytes:
    return hashlib.sha512(b).digest()[:32]


def fixture_header():
    """primary/src/tests/common.rs header(): author = keys().pop(), round 1, parents =
    digests of Certificate::genesis(&committee())."""
    keys = O.keys(4)
    author, secret = keys[-1]
    genesis = {Digest(d32(bytes(32) + struct.pack("<Q", 0) + pk)) for pk, _ in keys}
    h = Header(author=PublicKey(author), round=1, parents=genesis)
    hid = d32(h.digest_bytes())
    h.id = Digest(hid)
    h.signature = Signature.from_bytes(O.sign(secret, hid))
    return keys, h


def test_appendix_b_header_and_certificate(golden):
    ab = golden["keys"]["appendix_b"]
    keys, h = fixture_header()
    assert base64.b64encode(h.id.value).decode() == ab["header_id_b64"]
    assert h.signature.flatten().hex() == ab["header_sig"]
    cd = d32(h.id.value + struct.pack("<Q", 1) + h.author.value)
    assert base64.b64encode(cd).decode() == ab["certificate_digest_b64"]
    # certificate(header()): votes by every fixture key over Certificate::digest
    cert = Certificate(h, [(PublicKey(pk), Signature.from_bytes(O.sign(sk, cd))) for pk, sk in keys])
    committee = Committee({PublicKey(pk): Authority(1) for pk, _ in keys})
    from narwhal_amd.messages import pack_certificates, pack_committee
    p, c = pack_certificates([cert]), pack_committee(committee)
    st, ix = O.certificates_verify_many(c, p)
    assert st.tolist() == [0]
    st, _ = O.certificates_verify_many(c, p, headers_only=True)
    assert st.tolist() == [0]


def test_proposer_payload_header():
    """primary/src/tests/proposer_tests.rs:35-68: payload {Digest(name.0): 0} verifies."""
    keys = O.keys(4)
    name, secret = keys[-1]
    h = Header(author=PublicKey(name), round=1, payload={Digest(name): 0})
    h.id = Digest(d32(h.digest_bytes()))
    h.signature = Signature.from_bytes(O.sign(secret, h.id.value))
    assert h.digest_bytes() == name + struct.pack("<Q", 1) + name + struct.pack("<I", 0)
    committee = Committee({PublicKey(pk): Authority(1) for pk, _ in keys})
    from narwhal_amd.messages import pack_certificates, pack_committee
    st, _ = O.certificates_verify_many(pack_committee(committee), pack_certificates([h]),
                                       headers_only=True)
    assert st.tolist() == [0]


def test_header_digest_layout_orders():
    """BTreeMap / BTreeSet iteration = byte-lexicographic order of the digests."""
    a, b, c = Digest(b"\x02" * 32), Digest(b"\x01" * 32), Digest(b"\x03" + b"\0" * 31)
    h = Header(author=PublicKey(b"\x09" * 32), round=7, payload={a: 5, b: 6}, parents={c, a})
    exp = (b"\x09" * 32 + struct.pack("<Q", 7) + b.value + struct.pack("<I", 6) + a.value
           + struct.pack("<I", 5) + a.value + c.value)
    assert h.digest_bytes() == exp


@pytest.mark.parametrize("n,q", [(4, 3), (10, 7), (50, 34), (100, 67)])
def test_quorum_threshold(n, q):
    c = Committee({PublicKey(bytes([i]) * 32): Authority(1) for i in range(n)})
    assert c.quorum_threshold() == q == W.quorum(n)


def test_oracle_dag_error_classes():
    com, s, exp_st, exp_ix, cls = mutated_stream(N=4)
    z16 = np.random.Generator(np.random.PCG64(1)).integers(0, 256, size=(len(s["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = O.certificates_verify_many(com, s, z16)
    bad = [(c, int(a), int(b), int(x), int(y)) for c, a, b, x, y in
           zip(cls, st, exp_st, ix, exp_ix) if a != b or x != y]
    assert not bad, bad
    # random coefficients (OS CSPRNG): same verdicts on this deterministic set
    st2, ix2 = O.certificates_verify_many(com, s, None)
    assert np.array_equal(st2, exp_st) and np.array_equal(ix2, exp_ix)


HEADER_LEVEL = {"id_flip", "author_outsider", "author_zero_stake", "bad_worker_id",
                "header_sig_flip", "header_sig_high", "id_flip_and_bad_votes"}


def test_oracle_headers_only():
    """Header::verify has no genesis rule and never looks at votes."""
    com, s, exp_st, exp_ix, cls = mutated_stream(N=4)
    st, ix = O.certificates_verify_many(com, s, headers_only=True)
    for c, a, e, x, ex in zip(cls, st, exp_st, ix, exp_ix):
        if c.startswith("genesis"):
            assert a == 16
        elif c in HEADER_LEVEL:
            assert (a, x) == (e, ex), c
        else:
            assert (a, x) == (0, 0), c


def test_oracle_votes():
    com, p, n, exp = votes_case()
    assert O.votes_verify_many(com, p, n).tolist() == exp.tolist()


def test_certificate_stream_generator_honest():
    keys = O.keys(10)
    s = W.certificate_stream(12, keys, oracle_sign_many, oracle_digest_many, payload=2, seed=3)
    assert s["q"] == 7
    st, ix = O.certificates_verify_many(s["committee"], s)
    assert st.tolist() == [0] * 12
    # round / author layout (Certificate i: author keys[i % N], round 1 + i // N)
    hb = s["header_bytes"].reshape(12, -1)
    assert bytes(hb[3, :32]) == keys[3][0]
    assert struct.unpack("<Q", bytes(hb[11, 32:40]))[0] == 2
    assert hb.shape[1] == 40 + 36 * 2 + 32 * 7


@pytest.mark.parametrize("N", [4, 10, 100])
def test_mutate_votes_expectations_pinned_by_oracle(N):
    """workloads.mutate_votes (the bench's invalid-certificate legs) states each mutated
    certificate's Certificate::verify status and index by construction; the oracle agrees,
    with injected and with random coefficients (the mutations are all in the
    deterministic set: no torsion residuals)."""
    keys = O.keys(N)
    n = 30 if N < 100 else 9
    s = W.certificate_stream(n, keys, oracle_sign_many, oracle_digest_many, seed=N)
    bad = np.arange(1, n, 2)
    m, exp_st, exp_ix = W.mutate_votes(s, bad, seed=N)
    assert {int(x) for x in exp_st} == {0, 48 + 7, 48 + 1, 48 + 4}
    z16 = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(len(m["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = O.certificates_verify_many(s["committee"], m, z16)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    st, ix = O.certificates_verify_many(s["committee"], m)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    assert np.array_equal(s["vote_sigs"][0], m["vote_sigs"][0])   # input stream untouched
