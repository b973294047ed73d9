"""Pins the CPU oracle (oracle/libnw_oracle.so) against the committed golden fixtures
and independent implementations (hashlib, libsodium 1.0.18 when present).

The reference holds no known-answer vectors for this path; these
fixtures come from tests/golden/gen_golden.py (hashlib, libsodium, RFC 8032 literals,
SURVEY Appendix B literals).
"""
import base64
import ctypes
import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as O
from narwhal_amd import workloads as W

SODIUM = "/opt/conda/lib/libsodium.so"


def test_sha512_vectors(golden):
    for v in golden["sha512"]["vectors"]:
        assert O.sha512(bytes.fromhex(v["msg"])).hex() == v["sha512"], v["name"]


def test_sha512_worker_batches(golden):
    for v in golden["sha512"]["worker_batches"]:
        m = W.worker_batch(v["batch_id"], seed=v["seed"]).tobytes()
        assert len(m) == v["len"] == W.BATCH_BYTES
        assert O.sha512(m).hex() == v["sha512"]


def test_sha512_many_ragged():
    data, offs, lens = W.ragged_messages(300, 700, seed=3)
    out = O.sha512_digest32_many(data, offs, lens, nthreads=2)
    for i in range(300):
        m = data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
        assert out[i].tobytes() == hashlib.sha512(m).digest()[:32]


def test_reference_keys_fixture(golden):
    g = golden["keys"]
    ks = O.keys(4)
    for (pk, sk), ref in zip(ks, g["stdrng_zero_seed_keys"]):
        assert sk[:32].hex() == ref["seed"] and pk.hex() == ref["pk"]
    d = O.digest32(b"Hello, world!")
    assert d.hex() == g["hello_digest"]
    assert O.sign(ks[3][1], d).hex() == g["hello_sig_key3"]


def test_rfc8032(golden):
    for v in golden["keys"]["rfc8032"]:
        pk, sk = O.keypair_from_seed(bytes.fromhex(v["seed"]))
        assert pk.hex() == v["pk"]
        m = bytes.fromhex(v["msg"])
        assert O.sign(sk, m).hex() == v["sig"]
        assert O.verify_strict(m, pk, bytes.fromhex(v["sig"])) == O.OK


def test_edge_corpus(golden):
    for it in golden["edge_corpus"]["items"]:
        st = O.verify_strict(bytes.fromhex(it["msg"]), bytes.fromhex(it["pk"]), bytes.fromhex(it["sig"]))
        assert st == it["status"], it["class"]


def test_edge_corpus_many(golden):
    items = golden["edge_corpus"]["items"]
    msgs = np.array([np.frombuffer(bytes.fromhex(i["msg"]), np.uint8) for i in items])
    pks = np.array([np.frombuffer(bytes.fromhex(i["pk"]), np.uint8) for i in items])
    sigs = np.array([np.frombuffer(bytes.fromhex(i["sig"]), np.uint8) for i in items])
    st = O.verify_strict_many(msgs, pks, sigs, nthreads=2)
    assert list(st) == [i["status"] for i in items]


def test_batches(golden):
    for b in golden["batches"]["batches"]:
        n = len(b["pks"])
        pks = np.array([np.frombuffer(bytes.fromhex(p), np.uint8) for p in b["pks"]]).reshape(n, 32)
        sigs = np.array([np.frombuffer(bytes.fromhex(s), np.uint8) for s in b["sigs"]]).reshape(n, 64)
        z = np.frombuffer(bytes.fromhex(b["z"]), np.uint8).reshape(n, 16) if n else None
        st, idx = O.verify_batch(bytes.fromhex(b["digest"]), pks, sigs, z)
        assert (st, idx) == (b["status"], b["index"]), b["name"]


def test_batch_random_z_deterministic_set(golden):
    """Without injected z the verdict equals the injected-z verdict on every batch whose
    outcome does not depend on z."""
    for b in golden["batches"]["batches"]:
        if b["name"].startswith("torsion_residual"):
            continue
        n = len(b["pks"])
        pks = np.array([np.frombuffer(bytes.fromhex(p), np.uint8) for p in b["pks"]]).reshape(n, 32)
        sigs = np.array([np.frombuffer(bytes.fromhex(s), np.uint8) for s in b["sigs"]]).reshape(n, 64)
        st, _ = O.verify_batch(bytes.fromhex(b["digest"]), pks, sigs, None)
        assert st == b["status"], b["name"]


def test_msm_pippenger_equals_straus():
    """ge_msm switches algorithm at 190 points; both must give the same group element."""
    rng = np.random.Generator(np.random.PCG64(5))
    pts = [O.scalarmult_base(rng.bytes(32)) for _ in range(200)]
    sc = [rng.bytes(31) + b"\x00" for _ in range(200)]
    big, _ = O.msm(sc, pts)
    # split: sum of two Straus halves
    a, _ = O.msm(sc[:100], pts[:100])
    b, _ = O.msm(sc[100:], pts[100:])
    assert O.point_add(a, b) == big


@pytest.mark.skipif(not os.path.exists(SODIUM), reason="libsodium not present")
def test_against_libsodium_random():
    so = ctypes.CDLL(SODIUM)
    so.sodium_init()
    rng = np.random.Generator(np.random.PCG64(11))
    for i in range(40):
        seed = rng.bytes(32)
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        so.crypto_sign_seed_keypair(pk, sk, seed)
        m = rng.bytes(int(rng.integers(0, 200)))
        sig = ctypes.create_string_buffer(64)
        so.crypto_sign_detached(sig, None, m, ctypes.c_ulonglong(len(m)), sk)
        assert O.keypair_from_seed(seed)[0] == pk.raw
        assert O.sign(sk.raw, m) == sig.raw
        s = bytearray(sig.raw)
        if i % 2:
            s[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
        ok_sod = so.crypto_sign_verify_detached(bytes(s), m, ctypes.c_ulonglong(len(m)), pk.raw) == 0
        assert (O.verify_strict(m, pk.raw, bytes(s)) == 0) == ok_sod


def test_appendix_b_header_fixture(golden):
    """primary/src/tests/common.rs:96-112 header(): author = keys().pop() (key 3), round 1,
    parents = genesis digests; id = Sha512(author||round LE||parents)[..32]
    (primary/src/messages.rs:70-84). Signed by that key (Signature::new)."""
    ks = O.keys(4)
    author_pk, author_sk = ks[3]
    # Certificate::genesis(committee) digests: Sha512(header.id(0^32) || round 0 LE || origin)
    # (messages.rs:175-187, 226-234) for every authority, ordered as a BTreeSet.
    parents = sorted(O.digest32(bytes(32) + (0).to_bytes(8, "little") + pk) for pk, _ in ks)
    hdr = author_pk + (1).to_bytes(8, "little") + b"".join(parents)
    hid = O.digest32(hdr)
    ab = golden["keys"]["appendix_b"]
    assert base64.b64encode(hid).decode() == ab["header_id_b64"]
    assert O.sign(author_sk, hid).hex() == ab["header_sig"]
    cert = O.digest32(hid + (1).to_bytes(8, "little") + author_pk)
    assert base64.b64encode(cert).decode() == ab["certificate_digest_b64"]
