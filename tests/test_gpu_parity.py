"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle and the
golden fixtures. Bit-exact: digests, per-item status codes (not only verdicts), bitmaps,
batch status + failing index with injected z."""
import hashlib

import numpy as np
import pytest

from narwhal_amd import _lib
from narwhal_amd import crypto as C
from narwhal_amd import workloads as W
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _arr(hexes, width):
    if not hexes:
        return np.zeros((0, width), np.uint8)
    return np.array([np.frombuffer(bytes.fromhex(h), np.uint8) for h in hexes]).reshape(-1, width)


# ---------------------------------------------------------------- SHA-512 digests
def test_sha512_golden(golden):
    vecs = golden["sha512"]["vectors"]
    msgs = [bytes.fromhex(v["msg"]) for v in vecs]
    data = np.frombuffer(b"".join(msgs) or b"\0", np.uint8)
    lens = np.array([len(m) for m in msgs], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    out = C.sha512_digest32_many(data, offs, lens)
    for v, o in zip(vecs, out):
        assert o.tobytes().hex() == v["sha512"][:64], v["name"]


def test_sha512_worker_batches(golden):
    for v in golden["sha512"]["worker_batches"]:
        m = W.worker_batch(v["batch_id"], seed=v["seed"]).tobytes()
        assert C.sha512_digest(m).value.hex() == v["sha512"][:64]


def test_sha512_ragged_unaligned():
    data, offs, lens = W.ragged_messages(3000, 900, seed=9)
    # shift every message to an odd address to exercise the realignment path
    out = C.sha512_digest32_many(data, offs, lens)
    ref = O.sha512_digest32_many(data, offs, lens)
    assert np.array_equal(out, ref)
    d2 = np.concatenate([np.zeros(3, np.uint8), data])
    out2 = C.sha512_digest32_many(d2, offs + 3, lens)
    assert np.array_equal(out2, ref)


def test_sha512_every_tail_length_and_alignment():
    """Every length 0..400 (one, two and three padding layouts per block boundary, incl.
    len % 128 in [112, 128) where the length field spills into a padding-only block) at
    each of the 4 byte alignments."""
    lens = np.arange(0, 401, dtype=np.uint64)
    rng = np.random.Generator(np.random.PCG64(5))
    for shift in range(4):
        offs = (np.concatenate([[0], np.cumsum(lens)[:-1]]) + shift).astype(np.uint64)
        data = rng.integers(0, 256, size=int(lens.sum()) + shift + 1, dtype=np.uint8)
        out = C.sha512_digest32_many(data, offs, lens)
        for i in range(len(lens)):
            m = data[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes()
            assert out[i].tobytes() == hashlib.sha512(m).digest()[:32], (shift, i)


def test_sha512_reference_processor_fixture():
    """worker/src/tests/processor_tests.rs: digest == Sha512(serialized_batch)[..32]."""
    m = W.reference_serialized_batch()
    assert C.sha512_digest(m).value == hashlib.sha512(m).digest()[:32]


# ---------------------------------------------------------------- strict verify
def test_strict_edge_corpus(golden):
    items = golden["edge_corpus"]["items"]
    st, bm = C.verify_strict_many(_arr([i["msg"] for i in items], 32),
                                  _arr([i["pk"] for i in items], 32),
                                  _arr([i["sig"] for i in items], 64))
    exp = [i["status"] for i in items]
    bad = [(i["class"], int(s), e) for i, s, e in zip(items, st, exp) if s != e]
    assert not bad, bad
    bits = np.unpackbits(bm, bitorder="little")[:len(items)]
    assert list(bits) == [int(e == 0) for e in exp]


def test_strict_rfc8032_and_reference_keys(golden):
    """RFC 8032 section 7.1 keys (libsodium-pinned in tests/test_oracle.py): the GPU derives
    each RFC public key from its seed, and since Narwhal only ever signs 32-byte digests
    (crypto/src/lib.rs:185-204), each RFC message goes in as Digest(Sha512(msg)[..32]): the
    GPU signature over it equals the oracle's (RFC 8032 signing, pinned by libsodium),
    verifies, and fails for the neighbouring key."""
    vec = golden["keys"]["rfc8032"]
    seeds = np.array([np.frombuffer(bytes.fromhex(v["seed"]), np.uint8) for v in vec])
    pks = C.keypair_from_seed_many(seeds)
    assert [p.tobytes().hex() for p in pks] == [v["pk"] for v in vec]
    digs = np.array([np.frombuffer(O.digest32(bytes.fromhex(v["msg"])), np.uint8) for v in vec])
    sigs = C.sign_many(np.concatenate([seeds, pks], axis=1), digs)
    for v, d, sg in zip(vec, digs, sigs):
        sk = bytes.fromhex(v["seed"]) + bytes.fromhex(v["pk"])
        assert sg.tobytes() == O.sign(sk, d.tobytes())
    st, _ = C.verify_strict_many(digs, pks, sigs)
    assert st.tolist() == [0] * len(vec)
    st, _ = C.verify_strict_many(digs, np.roll(pks, 1, axis=0), sigs)
    assert all(x != 0 for x in st.tolist())
    ks = O.keys(4)
    d = C.Digest(O.digest32(b"Hello, world!"))
    sig = C.Signature.from_bytes(bytes.fromhex(golden["keys"]["hello_sig_key3"]))
    sig.verify(d, C.PublicKey(ks[3][0]))                      # verify_valid_signature
    with pytest.raises(C.CryptoError):                         # verify_invalid_signature
        sig.verify(C.Digest(O.digest32(b"Bad message!")), C.PublicKey(ks[3][0]))


def test_strict_random_vs_oracle():
    rng = np.random.Generator(np.random.PCG64(77))
    n = 3000
    seeds = [rng.bytes(32) for _ in range(64)]
    kps = [O.keypair_from_seed(s) for s in seeds]
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 64), np.uint8)
    for i in range(n):
        pk, sk = kps[i % 64]
        pks[i] = np.frombuffer(pk, np.uint8)
        sigs[i] = np.frombuffer(O.sign(sk, msgs[i].tobytes()), np.uint8)
    # tamper a quarter of them in random places
    for i in rng.choice(n, n // 4, replace=False):
        which = rng.integers(0, 3)
        if which == 0:
            sigs[i, rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))
        elif which == 1:
            pks[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
        else:
            msgs[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
    st, _ = C.verify_strict_many(msgs, pks, sigs)
    ref = O.verify_strict_many(msgs, pks, sigs)
    assert np.array_equal(st, ref)
    assert (ref == 0).sum() > n // 2


def test_strict_shared_digest_and_ragged_n():
    ks = O.keys(4)
    d = O.digest32(b"shared")
    for n in (1, 63, 64, 65, 257):
        pks = np.array([np.frombuffer(ks[i % 4][0], np.uint8) for i in range(n)])
        sigs = np.array([np.frombuffer(O.sign(ks[i % 4][1], d), np.uint8) for i in range(n)])
        if n > 5:
            sigs[5, 40] ^= 1
        st, bm = C.verify_strict_many(np.frombuffer(d, np.uint8), pks, sigs, shared_digest=True)
        exp = np.zeros(n, np.int32)
        if n > 5:
            exp[5] = 7
        assert np.array_equal(st, exp)
        assert np.array_equal(np.unpackbits(bm, bitorder="little")[:n], (exp == 0).astype(np.uint8))


# ---------------------------------------------------------------- batch verify
def test_batch_golden_injected_z(golden):
    for b in golden["batches"]["batches"]:
        n = len(b["pks"])
        votes = [(C.PublicKey(bytes.fromhex(p)), C.Signature.from_bytes(bytes.fromhex(s)))
                 for p, s in zip(b["pks"], b["sigs"])]
        z = bytes.fromhex(b["z"]) if n else None
        if b["status"] == 0:
            C.Signature.verify_batch(C.Digest(bytes.fromhex(b["digest"])), votes, z16=z)
        else:
            with pytest.raises(C.CryptoError) as ei:
                C.Signature.verify_batch(C.Digest(bytes.fromhex(b["digest"])), votes, z16=z)
            assert (ei.value.code, ei.value.index) == (b["status"], b["index"]), b["name"]


def test_batch_random_z_deterministic_set(golden):
    for b in golden["batches"]["batches"]:
        if b["name"].startswith("torsion_residual"):
            continue
        votes = [(C.PublicKey(bytes.fromhex(p)), C.Signature.from_bytes(bytes.fromhex(s)))
                 for p, s in zip(b["pks"], b["sigs"])]
        try:
            C.Signature.verify_batch(C.Digest(bytes.fromhex(b["digest"])), votes)
            got = 0
        except C.CryptoError as e:
            got = e.code
        assert got == b["status"], b["name"]


def test_reference_crypto_tests():
    """crypto/src/tests/crypto_tests.rs:79-115 verify_valid_batch / verify_invalid_batch."""
    d = C.Digest(O.digest32(b"Hello, world!"))
    ks = O.keys(4)
    keys = list(ks)
    votes = []
    for _ in range(3):
        pk, sk = keys.pop()
        votes.append((C.PublicKey(pk), C.Signature.from_bytes(O.sign(sk, d.value))))
    C.Signature.verify_batch(d, votes)
    keys = list(ks)
    votes = []
    for _ in range(2):
        pk, sk = keys.pop()
        votes.append((C.PublicKey(pk), C.Signature.from_bytes(O.sign(sk, d.value))))
    pk, _ = keys.pop()
    votes.append((C.PublicKey(pk), C.Signature()))
    with pytest.raises(C.CryptoError):
        C.Signature.verify_batch(d, votes)
    C.Signature.verify_batch(d, [])                      # empty -> Ok


def test_batch_many_vs_oracle():
    rng = np.random.Generator(np.random.PCG64(5))
    kps = [O.keypair_from_seed(rng.bytes(32)) for _ in range(100)]
    sizes = [0, 1, 3, 7, 34, 67, 3, 300, 5]
    nb = len(sizes)
    offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    digests = rng.integers(0, 256, size=(nb, 32), dtype=np.uint8)
    pks, sigs = [], []
    for b, s in enumerate(sizes):
        for j in range(s):
            pk, sk = kps[j % 100]
            pks.append(np.frombuffer(pk, np.uint8))
            sigs.append(np.frombuffer(O.sign(sk, digests[b].tobytes()), np.uint8))
    pks = np.array(pks)
    sigs = np.array(sigs)
    sigs[int(offsets[3]) + 2, 33] ^= 4        # batch 3: bad s
    pks[int(offsets[5]) + 10, 3] ^= 1         # batch 5: bad key
    z = rng.integers(0, 256, size=(len(pks), 16), dtype=np.uint8)
    st = C.verify_batch_many(digests, pks, sigs, offsets, z16=z)
    ref = O.verify_batch_many(digests, pks, sigs, offsets, z16=z)
    assert np.array_equal(st, ref)
    assert st[3] != 0 and st[5] != 0 and st[0] == 0 and st[7] == 0


# ---------------------------------------------------------------- keygen / signing
def test_keygen_and_sign_vs_oracle(golden):
    seeds = O.stdrng_seeds(300)
    pks = C.keypair_from_seed_many(np.array([np.frombuffer(s, np.uint8) for s in seeds]))
    for s, pk in zip(seeds, pks):
        assert pk.tobytes() == O.keypair_from_seed(s)[0]
    assert [p.tobytes().hex() for p in pks[:4]] == [k["pk"] for k in golden["keys"]["stdrng_zero_seed_keys"]]
    rng = np.random.Generator(np.random.PCG64(8))
    digests = rng.integers(0, 256, size=(300, 32), dtype=np.uint8)
    sks = np.concatenate([np.array([np.frombuffer(s, np.uint8) for s in seeds]), pks], axis=1)
    sigs = C.sign_many(sks, digests)
    for i in range(300):
        assert sigs[i].tobytes() == O.sign(sks[i].tobytes(), digests[i].tobytes())
    # reference fixture: keys().pop() signs the "Hello, world!" digest
    pk, sk = C.generate_keypair(lambda n: O.stdrng_seeds(4)[3])
    d = C.Digest(O.digest32(b"Hello, world!"))
    sig = C.Signature.new(d, sk)
    assert sig.flatten().hex() == golden["keys"]["hello_sig_key3"]
    sig.verify(d, pk)


@pytest.mark.gpu
def test_prepare_then_strict():
    """nw_prepare builds the lazily built strict tables now (also under NW_ALL_DEVICES);
    verification afterwards is unchanged."""
    L = _lib.lib()
    assert L.nw_prepare() == 0, L.nw_last_error()
    assert L.nw_set_device(-1) == 0
    try:
        assert L.nw_prepare() == 0, L.nw_last_error()
    finally:
        assert L.nw_set_device(0) == 0
    ks = O.keys(2)
    d = O.digest32(b"prepare")
    pks = np.array([np.frombuffer(ks[i % 2][0], np.uint8) for i in range(4)])
    sigs = np.array([np.frombuffer(O.sign(ks[i % 2][1], d), np.uint8) for i in range(4)])
    sigs[1, 40] ^= 4
    st, _ = C.verify_strict_many(np.frombuffer(d, np.uint8), pks, sigs, shared_digest=True)
    ref = O.verify_strict_many(np.frombuffer(d, np.uint8), pks, sigs, shared_msg=True)
    assert np.array_equal(st, ref)
