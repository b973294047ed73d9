"""GPU parity for crypto::Signature::verify_batch over many batches (nw_batch.hip) against
the oracle, with injected coefficients, across the launch plans: one vote per chunk, whole
batches per chunk, balanced multi-chunk batches, and several workspace slices
(NW_BATCH_CHUNK / NW_BATCH_SLICE_UNITS test hooks). Status AND failing index bit-exact."""
import numpy as np
import pytest

from narwhal_amd import crypto as C
from oracle import oracle as O

pytestmark = pytest.mark.gpu
L_ORDER = 2**252 + 27742317777372353535851937790883648493


def _mutate(sigs, pk, i, c):
    """One vote broken in failure class c (0..5)."""
    if c == 0:
        sigs[i, 40] ^= 1                        # equation
    elif c == 1:
        sigs[i, 63] |= 0x20                     # s high bits
    elif c == 2:
        v = int.from_bytes(sigs[i, 32:].tobytes(), "little") + L_ORDER
        sigs[i, 32:] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)   # s >= l
    elif c == 3:
        sigs[i, :32] = np.frombuffer((2).to_bytes(32, "little"), np.uint8)  # R off-curve
    elif c == 4:
        pk[i] = np.frombuffer((7).to_bytes(32, "little"), np.uint8)         # A off-curve
    else:
        sigs[i, :32] = 0                        # R = small-order point (y = 0)


def _corpus_sizes(sizes, rng, every=4):
    nb = len(sizes)
    off = np.zeros(nb + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    n = int(off[-1])
    seeds = rng.integers(0, 256, size=(64, 32), dtype=np.uint8)
    pks = C.keypair_from_seed_many(seeds)
    key = rng.integers(0, 64, size=n)
    sks = np.concatenate([seeds, pks], axis=1)[key]
    dig = rng.integers(0, 256, size=(nb, 32), dtype=np.uint8)
    bidx = np.repeat(np.arange(nb), sizes)
    sigs = C.sign_many(sks, dig[bidx])
    pk = pks[key].copy()
    # mutate 1 in `every` non-empty batches (none for every=0), one vote each, with every
    # failure class
    for b in (np.nonzero(sizes)[0][::every] if every else []):
        i = int(off[b] + rng.integers(0, sizes[b]))
        _mutate(sigs, pk, i, int(rng.integers(0, 6)))
    z16 = rng.integers(0, 256, size=(max(n, 1), 16), dtype=np.uint8)
    return dig, pk, sigs, off, z16


def _corpus(nb, seed, max_n=40, empty=True):
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = rng.integers(0 if empty else 1, max_n + 1, size=nb)
    sizes[0] = 0 if empty else sizes[0]
    return _corpus_sizes(sizes, rng)


@pytest.mark.parametrize("chunk,slice_units", [("1", ""), ("4", ""), ("128", ""), ("3", "97")])
def test_batch_plans_vs_oracle(monkeypatch, chunk, slice_units):
    monkeypatch.setenv("NW_BATCH_CHUNK", chunk)
    monkeypatch.setenv("NW_BATCH_SLICE_UNITS", slice_units)
    dig, pk, sigs, off, z16 = _corpus(300, seed=int(chunk) * 7 + len(slice_units))
    st = C.verify_batch_many(dig, pk, sigs, off, z16)
    ref = O.verify_batch_many(dig, pk, sigs, off, z16)
    assert np.array_equal(st, ref), np.nonzero(st != ref)
    assert (st != 0).any() and (st == 0).any()


def test_batch_fail_index_vs_oracle(monkeypatch):
    monkeypatch.setenv("NW_BATCH_CHUNK", "2")
    dig, pk, sigs, off, z16 = _corpus(40, seed=3, empty=False)
    for b in range(40):
        a, e = int(off[b]), int(off[b + 1])
        d = C.Digest(dig[b].tobytes())
        votes = [(C.PublicKey(pk[i].tobytes()), C.Signature.from_bytes(sigs[i].tobytes()))
                 for i in range(a, e)]
        ost, oidx = O.verify_batch(dig[b].tobytes(), pk[a:e], sigs[a:e], z16[a:e])
        try:
            C.Signature.verify_batch(d, votes, z16=z16[a:e].tobytes())
            got = (0, None)
        except C.CryptoError as err:
            got = (err.code, err.index)
        assert got[0] == ost, b
        if ost:
            assert got[1] == oidx, b


@pytest.mark.parametrize("chunk", ["", "64"])
def test_large_uniform_batches(monkeypatch, chunk):
    """The bench's config-2 shape (uniform batches): default plan and chunk = batch."""
    monkeypatch.setenv("NW_BATCH_CHUNK", chunk)
    nb, q = 9000, 30
    rng = np.random.Generator(np.random.PCG64(5))
    seeds = rng.integers(0, 256, size=(q, 32), dtype=np.uint8)
    pks = C.keypair_from_seed_many(seeds)
    sks = np.concatenate([seeds, pks], axis=1)
    dig = rng.integers(0, 256, size=(nb, 32), dtype=np.uint8)
    sigs = C.sign_many(np.tile(sks, (nb, 1)), np.repeat(dig, q, axis=0))
    pk = np.tile(pks, (nb, 1))
    bad = rng.choice(nb, 50, replace=False)
    sigs[bad * q + 7, 33] ^= 4
    off = (np.arange(nb + 1) * q).astype(np.uint64)
    st = C.verify_batch_many(dig, pk, sigs, off)
    exp = np.zeros(nb, np.int32)
    exp[bad] = 7
    assert np.array_equal(st, exp)


# ---- Pippenger path (batches of >= NW_BATCH_PIPPENGER_MIN votes) -------------------------
@pytest.mark.parametrize("slice_units", ["", "2600"])
def test_pippenger_mixed_vs_oracle(monkeypatch, slice_units):
    """Large batches (Pippenger) interleaved with small ones (Straus) in one call, every
    failure class, several slices: status and first failing index bit-exact."""
    monkeypatch.setenv("NW_BATCH_PIPPENGER_MIN", "400")
    monkeypatch.setenv("NW_BATCH_SLICE_UNITS", slice_units)
    rng = np.random.Generator(np.random.PCG64(11 + len(slice_units)))
    sizes = np.array([400, 3, 0, 1200, 17, 401, 650, 2, 399, 900, 512, 1000], np.int64)
    dig, pk, sigs, off, z16 = _corpus_sizes(sizes, rng, every=1)
    # a second failure later in some large batches: the first one must be reported
    for b in (3, 6, 9):
        i = int(off[b + 1]) - 5
        _mutate(sigs, pk, i, 3)
    st = C.verify_batch_many(dig, pk, sigs, off, z16)
    for b in range(len(sizes)):
        a, e = int(off[b]), int(off[b + 1])
        ost, oidx = O.verify_batch(dig[b].tobytes(), pk[a:e], sigs[a:e], z16[a:e])
        assert st[b] == ost, (b, st[b], ost)
        votes = [(C.PublicKey(pk[i].tobytes()), C.Signature.from_bytes(sigs[i].tobytes()))
                 for i in range(a, e)]
        try:
            C.Signature.verify_batch(C.Digest(dig[b].tobytes()), votes,
                                     z16=z16[a:e].tobytes())
            got = (0, None)
        except C.CryptoError as err:
            got = (err.code, err.index)
        assert got[0] == ost, b
        if ost:
            assert got[1] == oidx, (b, got, oidx)


def test_pippenger_valid_and_equation(monkeypatch):
    """Honest large batches are Ok with random (device ChaCha20) and with injected z; one
    bad equation anywhere is Err 7; skewed z (all equal: every vote in the same buckets)."""
    rng = np.random.Generator(np.random.PCG64(21))
    sizes = np.array([10000, 4096, 777], np.int64)
    dig, pk, sigs, off, z16 = _corpus_sizes(sizes, rng, every=0)
    assert (C.verify_batch_many(dig, pk, sigs, off) == 0).all()
    assert (C.verify_batch_many(dig, pk, sigs, off, z16) == 0).all()
    same = np.tile(z16[:1], (len(z16), 1))
    assert (C.verify_batch_many(dig, pk, sigs, off, same) == 0).all()
    sigs[int(off[1]) + 4000, 35] ^= 0x10
    st = C.verify_batch_many(dig, pk, sigs, off, same)
    assert list(st) == [0, 7, 0]
    st = C.verify_batch_many(dig, pk, sigs, off)
    assert list(st) == [0, 7, 0]


def test_pippenger_config1_shape():
    """Config 1: 10k pairs on the reference digest, default threshold; the Err
    variant has vote 9,999 = Signature::default()."""
    rng = np.random.Generator(np.random.PCG64(31))
    dig, pk, sigs, off, _ = _corpus_sizes(np.array([10000]), rng, every=0)
    d = C.Digest(dig[0].tobytes())
    votes = [(C.PublicKey(pk[i].tobytes()), C.Signature.from_bytes(sigs[i].tobytes()))
             for i in range(10000)]
    C.Signature.verify_batch(d, votes)
    votes[9999] = (votes[9999][0], C.Signature.from_bytes(bytes(64)))
    with pytest.raises(C.CryptoError) as e:
        C.Signature.verify_batch(d, votes)
    ost, oidx = O.verify_batch(dig[0].tobytes(), pk, np.concatenate(
        [sigs[:9999], np.zeros((1, 64), np.uint8)]), rng.integers(0, 256, (10000, 16), dtype=np.uint8))
    assert (e.value.code, e.value.index) == (ost, oidx)


@pytest.mark.parametrize("n,cls,skew", [(2925, None, False), (3000, 0, False), (4096, 3, True),
                                        (10000, 0, False), (10000, None, True), (10000, 5, False),
                                        (12288, 4, False), (16384, 2, False), (16385, 1, False),
                                        (20000, 4, False)])
def test_pippenger_one_call_fused_tail(n, cls, skew):
    """One batch alone in a call (config 1's shape): 2,925 <= n <= 16,384 takes the fused
    head and tail (k_pip_points_sorted, k_pip_tail_fused: launches ordered inside by
    completion counters), larger n the separate kernels. Status and first failing index ==
    the oracle's, with injected z, every failure class, and skewed z (all equal: every vote
    in the same buckets)."""
    rng = np.random.Generator(np.random.PCG64(n + 7 * (cls or 0) + skew))
    dig, pk, sigs, off, z16 = _corpus_sizes(np.array([n]), rng, every=0)
    if skew:
        z16 = np.tile(z16[:1], (n, 1))
    if cls is not None:
        _mutate(sigs, pk, int(rng.integers(0, n)), cls)
    ost, oidx = O.verify_batch(dig[0].tobytes(), pk, sigs, z16)
    votes = [(C.PublicKey(pk[i].tobytes()), C.Signature.from_bytes(sigs[i].tobytes()))
             for i in range(n)]
    try:
        C.Signature.verify_batch(C.Digest(dig[0].tobytes()), votes, z16=z16.tobytes())
        got = (0, None)
    except C.CryptoError as err:
        got = (err.code, err.index)
    assert got[0] == ost
    if ost:
        assert got[1] == oidx
    assert (ost == 0) == (cls is None)


def test_pippenger_one_call_fused_concurrent():
    """Four threads, each verifying its own lone large batch at once (four fused launches
    side by side on their jobs' streams, each ordered by its own counters): every verdict and
    first failing index == the oracle's."""
    import threading
    rng = np.random.Generator(np.random.PCG64(77))
    cases = []
    for k in range(4):
        n = 4000 + 1500 * k
        dig, pk, sigs, off, z16 = _corpus_sizes(np.array([n]), rng, every=0)
        if k % 2:
            _mutate(sigs, pk, int(rng.integers(0, n)), int(rng.integers(0, 6)))
        cases.append((dig, pk, sigs, z16, O.verify_batch(dig[0].tobytes(), pk, sigs, z16)))
    got = [None] * len(cases)

    def run(k):
        dig, pk, sigs, z16, _ = cases[k]
        votes = [(C.PublicKey(pk[i].tobytes()), C.Signature.from_bytes(sigs[i].tobytes()))
                 for i in range(len(pk))]
        out = []
        for _ in range(5):
            try:
                C.Signature.verify_batch(C.Digest(dig[0].tobytes()), votes, z16=z16.tobytes())
                out.append((0, None))
            except C.CryptoError as err:
                out.append((err.code, err.index))
        got[k] = out

    th = [threading.Thread(target=run, args=(k,)) for k in range(len(cases))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for k, (_, _, _, _, (ost, oidx)) in enumerate(cases):
        for code, idx in got[k]:
            assert code == ost, (k, code, ost)
            if ost:
                assert idx == oidx, (k, idx, oidx)
