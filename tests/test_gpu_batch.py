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


def _corpus(nb, seed, max_n=40, empty=True):
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = rng.integers(0 if empty else 1, max_n + 1, size=nb)
    sizes[0] = 0 if empty else sizes[0]
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
    # mutate ~1 in 4 non-empty batches, one vote each, with every failure class
    for b in np.nonzero(sizes)[0][::4]:
        i = int(off[b] + rng.integers(0, sizes[b]))
        c = int(rng.integers(0, 6))
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
    z16 = rng.integers(0, 256, size=(max(n, 1), 16), dtype=np.uint8)
    return dig, pk, sigs, off, z16


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
