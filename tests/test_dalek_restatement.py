"""The timed CPU baseline (oracle/nw_dalek.c, the dalek-equivalent restatement bench.py's
cpu_baseline legs run) gives the checker's verdicts bit for bit (VERDICT r05 next-round
item 2): the golden edge corpus and batches, a 10k random strict set, batches on both sides
of every Straus / Pippenger window threshold with z-dependent torsion residuals, and the
certificate streams of the message tests, all with injected z.

Both engines are test infrastructure (oracle/); neither is the product.
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests import cert_cases as CC
from tests import irregular as IR


def _arr(hexes, width):
    return np.array([np.frombuffer(bytes.fromhex(h), np.uint8) for h in hexes]).reshape(-1, width)


def test_edge_corpus(golden):
    items = golden["edge_corpus"]["items"]
    for it in items:
        st = O.verify_strict(bytes.fromhex(it["msg"]), bytes.fromhex(it["pk"]),
                             bytes.fromhex(it["sig"]), engine="dalek")
        assert st == it["status"], it["class"]
    st = O.verify_strict_many(_arr([i["msg"] for i in items], 32), _arr([i["pk"] for i in items], 32),
                              _arr([i["sig"] for i in items], 64), nthreads=4, engine="dalek")
    assert list(st) == [i["status"] for i in items]


def test_golden_batches(golden):
    for b in golden["batches"]["batches"]:
        n = len(b["pks"])
        pks, sigs = _arr(b["pks"], 32).reshape(n, 32), _arr(b["sigs"], 64).reshape(n, 64)
        z = np.frombuffer(bytes.fromhex(b["z"]), np.uint8).reshape(n, 16) if n else None
        got = O.verify_batch(bytes.fromhex(b["digest"]), pks, sigs, z, engine="dalek")
        assert got == (b["status"], b["index"]), b["name"]
        if not b["name"].startswith("torsion_residual"):   # verdict independent of z
            st, _ = O.verify_batch(bytes.fromhex(b["digest"]), pks, sigs, None, engine="dalek")
            assert st == b["status"], b["name"]


def _random_strict_set(n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    keys = [O.keypair_from_seed(rng.bytes(32)) for _ in range(64)]
    msgs = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    pks = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 64), np.uint8)
    for i in range(n):
        pk, sk = keys[i % len(keys)]
        pks[i] = np.frombuffer(pk, np.uint8)
        sigs[i] = np.frombuffer(O.sign(sk, msgs[i].tobytes()), np.uint8)
    bad = rng.random(n) < 0.2
    for i in np.nonzero(bad)[0]:
        j = int(rng.integers(0, 3))
        if j == 0:
            sigs[i, int(rng.integers(0, 64))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif j == 1:
            pks[i, int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        else:
            msgs[i, int(rng.integers(0, 32))] ^= np.uint8(1)
    return msgs, pks, sigs


@pytest.mark.slow
def test_random_strict_10k():
    msgs, pks, sigs = _random_strict_set(10_000, 7)
    want = O.verify_strict_many(msgs, pks, sigs, nthreads=8)
    got = O.verify_strict_many(msgs, pks, sigs, nthreads=8, engine="dalek")
    assert np.array_equal(got, want)
    assert (want == 0).sum() > 7_000 and len(set(want.tolist())) >= 4


def test_double_base_vs_checker():
    """[a]A + [b]B by the NAF-5 / affine NAF-8 chain equals the checker's point arithmetic,
    for a up to 2^255 (above l; dalek's NAF takes scalars below 2^255, and k < l) and
    b < 2^253 (s < l), and small or zero scalars."""
    rng = np.random.Generator(np.random.PCG64(3))
    for t in range(40):
        A = O.scalarmult_base(rng.bytes(32))
        a = rng.bytes(31) + bytes([int(rng.integers(0, 128))]) if t % 4 else bytes([t]) + bytes(31)
        b = rng.bytes(31) + bytes([int(rng.integers(0, 32))]) if t % 5 else bytes(32)
        want = O.point_add(O.scalarmult(a, A), O.scalarmult_base(b))
        assert O.double_base(a, A, b) == want, t


def _irregular_batch(n, seed, bad=0):
    """n votes over one digest by mixed-order / honest members (z-dependent residuals) and
    ``bad`` random damaged signatures."""
    rng = np.random.Generator(np.random.PCG64([seed, n]))
    members = IR.committee_members(8, rng, n_irregular=3, kinds=("mixed",))
    digest = rng.bytes(32)
    pks = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 64), np.uint8)
    for i in range(n):
        m = members[i % len(members)]
        pks[i] = np.frombuffer(m.pk, np.uint8)
        sigs[i] = np.frombuffer(m.sign(digest), np.uint8)
    for i in rng.choice(n, size=bad, replace=False):
        sigs[i, int(rng.integers(0, 32))] ^= np.uint8(4)
    z = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    return digest, pks, sigs, z


@pytest.mark.slow
@pytest.mark.parametrize("n", [1, 2, 94, 95, 249, 250, 399, 400])
def test_batches_at_msm_thresholds(n):
    """2n + 1 points: 189 / 191 straddle Straus -> Pippenger, 499 / 501 and 799 / 801 the
    window widths 6 -> 7 -> 8. Injected z, torsion residuals (the verdict depends on z),
    damaged votes: (status, index) equal the checker's."""
    verdicts = set()
    for seed in range(3):
        digest, pks, sigs, z = _irregular_batch(n, seed, bad=seed % 2)
        want = O.verify_batch(digest, pks, sigs, z)
        got = O.verify_batch(digest, pks, sigs, z, engine="dalek")
        assert got == want, (n, seed)
        verdicts.add(want[0])
    assert verdicts


def test_batch_many_threads():
    rng = np.random.Generator(np.random.PCG64(9))
    batches = [_irregular_batch(int(k), 100 + i) for i, k in enumerate(rng.integers(0, 40, 12))]
    dg = np.stack([np.frombuffer(b[0], np.uint8) for b in batches])
    pks = np.concatenate([b[1] for b in batches])
    sigs = np.concatenate([b[2] for b in batches])
    z = np.concatenate([b[3] for b in batches])
    off = np.cumsum([0] + [len(b[1]) for b in batches]).astype(np.uint64)
    want = O.verify_batch_many(dg, pks, sigs, off, z, nthreads=4)
    got = O.verify_batch_many(dg, pks, sigs, off, z, nthreads=4, engine="dalek")
    assert np.array_equal(got, want)


def test_certificates_mutated_stream():
    com, p, exp_st, exp_ix, _ = CC.mutated_stream(N=4, copies=1)
    z = np.random.Generator(np.random.PCG64(1)).integers(0, 256, size=(max(len(p["vote_pks"]), 1), 16),
                                                           dtype=np.uint8)
    st, ix = O.certificates_verify_many(com, p, z, engine="dalek")
    assert list(st) == list(exp_st) and list(ix) == list(exp_ix)


@pytest.mark.parametrize("N", [4, 10])
def test_certificates_irregular(N):
    com, p, _ = IR.irregular_stream(N, 24, seed=N)
    z = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(len(p["vote_pks"]), 16),
                                                           dtype=np.uint8)
    want = O.certificates_verify_many(com, p, z)
    got = O.certificates_verify_many(com, p, z, engine="dalek")
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    hw = O.certificates_verify_many(com, p, None, headers_only=True)
    hg = O.certificates_verify_many(com, p, None, headers_only=True, engine="dalek")
    assert np.array_equal(hw[0], hg[0])
