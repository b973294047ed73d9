"""CPU checks of tests/irregular.py's constructions (the irregular committee members the GPU
fuzz uses): each kind behaves under the oracle's verify_strict / verify_batch as its
docstring says, and a stream over such a committee has coefficient-dependent verdicts."""
import hashlib

import numpy as np

from oracle import oracle as O

import irregular as I


def test_small_order_encodings_decode_and_are_small():
    encs = I.small_order_encodings()
    assert len(encs) >= 12
    for e in encs:
        assert O.decompress(e) is not None and O.is_small_order(e) == 1
    for e in I.noncanonical_large_encodings():
        assert int.from_bytes(e, "little") % 2**255 >= I.P_FIELD
        assert O.decompress(e) is not None and O.is_small_order(e) == 0


def test_member_kinds_under_the_oracle():
    rng = np.random.Generator(np.random.PCG64(3))
    msg = hashlib.sha512(b"irregular").digest()[:32]
    seen_strict_ok_mixed = seen_batch_split = False
    for _ in range(12):
        m = I.Member("mixed", rng)
        assert O.decompress(m.pk) is not None and O.is_small_order(m.pk) == 0
        for _ in range(6):
            sig = m.sign(msg)
            st = O.verify_strict(msg, m.pk, sig)
            assert st in (0, 7)
            seen_strict_ok_mixed |= st == 0
            # a lone vote's batch verdict: depends on z whenever the residual is torsion
            outs = {O.verify_batch(msg, np.frombuffer(m.pk, np.uint8),
                                   np.frombuffer(sig, np.uint8),
                                   rng.integers(0, 256, size=(1, 16), dtype=np.uint8))[0]
                    for _ in range(24)}
            seen_batch_split |= outs == {0, 7}
    assert seen_strict_ok_mixed and seen_batch_split
    s = I.Member("small", rng)
    assert O.verify_strict(msg, s.pk, s.sign(msg)) in (5, 6)
    u = I.Member("undecodable", rng)
    assert O.verify_strict(msg, u.pk, u.sign(msg)) == 3
    nc = I.Member("noncanon", rng)
    assert O.verify_strict(msg, nc.pk, nc.sign(msg)) == 7


def test_irregular_stream_has_coefficient_dependent_certificates():
    com, p, kinds = I.irregular_stream(7, 60, seed=5, n_irregular=3, kinds=("mixed", "small"))
    assert sum(k != "honest" for k in kinds) == 3
    poss = I.possible_verdicts(com, p, 16, seed=1)
    assert any(len(v) > 1 for v in poss)           # z decides some certificates
    st, ix = O.certificates_verify_many(com, p, headers_only=True)
    assert {int(x) for x in st} >= {0, 32 + 5}     # small-order authors fail the header
    com, p, _ = I.irregular_stream(10, 60, seed=6, n_irregular=1, kinds=("mixed",))
    poss = I.possible_verdicts(com, p, 16, seed=2)
    assert any(v == {(0, 0)} for v in poss)        # votes without the mixed key: always Ok
    assert any(v == {(0, 0), (48 + 7, 7)} for v in poss)


def test_one_certificate_slice_and_widened_search():
    com, p, _ = I.irregular_stream(7, 30, seed=8, n_irregular=2, kinds=("mixed",))
    rng = np.random.Generator(np.random.PCG64(4))
    z16 = rng.integers(0, 256, size=(len(p["vote_pks"]), 16), dtype=np.uint8)
    st, ix = O.certificates_verify_many(com, p, z16)
    vo = p["vote_offsets"]
    for i in range(len(st)):
        q = I.one_certificate(p, i)
        s1, x1 = O.certificates_verify_many(com, q, z16[int(vo[i]):int(vo[i + 1])])
        assert (int(s1[0]), int(x1[0])) == (int(st[i]), int(ix[i]))
    poss = I.possible_verdicts(com, p, 16, seed=3)
    split = [i for i, v in enumerate(poss) if len(v) > 1]
    assert split
    for i in split[:3]:
        for v in poss[i]:
            assert I.verdict_possible(com, p, i, v, seed=9, sets=512)
    # a verdict no coefficient set gives
    assert not I.verdict_possible(com, p, split[0], (48 + 4, 0), seed=9, sets=64)
