"""Seeded differential fuzz of Certificate::verify / Header::verify: honest certificates with
random byte-level damage — single-byte xors anywhere in the header bytes, id, header
signature, vote keys and vote signatures; R or A replaced by encodings the construction
never makes (small-order points, y >= p, the sign bit on x = 0, off-curve y); s pushed to
s + l or given high bits; votes duplicated, dropped or reordered — so that the checks meet
inputs no hand-written class reaches. Every status and index from the GPU (the one-launch
small-job kernel, the bulk pipeline, and the native aggregation service) must equal the
oracle's, with injected batch coefficients where the verdict depends on them.

Parity here is against the oracle (oracle/nw_oracle.c, pinned by tests/test_oracle.py);
for the encodings no reference fixture holds (y >= p with a large-order point, x = 0 with
the sign bit), the oracle's restatement of curve25519-dalek's decompression is the anchor
(DESIGN.md section 2)."""
import numpy as np
import pytest

from narwhal_amd import _lib
from narwhal_amd import messages as M
from narwhal_amd import workloads as W
from oracle import oracle as O

from cert_cases import oracle_digest_many, oracle_sign_many
from test_gpu_messages import _Com

pytestmark = pytest.mark.gpu

P_FIELD = 2**255 - 19
L_ORDER = 2**252 + 27742317777372353535851937790883648493
T8 = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")


def _odd_encodings():
    """32-byte point encodings outside what honest signing produces."""
    out = [bytes.fromhex("01" + "00" * 31),                    # identity
           (P_FIELD + 1).to_bytes(32, "little"),                # identity, y = p + 1
           bytes(31) + b"\x80",                                 # y = 0, sign bit (x^2 = -1/..)
           (1).to_bytes(32, "little")[:31] + b"\x80",           # identity with the sign bit
           (2).to_bytes(32, "little"),                          # off the curve
           (P_FIELD - 1).to_bytes(32, "little"),                # y = -1: order 2
           T8]
    for k in range(2, 8):                                       # the 8-torsion points
        out.append(O.scalarmult(k.to_bytes(32, "little"), T8))
    return [e for e in out if e is not None]


def _damage(s: dict, rng: np.random.Generator, frac: float):
    """Copy of the packed stream with about `frac` of the certificates damaged."""
    recs = []
    hb = s["header_bytes"].tobytes()
    ho, vo = s["header_offsets"], s["vote_offsets"]
    odd = _odd_encodings()
    for i in range(len(ho) - 1):
        r = {"hb": bytearray(hb[int(ho[i]):int(ho[i + 1])]), "pc": int(s["payload_counts"][i]),
             "id": bytearray(s["ids"][i].tobytes()), "sig": bytearray(s["header_sigs"][i].tobytes()),
             "vpk": [bytearray(x.tobytes()) for x in s["vote_pks"][int(vo[i]):int(vo[i + 1])]],
             "vsig": [bytearray(x.tobytes()) for x in s["vote_sigs"][int(vo[i]):int(vo[i + 1])]]}
        if rng.random() < frac:
            kind = int(rng.integers(0, 11))
            q = len(r["vpk"])
            v = int(rng.integers(0, q)) if q else 0
            if kind == 0:   # a byte of the header bytes (author, round, payload, parents)
                r["hb"][int(rng.integers(0, len(r["hb"])))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 1:
                r["id"][int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 2:
                r["sig"][int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 3 and q:
                r["vsig"][v][int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 4 and q:
                r["vpk"][v][int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 5 and q:   # R of a vote: an odd encoding
                r["vsig"][v][:32] = odd[int(rng.integers(0, len(odd)))]
            elif kind == 6:         # R of the header signature: an odd encoding
                r["sig"][:32] = odd[int(rng.integers(0, len(odd)))]
            elif kind == 7 and q:   # s + l, or high bits
                sv = int.from_bytes(bytes(r["vsig"][v][32:]), "little")
                sv = sv + L_ORDER if rng.random() < 0.5 else sv | (1 << 254)
                r["vsig"][v][32:] = (sv % 2**256).to_bytes(32, "little")
            elif kind == 8 and q > 1:   # a vote duplicated over another
                r["vpk"][v], r["vsig"][v] = bytearray(r["vpk"][v - 1]), bytearray(r["vsig"][v - 1])
            elif kind == 9 and q > 1:   # a vote dropped
                del r["vpk"][v], r["vsig"][v]
            elif kind == 10 and q > 1:  # two votes swapped (order matters for the index)
                w = int(rng.integers(0, q))
                r["vpk"][v], r["vpk"][w] = r["vpk"][w], r["vpk"][v]
                r["vsig"][v], r["vsig"][w] = r["vsig"][w], r["vsig"][v]
        recs.append(r)
    n = len(recs)
    out = {"header_bytes": np.frombuffer(b"".join(bytes(r["hb"]) for r in recs), np.uint8).copy(),
           "header_offsets": np.concatenate([[0], np.cumsum([len(r["hb"]) for r in recs])]).astype(np.uint64),
           "payload_counts": np.array([r["pc"] for r in recs], np.uint32),
           "ids": np.frombuffer(b"".join(bytes(r["id"]) for r in recs), np.uint8).reshape(n, 32).copy(),
           "header_sigs": np.frombuffer(b"".join(bytes(r["sig"]) for r in recs), np.uint8).reshape(n, 64).copy(),
           "vote_offsets": np.concatenate([[0], np.cumsum([len(r["vpk"]) for r in recs])]).astype(np.uint64)}
    out["vote_pks"] = np.frombuffer(b"".join(bytes(x) for r in recs for x in r["vpk"]) or bytes(32),
                                    np.uint8).reshape(-1, 32).copy()[:int(out["vote_offsets"][-1])]
    out["vote_sigs"] = np.frombuffer(b"".join(bytes(x) for r in recs for x in r["vsig"]) or bytes(64),
                                     np.uint8).reshape(-1, 64).copy()[:int(out["vote_offsets"][-1])]
    return out


@pytest.mark.parametrize("N,n,seed", [(4, 600, 1), (10, 300, 2), (50, 60, 3), (4, 2000, 4),
                                      (7, 700, 5), (10, 1000, 6), (20, 200, 7), (50, 120, 8)])
def test_fuzz_certificates_small_and_bulk_vs_oracle(monkeypatch, N, n, seed):
    keys = O.keys(N)
    s = W.certificate_stream(n, keys, oracle_sign_many, oracle_digest_many, payload=seed % 3,
                             seed=700 + seed)
    rng = np.random.Generator(np.random.PCG64(seed))
    d = _damage(s, rng, 0.5)
    com = _Com(s["committee"])
    z16 = rng.integers(0, 256, size=(len(d["vote_pks"]), 16), dtype=np.uint8)
    ost, oix = O.certificates_verify_many(s["committee"], d, z16)
    assert len(set(ost.tolist())) >= 5, sorted(set(ost.tolist()))   # the damage reaches many checks
    for small in ("1", "0"):
        monkeypatch.setenv("NW_SMALL", small)
        M.verify_certificates_many(com, d, z16)          # a committee's first job builds tables
        s0, p0 = _lib.path_stats()
        st, ix = M.verify_certificates_many(com, d, z16)
        s1, p1 = _lib.path_stats()
        assert (s1 > s0) if small == "1" else (s1 == s0 and p1 > p0)
        bad = [(i, int(a), int(b), int(x), int(y)) for i, (a, b, x, y)
               in enumerate(zip(st, ost, ix, oix)) if a != b or x != y]
        assert not bad, (small, bad[:10])
    # headers only, the same damage
    monkeypatch.setenv("NW_SMALL", "1")
    hst, hix = M.verify_headers_many(com, d)
    ohst, ohix = O.certificates_verify_many(s["committee"], d, headers_only=True)
    assert hst.tolist() == ohst.tolist() and hix.tolist() == ohix.tolist()


def test_fuzz_certificates_through_service_vs_oracle():
    """The same damaged certificates one by one through the native service (random CSPRNG
    coefficients there): statuses and indices == the oracle's wherever the verdict does not
    depend on the coefficients, i.e. for every certificate the oracle gives the same answer
    under two different coefficient sets."""
    import asyncio
    from narwhal_amd import service as S
    from test_service import _rows
    keys = O.keys(10)
    s = W.certificate_stream(300, keys, oracle_sign_many, oracle_digest_many, seed=777)
    rng = np.random.Generator(np.random.PCG64(9))
    d = _damage(s, rng, 0.5)
    z_a = rng.integers(0, 256, size=(len(d["vote_pks"]), 16), dtype=np.uint8)
    z_b = rng.integers(0, 256, size=(len(d["vote_pks"]), 16), dtype=np.uint8)
    oa, oia = O.certificates_verify_many(s["committee"], d, z_a)
    ob, oib = O.certificates_verify_many(s["committee"], d, z_b)
    stable = (oa == ob) & (oia == oib)
    rows = _rows(d)

    async def main():
        svc = S.NativeService(s["committee"], max_delay=0.0002, hedge=0)
        got = await asyncio.gather(*[svc.certificate_status(r) for r in rows])
        svc.close()
        return got

    got = asyncio.run(main())
    bad = [(i, got[i], (int(oa[i]), int(oia[i]))) for i in range(len(rows))
           if stable[i] and got[i] != (int(oa[i]), int(oia[i]))]
    assert not bad, bad[:10]
    assert stable.mean() > 0.9


# ---- irregular committee members ----------------------------------
# Committees holding mixed-order (aB + T), small-order (every decodable encoding),
# non-canonical large-order and undecodable keys, as header authors and as voters at every
# index (tests/irregular.py), plus the byte damage above on a quarter of the certificates.
# Injected coefficients: every (status, index) == the oracle on the small-job kernel, the
# bulk keyed pipeline and the per-certificate path. Random coefficients (the service, the
# merged-group and small-group policies): every verdict is one the oracle gives for some
# coefficient set (irregular.possible_verdicts over 64 sets, widened to 4,096 more sets for a
# verdict outside them: irregular.verdict_possible).
IRREGULAR_SHAPES = [(4, 160, 21), (7, 160, 22), (10, 120, 23), (20, 60, 24), (50, 24, 25),
                    (100, 12, 26)]
INJECTED_PATHS = ({"NW_SMALL": "1"}, {"NW_SMALL": "0"}, {"NW_SMALL": "0", "NW_CERT_MERGE": "0"})
RANDOM_PATHS = ({"NW_SMALL": "1"}, {"NW_SMALL": "0"}, {"NW_SMALL": "0", "NW_CERT_KEYED": "0"},
                {"NW_SMALL": "0", "NW_CERT_KEYED": "0", "NW_CERT_SMALL_K": "4"},
                {"NW_SMALL": "0", "NW_CERT_KEYED": "0", "NW_CERT_GROUP_VOTES": "256"})
ENV_KEYS = ("NW_SMALL", "NW_CERT_MERGE", "NW_CERT_KEYED", "NW_CERT_SMALL_K",
            "NW_CERT_GROUP_VOTES")


def _irregular_case(N, n, seed):
    import irregular as I
    com, s, kinds = I.irregular_stream(N, n, seed)
    rng = np.random.Generator(np.random.PCG64([seed, 5]))
    d = _damage(s, rng, 0.25)
    z16 = rng.integers(0, 256, size=(len(d["vote_pks"]), 16), dtype=np.uint8)
    return com, d, z16, kinds


def _set_env(monkeypatch, env):
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("N,n,seed", IRREGULAR_SHAPES)
def test_fuzz_irregular_committees_injected_vs_oracle(monkeypatch, N, n, seed):
    com, d, z16, kinds = _irregular_case(N, n, seed)
    assert any(k != "honest" for k in kinds)
    ost, oix = O.certificates_verify_many(com, d, z16)
    for env in INJECTED_PATHS:
        _set_env(monkeypatch, env)
        for rep in range(2):                              # the first call builds the tables
            st, ix = M.verify_certificates_many(_Com(com), d, z16)
            bad = [(i, int(a), int(b), int(x), int(y)) for i, (a, b, x, y)
                   in enumerate(zip(st, ost, ix, oix)) if a != b or x != y]
            assert not bad, (env, rep, kinds, bad[:10])
    ohst, ohix = O.certificates_verify_many(com, d, headers_only=True)
    for small in ("1", "0"):
        _set_env(monkeypatch, {"NW_SMALL": small})
        hst, hix = M.verify_headers_many(_Com(com), d)
        assert hst.tolist() == ohst.tolist() and hix.tolist() == ohix.tolist(), small


@pytest.mark.parametrize("N,n,seed", IRREGULAR_SHAPES[:4])
def test_fuzz_irregular_committees_random_z(monkeypatch, N, n, seed):
    import irregular as I
    com, d, _, kinds = _irregular_case(N, n, seed)
    poss = I.possible_verdicts(com, d, 64, seed)
    assert any(len(v) > 1 for v in poss)                  # z decides some certificates
    for env in RANDOM_PATHS:
        _set_env(monkeypatch, env)
        for rep in range(2):
            st, ix = M.verify_certificates_many(_Com(com), d, None)
            bad = [(i, int(a), int(x), sorted(poss[i])) for i, (a, x) in enumerate(zip(st, ix))
                   if (int(a), int(x)) not in poss[i]
                   and not I.verdict_possible(com, d, i, (a, x), seed)]
            assert not bad, (env, rep, kinds, bad[:10])


def test_fuzz_irregular_committees_through_service():
    import asyncio
    import irregular as I
    from narwhal_amd import service as S
    from test_service import _rows
    com, d, _, kinds = _irregular_case(10, 120, 31)
    poss = I.possible_verdicts(com, d, 64, 31)
    rows = _rows(d)

    async def main():
        svc = S.NativeService(com, max_delay=0.0002, hedge=0)
        got = await asyncio.gather(*[svc.certificate_status(r) for r in rows])
        got += await asyncio.gather(*[svc.certificate_status(r) for r in rows[::-1]])
        svc.close()
        return got

    got = asyncio.run(main())
    n = len(rows)
    pairs = [(i, got[i]) for i in range(n)] + [(n - 1 - j, got[n + j]) for j in range(n)]
    bad = [(i, g, sorted(poss[i])) for i, g in pairs
           if tuple(g) not in poss[i] and not I.verdict_possible(com, d, i, g, 31)]
    assert not bad, (kinds, bad[:10])


_FALLBACK_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from narwhal_amd import _lib
from narwhal_amd import messages as M
from oracle import oracle as O
from test_gpu_fuzz import _irregular_case
from test_gpu_messages import _Com
L = _lib.lib()
assert L.nw_prepare() == -4, L.nw_last_error()      # no room for the keyed tables
for N, n, seed in ((4, 80, 41), (10, 60, 42), (20, 30, 43)):
    com, d, z16, kinds = _irregular_case(N, n, seed)
    ost, oix = O.certificates_verify_many(com, d, z16)
    for _ in range(2):
        st, ix = M.verify_certificates_many(_Com(com), d, z16)
        assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist(), (N, kinds)
    hst, hix = M.verify_headers_many(_Com(com), d)
    ohst, ohix = O.certificates_verify_many(com, d, headers_only=True)
    assert hst.tolist() == ohst.tolist() and hix.tolist() == ohix.tolist(), N
small, pipe = _lib.path_stats()
assert small == 0 and pipe > 0, (small, pipe)
print("IRREGULAR_FALLBACK_OK")
"""


def test_fuzz_irregular_committees_unkeyed_fallback():
    """The same construction with no room for the keyed tables (NW_DEVICE_MEM_LIMIT, as
    tests/test_gpu_memory.py): the unkeyed strict ladder and per-certificate verify_batch."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NW_DEVICE_MEM_LIMIT=str(3 * 10**9))
    r = subprocess.run([sys.executable, "-c", f"ROOT = {root!r}\n" + _FALLBACK_CHILD], env=env,
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "IRREGULAR_FALLBACK_OK" in r.stdout, r.stderr[-3000:]


# ---- Signature::verify_batch / verify over irregular keys (Straus, Pippenger, fused) ------
# Batches whose votes come from a key pool with mixed-order, small-order, non-canonical and
# undecodable members (tests/irregular.py) among honest ones, with a sprinkle of byte damage,
# odd R encodings, s + l and high bits; sizes across the chunked-Straus path, the Pippenger
# path (n >= 512) and config 1's fused one-call launches (a lone batch of 2,925..16,384).
# Injected coefficients: every batch status == the oracle's; every item's strict status too.
def _irregular_vote_corpus(sizes, seed, bad=0.03, irr=0.08, kinds=None):
    """kinds: the irregular member kinds (default all); the decodable ones alone let large
    batches reach the random linear combination instead of failing fast on a decode."""
    import irregular as I
    from narwhal_amd import crypto as C
    rng = np.random.Generator(np.random.PCG64([seed, 77]))
    honest = [I.Member("honest", rng, kp) for kp in O.keys(48)]
    odd_kinds = [I.Member(k, rng) for k in (kinds or I.KINDS) for _ in range(3)]
    nb = len(sizes)
    off = np.zeros(nb + 1, np.uint64)
    off[1:] = np.cumsum(sizes)
    n = int(off[-1])
    dig = rng.integers(0, 256, size=(nb, 32), dtype=np.uint8)
    bidx = np.repeat(np.arange(nb), sizes)
    who = rng.integers(0, len(honest), size=n)
    irregular_item = rng.random(n) < irr
    pks = np.array([np.frombuffer(honest[w].pk, np.uint8) for w in who]).reshape(-1, 32)
    sks = np.array([np.frombuffer(honest[w].sk, np.uint8) for w in who]).reshape(-1, 64)
    sigs = C.sign_many(sks, dig[bidx]) if n else np.zeros((0, 64), np.uint8)
    odd = _odd_encodings()
    for i in np.nonzero(irregular_item)[0]:
        m = odd_kinds[int(rng.integers(0, len(odd_kinds)))]
        pks[i] = np.frombuffer(m.pk, np.uint8)
        sigs[i] = np.frombuffer(m.sign(dig[bidx[i]].tobytes()), np.uint8)
    for i in np.nonzero(rng.random(n) < bad)[0]:
        kind = int(rng.integers(0, 5 if kinds is None else 4))   # no key damage with kinds
        if kind == 0:
            sigs[i, int(rng.integers(0, 64))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif kind == 1:
            sigs[i, :32] = np.frombuffer(odd[int(rng.integers(0, len(odd)))], np.uint8)
        elif kind == 2:
            v = int.from_bytes(sigs[i, 32:].tobytes(), "little") + L_ORDER
            sigs[i, 32:] = np.frombuffer((v % 2**256).to_bytes(32, "little"), np.uint8)
        elif kind == 3:
            sigs[i, 63] |= np.uint8(0x40)
        else:
            pks[i, int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    z16 = rng.integers(0, 256, size=(max(n, 1), 16), dtype=np.uint8)
    return dig, pks, sigs, off, z16, bidx


DECODABLE = ("mixed", "small", "noncanon")


@pytest.mark.parametrize("sizes,seed,irr,bad,kinds", [
    ([0, 1, 2, 3, 5, 8, 17, 33, 67, 100, 189, 190, 300], 61, 0.08, 0.03, None),
    ([1, 2, 3, 5, 8, 17, 33, 67, 100, 189, 190, 300] * 2, 67, 0.01, 0.002, DECODABLE),
    ([511, 512, 600, 1024, 40, 7], 62, 0.003, 0.0005, DECODABLE),
    ([2000, 3, 64, 900], 63, 0.002, 0.0005, DECODABLE),
    ([3000], 64, 0.001, 0.0, DECODABLE), ([5000], 65, 0.0006, 0.0, ("mixed",)),
    ([700], 66, 0.003, 0.0, ("mixed", "small")), ([3000], 68, 0.08, 0.03, None)])
def test_fuzz_irregular_keys_verify_batch_and_strict(sizes, seed, irr, bad, kinds):
    from narwhal_amd import crypto as C
    dig, pks, sigs, off, z16, bidx = _irregular_vote_corpus(np.array(sizes), seed, bad, irr, kinds)
    ost = O.verify_batch_many(dig, pks, sigs, off, z16)
    for rep in range(2):
        st = C.verify_batch_many(dig, pks, sigs, off, z16)
        assert st.tolist() == ost.tolist(), (rep, st.tolist(), ost.tolist())
    if len(pks):
        sst, _ = C.verify_strict_many(dig[bidx], pks, sigs)
        osst = O.verify_strict_many(dig[bidx], pks, sigs)
        bad = np.nonzero(sst != osst)[0]
        assert not len(bad), [(int(i), int(sst[i]), int(osst[i])) for i in bad[:10]]
    # one batch alone through the blocking call: status AND failing index (crypto_tests.rs
    # 96-115 shape), against the oracle's verify_batch
    b = int(np.argmax(np.diff(off)))
    a, e = int(off[b]), int(off[b + 1])
    votes = [(C.PublicKey(pks[i].tobytes()), C.Signature.from_bytes(sigs[i].tobytes()))
             for i in range(a, e)]
    ost1, oix1 = O.verify_batch(dig[b].tobytes(), pks[a:e], sigs[a:e], z16[a:e])
    try:
        C.Signature.verify_batch(C.Digest(dig[b].tobytes()), votes, z16=z16[a:e].tobytes())
        got = (0, 0)
    except C.CryptoError as err:
        got = (err.code, err.index)
    assert got == (ost1, oix1 if ost1 else 0), (got, ost1, oix1)
