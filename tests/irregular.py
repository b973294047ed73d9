"""Certificate streams over committees with IRREGULAR members (test infrastructure: built
with the oracle's group operations, never shipped).

VERDICT r04 item 2: the round-3 parity bug lived in committee keys with a torsion
component, and the differential fuzz only ever used honest committees. Here a committee of
N members holds some members whose key is

* ``mixed``     A = aB + T, T a nonzero 8-torsion point (decodes, not small order): signs
                with its scalar a, R = rB honest (residual kT), or R = rB + T' with T'
                chosen so that the residual T' + kT is zero (then dalek's verify_strict
                ACCEPTS, yet verify_batch weighs A by z k mod l and keeps a torsion term);
* ``small``     A in E[8], every encoding dalek decodes (canonical, y = p + 1 / y = p for
                the identity and the order-4 points, the sign bit on x = 0): signatures with
                R = [s]B + T', i.e. a pure torsion residual;
* ``noncanon``  y = p + t (t < 19) that decodes to a large-order point with unknown
                discrete log: random signatures;
* ``undecodable`` y off the curve: every use fails A's decompression.

Headers are authored by every kind of member and votes come from q consecutive members, so
each irregular key appears as header author and as voter at every position. Verdicts of
such certificates depend on the batch coefficients: they are compared with injected z, and
with random z against the set of verdicts the oracle produces over many coefficient sets
(``possible_verdicts``). The construction follows primary/src/messages.rs:189-215 and
crypto/src/lib.rs:200-219 (Signature::verify / verify_batch on the member keys).
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

from narwhal_amd import messages as M
from narwhal_amd.crypto import PublicKey, Signature
from oracle import oracle as O

P_FIELD = 2**255 - 19
L_ORDER = 2**252 + 27742317777372353535851937790883648493
T8 = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")
IDENTITY = bytes.fromhex("01" + "00" * 31)
KINDS = ("mixed", "small", "noncanon", "undecodable")


def _le(x: int) -> bytes:
    return (x % 2**256).to_bytes(32, "little")


def torsion_points() -> list[bytes]:
    """[j]T8 for j = 0..7 (canonical encodings; j = 0 is the identity)."""
    return [IDENTITY] + [O.scalarmult(_le(j), T8) for j in range(1, 8)]


def small_order_encodings() -> list[bytes]:
    """Every small-order encoding dalek's decompression accepts: the 8 canonical points,
    the identity as y = p + 1 (both signs: x = 0 with the sign bit decodes), y = 0 as y = p
    (order 4), and y = -1 (order 2) with the sign bit."""
    out = torsion_points()
    out += [_le(P_FIELD + 1), _le(P_FIELD + 1 + 2**255), _le(1 + 2**255),
            _le(P_FIELD), _le(P_FIELD + 2**255), _le(P_FIELD - 1 + 2**255)]
    return [e for e in dict.fromkeys(out) if O.decompress(e) is not None]


def noncanonical_large_encodings() -> list[bytes]:
    """y = p + t, t in 2..18, either sign, that decode to a point of large order."""
    out = []
    for t in range(2, 19):
        for sign in (0, 1):
            e = _le(P_FIELD + t + (sign << 255))
            if O.decompress(e) is not None and not O.is_small_order(e):
                out.append(e)
    return out


def _rand_scalar(rng) -> bytes:
    return _le(int.from_bytes(rng.bytes(32), "little") % L_ORDER)


class Member:
    """A committee member and how it signs a 32-byte message."""

    def __init__(self, kind: str, rng: np.random.Generator, honest=None):
        self.kind, self.rng = kind, rng
        tors = torsion_points()
        if kind == "honest":
            self.pk, self.sk = honest
        elif kind == "mixed":
            self.a = _rand_scalar(rng)
            self.T = tors[int(rng.integers(1, 8))]
            self.pk = O.point_add(O.scalarmult_base(self.a), self.T)
        elif kind == "small":
            encs = small_order_encodings()
            self.pk = encs[int(rng.integers(0, len(encs)))]
        elif kind == "noncanon":
            encs = noncanonical_large_encodings()
            self.pk = encs[int(rng.integers(0, len(encs)))]
        elif kind == "undecodable":
            while True:
                e = _le(int(rng.integers(2, 1 << 62)) + (int(rng.integers(0, 2)) << 255))
                if O.decompress(e) is None:
                    self.pk = e
                    break
        else:
            raise ValueError(kind)

    def sign(self, msg: bytes) -> bytes:
        rng = self.rng
        if self.kind == "honest":
            return O.sign(self.sk, msg)
        if self.kind == "mixed":
            mode = int(rng.integers(0, 3))
            if mode == 0:                                    # honest R: residual kT
                return O.sign_raw(self.a, rng.bytes(32), self.pk, msg)
            tors = torsion_points()
            for _ in range(64):                              # R = rB + T', residual T' + kT
                r = _rand_scalar(rng)
                Tp = tors[int(rng.integers(0, 8))]
                R = O.point_add(O.scalarmult_base(r), Tp)
                k = O.hram(R, self.pk, msg)
                s = O.scalar_add(r, O.scalar_mul(k, self.a))
                kT = O.scalarmult(k, self.T)
                zero = O.point_add(Tp, kT) == IDENTITY
                if mode == 1 or zero:                        # mode 2: strict-valid ones
                    return R + s
            return R + s
        if self.kind == "small":                             # R = [s]B + T'
            s = _rand_scalar(rng)
            Tp = torsion_points()[int(rng.integers(0, 8))]
            return O.point_add(O.scalarmult_base(s), Tp) + s
        # noncanon / undecodable: no discrete log; a random well-formed signature
        return O.scalarmult_base(_rand_scalar(rng)) + _rand_scalar(rng)


def committee_members(N: int, rng: np.random.Generator, n_irregular: int | None = None,
                      kinds=KINDS) -> list[Member]:
    """N members, ``n_irregular`` of them (default 1..min(4, N - 1)) of random irregular
    kinds, the rest the reference's keys() fixture stream; in committee (pk) order."""
    if n_irregular is None:
        n_irregular = int(rng.integers(1, min(4, N - 1) + 1))
    honest = O.keys(N)
    out = [Member("honest", rng, honest[i]) for i in range(N - n_irregular)]
    seen = {m.pk for m in out}
    while len(out) < N:
        m = Member(kinds[int(rng.integers(0, len(kinds)))], rng)
        if m.pk not in seen:
            seen.add(m.pk)
            out.append(m)
    return sorted(out, key=lambda m: m.pk)


def irregular_stream(N: int, n: int, seed: int, n_irregular: int | None = None,
                     kinds=KINDS) -> tuple[dict, dict, list[str]]:
    """(packed committee, packed certificate stream, member kinds in committee order):
    n certificates, author = member i mod N (shifted per round so that every member
    authors), votes by q = quorum(N) consecutive members from the author (some rotated so
    that an irregular vote sits at every index), all over the real Certificate::digest."""
    rng = np.random.Generator(np.random.PCG64([seed, N, 51]))
    members = committee_members(N, rng, n_irregular, kinds)
    com = M.Committee({PublicKey(m.pk): M.Authority(1) for m in members})
    q = com.quorum_threshold()
    d32 = lambda b: hashlib.sha512(b).digest()[:32]
    certs = []
    for i in range(n):
        ai = (i + i // N) % N
        author = members[ai]
        parents = {M.Digest(rng.bytes(32)) for _ in range(int(rng.integers(0, 3)))}
        h = M.Header(author=PublicKey(author.pk), round=1 + i // N, parents=parents)
        h.id = M.Digest(d32(h.digest_bytes()))
        h.signature = Signature.from_bytes(author.sign(h.id.value))
        c = M.Certificate(h)
        cd = d32(h.id.value + struct.pack("<Q", h.round) + author.pk)
        voters = [members[(ai + j) % N] for j in range(q)]
        votes = [(PublicKey(v.pk), Signature.from_bytes(v.sign(cd))) for v in voters]
        r = int(rng.integers(0, q))
        c.votes = votes[r:] + votes[:r]
        certs.append(c)
    return com.packed(), M.pack_certificates(certs), [m.kind for m in members]


def possible_verdicts(committee: dict, p: dict, sets: int, seed: int) -> list[set]:
    """Per certificate, the (status, index) pairs the oracle gives over ``sets`` random
    coefficient sets: what a random-z run may return. A certificate whose verdict depends on
    z has Ok with probability >= 1/8, so 64 sets miss it with probability < 2e-4."""
    rng = np.random.Generator(np.random.PCG64([seed, 97]))
    nv = len(p["vote_pks"])
    out = [set() for _ in range(len(p["header_offsets"]) - 1)]
    for _ in range(sets):
        z16 = rng.integers(0, 256, size=(nv, 16), dtype=np.uint8)
        st, ix = O.certificates_verify_many(committee, p, z16)
        for i, (a, b) in enumerate(zip(st, ix)):
            out[i].add((int(a), int(b)))
    return out


def one_certificate(p: dict, i: int) -> dict:
    """Certificate i of packed stream p as a one-certificate stream (same layout)."""
    ho, vo = p["header_offsets"], p["vote_offsets"]
    a, b, va, vb = int(ho[i]), int(ho[i + 1]), int(vo[i]), int(vo[i + 1])
    return {"header_bytes": np.ascontiguousarray(p["header_bytes"][a:b]),
            "header_offsets": np.array([0, b - a], np.uint64),
            "payload_counts": np.ascontiguousarray(p["payload_counts"][i:i + 1]),
            "ids": np.ascontiguousarray(p["ids"][i:i + 1]),
            "header_sigs": np.ascontiguousarray(p["header_sigs"][i:i + 1]),
            "vote_offsets": np.array([0, vb - va], np.uint64),
            "vote_pks": np.ascontiguousarray(p["vote_pks"][va:vb]),
            "vote_sigs": np.ascontiguousarray(p["vote_sigs"][va:vb])}


def verdict_possible(committee: dict, p: dict, i: int, verdict: tuple, seed: int,
                     sets: int = 4096) -> bool:
    """Whether the oracle gives ``verdict`` for certificate i under some of ``sets`` further
    random coefficient sets (certificate i alone). ``possible_verdicts``' 64 sets miss a
    z-dependent verdict of probability 1/8 with probability 1.9e-4 per certificate, i.e.
    about twice in a 1,000-seed campaign (10^4 z-dependent certificates); a run's verdict
    outside those 64 sets is a mismatch only if this wider search does not find it either."""
    q = one_certificate(p, i)
    nv = len(q["vote_pks"])
    rng = np.random.Generator(np.random.PCG64([seed, i, 131]))
    want = (int(verdict[0]), int(verdict[1]))
    for _ in range(sets):
        z16 = rng.integers(0, 256, size=(max(nv, 1), 16), dtype=np.uint8)
        st, ix = O.certificates_verify_many(committee, q, z16)
        if (int(st[0]), int(ix[0])) == want:
            return True
    return False
