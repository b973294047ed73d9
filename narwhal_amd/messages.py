"""Host-side mirror of the reference's primary messages over the MI355X engine.

Reference: /root/reference/primary/src/messages.rs and config/src/lib.rs. Same names,
fields, digest layouts, check order and errors, so the reference's tests read the same:

    Committee.stake / quorum_threshold / worker       config/src/lib.rs:139-212
    Header.digest  = Sha512(author || round LE || (digest || worker_id LE)* || parents*)
                                                      messages.rs:70-84
    Header.verify(committee)                          messages.rs:48-67
    Vote.digest    = Sha512(id || round LE || origin) messages.rs:145-153
    Vote.verify(committee)                            messages.rs:131-142
    Certificate.digest = Sha512(header.id || round LE || origin)   messages.rs:226-234
    Certificate.verify(committee)                     messages.rs:189-215
    Certificate.genesis / __eq__                      messages.rs:174-187, 247-254
    DagError variants                                 primary/src/error.rs:26-59

Every digest and signature check runs in the gfx950 kernels through the C ABI
(nw_headers_verify_many, nw_votes_verify_many, nw_certificates_verify_many,
nw_sha512_digest32_many); the committee / quorum bookkeeping is checked on the device
too, in the same kernels (nw_cert.hip). The bulk helpers (verify_*_many) are the
aggregation entry points: one call verifies a whole stream of messages.
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import check
from .crypto import (CryptoError, Digest, PublicKey, SecretKey, Signature, sha512_digest,
                     sha512_digest32_many)

__all__ = ["Authority", "Committee", "ConfigError", "Header", "Vote", "Certificate",
           "DagError", "InvalidSignature", "InvalidHeaderId", "MalformedHeader",
           "UnknownAuthority", "AuthorityReuse", "CertificateRequiresQuorum",
           "pack_committee", "pack_certificates", "verify_certificates_many",
           "verify_headers_many", "verify_votes_many", "raise_for_status"]

# NW_DAG_* (include/narwhal_amd.h)
DAG_INVALID_HEADER_ID = 16
DAG_UNKNOWN_AUTHORITY = 17
DAG_MALFORMED_HEADER = 18
DAG_AUTHORITY_REUSE = 19
DAG_REQUIRES_QUORUM = 20
DAG_INVALID_SIGNATURE = 32
DAG_INVALID_VOTES = 48


# ----------------------------------------------------------------------------- errors
class DagError(Exception):
    """primary::DagError (error.rs:26-59). ``code`` = the NW_DAG_* status."""
    code = 0


class InvalidSignature(DagError):
    """DagError::InvalidSignature(CryptoError)."""

    def __init__(self, crypto: CryptoError, code: int):
        self.crypto = crypto
        self.code = code
        super().__init__(f"Invalid signature ({crypto})")


class InvalidHeaderId(DagError):
    code = DAG_INVALID_HEADER_ID

    def __init__(self):
        super().__init__("Invalid header id")


class MalformedHeader(DagError):
    code = DAG_MALFORMED_HEADER

    def __init__(self, digest: Digest):
        self.digest = digest
        super().__init__(f"Malformed header {digest}")


class UnknownAuthority(DagError):
    code = DAG_UNKNOWN_AUTHORITY

    def __init__(self, pk: PublicKey):
        self.public_key = pk
        super().__init__(f"Received message from unknown authority {pk}")


class AuthorityReuse(DagError):
    code = DAG_AUTHORITY_REUSE

    def __init__(self, pk: PublicKey):
        self.public_key = pk
        super().__init__(f"Authority {pk} appears in quorum more than once")


class CertificateRequiresQuorum(DagError):
    code = DAG_REQUIRES_QUORUM

    def __init__(self):
        super().__init__("Received certificate without a quorum")


class ConfigError(Exception):
    """config::ConfigError::NotInCommittee."""


# ----------------------------------------------------------------------------- committee
@dataclass
class Authority:
    """config::Authority (lib.rs:129-137); network addresses are not on this path, so
    ``workers`` keeps only the WorkerId keys (mapped to an opaque address value)."""
    stake: int
    workers: dict[int, object] = field(default_factory=lambda: {0: None})


class Committee:
    """config::Committee: BTreeMap<PublicKey, Authority> (iteration in key order)."""

    def __init__(self, authorities: dict[PublicKey, Authority]):
        self.authorities = dict(sorted(authorities.items()))
        self._packed = None

    def size(self) -> int:
        return len(self.authorities)

    def stake(self, name: PublicKey) -> int:
        a = self.authorities.get(name)
        return 0 if a is None else a.stake

    def quorum_threshold(self) -> int:
        total = sum(a.stake for a in self.authorities.values()) & 0xFFFFFFFF
        return ((2 * total) & 0xFFFFFFFF) // 3 + 1

    def validity_threshold(self) -> int:
        total = sum(a.stake for a in self.authorities.values()) & 0xFFFFFFFF
        return (total + 2) // 3

    def worker(self, to: PublicKey, wid: int):
        a = self.authorities.get(to)
        if a is None or wid not in a.workers:
            raise ConfigError(f"Node {to} is not in the committee")
        return a.workers[wid]

    def packed(self):
        if self._packed is None:
            self._packed = pack_committee(self)
        return self._packed


class _CCommittee(ctypes.Structure):
    _fields_ = [("nauth", ctypes.c_size_t), ("pks", ctypes.c_void_p),
                ("stakes", ctypes.c_void_p), ("worker_offsets", ctypes.c_void_p),
                ("worker_ids", ctypes.c_void_p)]


class _CCertificates(ctypes.Structure):
    _fields_ = [("n", ctypes.c_size_t), ("header_bytes", ctypes.c_void_p),
                ("header_offsets", ctypes.c_void_p), ("payload_counts", ctypes.c_void_p),
                ("ids", ctypes.c_void_p), ("header_sigs", ctypes.c_void_p),
                ("vote_offsets", ctypes.c_void_p), ("vote_pks", ctypes.c_void_p),
                ("vote_sigs", ctypes.c_void_p), ("header_bytes_len", ctypes.c_size_t),
                ("nvotes", ctypes.c_size_t), ("host_vote_offsets", ctypes.c_void_p)]


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def pack_committee(c: Committee) -> dict[str, np.ndarray]:
    """Structure-of-arrays committee (nw_committee): keys sorted by bytes."""
    names = list(c.authorities)
    pks = np.frombuffer(b"".join(n.value for n in names) or b"", np.uint8).reshape(-1, 32).copy()
    stakes = np.array([c.authorities[n].stake for n in names], np.uint32)
    wids = [sorted(c.authorities[n].workers) for n in names]
    wo = np.zeros(len(names) + 1, np.uint64)
    wo[1:] = np.cumsum([len(w) for w in wids]) if names else []
    wflat = np.array([w for ws in wids for w in ws], np.uint32)
    return {"pks": pks, "stakes": stakes, "worker_offsets": wo,
            "worker_ids": wflat if len(wflat) else np.zeros(1, np.uint32)}


def committee_struct(p: dict[str, np.ndarray]) -> _CCommittee:
    return _CCommittee(len(p["stakes"]), _p(p["pks"]), _p(p["stakes"]), _p(p["worker_offsets"]),
                       _p(p["worker_ids"]))


# ----------------------------------------------------------------------------- messages
@dataclass
class Header:
    author: PublicKey = field(default_factory=PublicKey)
    round: int = 0
    payload: dict[Digest, int] = field(default_factory=dict)
    parents: set[Digest] = field(default_factory=set)
    id: Digest = field(default_factory=Digest)
    signature: Signature = field(default_factory=Signature)

    def digest_bytes(self) -> bytes:
        """The bytes `Hash for Header` feeds the hasher (messages.rs:70-84)."""
        out = [self.author.value, struct.pack("<Q", self.round)]
        for d in sorted(self.payload):              # BTreeMap order
            out += [d.value, struct.pack("<I", self.payload[d])]
        out += [d.value for d in sorted(self.parents)]   # BTreeSet order
        return b"".join(out)

    def digest(self) -> Digest:
        return sha512_digest(self.digest_bytes())

    @classmethod
    def new(cls, author: PublicKey, round: int, payload: dict[Digest, int],
            parents: set[Digest], secret: SecretKey) -> "Header":
        """Header::new with the SignatureService replaced by the secret it wraps."""
        h = cls(author, round, dict(payload), set(parents))
        h.id = h.digest()
        h.signature = Signature.new(h.id, secret)
        return h

    def verify(self, committee: Committee) -> None:
        st, ix = verify_headers_many(committee, [self])
        raise_for_status(int(st[0]), int(ix[0]), self, None)

    def __eq__(self, other) -> bool:    # tests/common.rs:16-20
        return isinstance(other, Header) and self.id == other.id


@dataclass
class Vote:
    id: Digest
    round: int
    origin: PublicKey
    author: PublicKey
    signature: Signature = field(default_factory=Signature)

    def digest(self) -> Digest:
        return sha512_digest(self.id.value + struct.pack("<Q", self.round) + self.origin.value)

    @classmethod
    def new(cls, header: Header, author: PublicKey, secret: SecretKey) -> "Vote":
        v = cls(header.id, header.round, header.author, author)
        v.signature = Signature.new(v.digest(), secret)
        return v

    def verify(self, committee: Committee) -> None:
        st = verify_votes_many(committee, [self])
        raise_for_status(int(st[0]), 0, None, self)


@dataclass
class Certificate:
    header: Header = field(default_factory=Header)
    votes: list[tuple[PublicKey, Signature]] = field(default_factory=list)

    @staticmethod
    def genesis(committee: Committee) -> list["Certificate"]:
        return [Certificate(Header(author=name)) for name in committee.authorities]

    def round(self) -> int:
        return self.header.round

    def origin(self) -> PublicKey:
        return self.header.author

    def digest(self) -> Digest:
        return sha512_digest(self.header.id.value + struct.pack("<Q", self.round())
                             + self.origin().value)

    def verify(self, committee: Committee, z16: bytes | None = None) -> None:
        st, ix = verify_certificates_many(committee, [self],
                                          None if z16 is None else np.frombuffer(z16, np.uint8))
        raise_for_status(int(st[0]), int(ix[0]), self.header, None, self.votes)

    def __eq__(self, other) -> bool:    # messages.rs:247-254
        return (isinstance(other, Certificate) and self.header.id == other.header.id
                and self.round() == other.round() and self.origin() == other.origin())


# ----------------------------------------------------------------------------- bulk paths
def pack_certificates(items: Sequence[Certificate | Header]) -> dict[str, np.ndarray]:
    """nw_certificates SoA arrays for Certificates (or bare Headers: no votes)."""
    headers = [c.header if isinstance(c, Certificate) else c for c in items]
    hb = [h.digest_bytes() for h in headers]
    ho = np.zeros(len(hb) + 1, np.uint64)
    ho[1:] = np.cumsum([len(b) for b in hb]) if hb else []
    votes = [c.votes if isinstance(c, Certificate) else [] for c in items]
    vo = np.zeros(len(items) + 1, np.uint64)
    vo[1:] = np.cumsum([len(v) for v in votes]) if items else []
    vpk = b"".join(pk.value for vs in votes for pk, _ in vs)
    vsig = b"".join(s.flatten() for vs in votes for _, s in vs)
    return {
        "header_bytes": np.frombuffer(b"".join(hb) or b"\0", np.uint8).copy(),
        "header_offsets": ho,
        "payload_counts": np.array([len(h.payload) for h in headers], np.uint32),
        "ids": np.frombuffer(b"".join(h.id.value for h in headers) or b"\0" * 32,
                             np.uint8).reshape(-1, 32).copy(),
        "header_sigs": np.frombuffer(b"".join(h.signature.flatten() for h in headers)
                                     or b"\0" * 64, np.uint8).reshape(-1, 64).copy(),
        "vote_offsets": vo,
        "vote_pks": np.frombuffer(vpk or b"\0" * 32, np.uint8).reshape(-1, 32).copy(),
        "vote_sigs": np.frombuffer(vsig or b"\0" * 64, np.uint8).reshape(-1, 64).copy(),
    }


def certificates_struct(p: dict[str, np.ndarray], n: int) -> _CCertificates:
    return _CCertificates(n, _p(p["header_bytes"]), _p(p["header_offsets"]),
                          _p(p["payload_counts"]), _p(p["ids"]), _p(p["header_sigs"]),
                          _p(p["vote_offsets"]), _p(p["vote_pks"]), _p(p["vote_sigs"]),
                          int(p["header_offsets"][-1]), int(p["vote_offsets"][-1]), None)


def verify_certificates_many(committee: Committee, certs: Sequence[Certificate] | dict,
                             z16: np.ndarray | None = None) -> tuple[np.ndarray, np.ndarray]:
    """n x Certificate::verify on the GPU -> (status int32[n] NW_DAG_*, index uint64[n]).
    ``certs`` may be a list of Certificate or an already packed SoA dict."""
    p = certs if isinstance(certs, dict) else pack_certificates(certs)
    n = len(p["header_offsets"]) - 1
    st = np.zeros(n, np.int32)
    ix = np.zeros(n, np.uint64)
    cp = committee.packed()
    cc, cs = committee_struct(cp), certificates_struct(p, n)
    zp = None
    if z16 is not None:
        z16 = np.ascontiguousarray(z16, np.uint8)
        zp = _p(z16)
    check(_lib.lib().nw_certificates_verify_many(ctypes.byref(cc), ctypes.byref(cs), zp, _p(st),
                                                 _p(ix)), "nw_certificates_verify_many")
    return st, ix


def verify_headers_many(committee: Committee, headers: Sequence[Header] | dict
                        ) -> tuple[np.ndarray, np.ndarray]:
    """n x Header::verify on the GPU -> (status int32[n], index uint64[n])."""
    p = headers if isinstance(headers, dict) else pack_certificates(headers)
    n = len(p["header_offsets"]) - 1
    st = np.zeros(n, np.int32)
    ix = np.zeros(n, np.uint64)
    cp = committee.packed()
    cc, cs = committee_struct(cp), certificates_struct(p, n)
    check(_lib.lib().nw_headers_verify_many(ctypes.byref(cc), ctypes.byref(cs), _p(st), _p(ix)),
          "nw_headers_verify_many")
    return st, ix


def pack_votes(votes: Sequence[Vote]) -> dict[str, np.ndarray]:
    def cat(xs, w):
        return np.frombuffer(b"".join(xs) or b"\0" * w, np.uint8).reshape(-1, w).copy()
    return {"ids": cat([v.id.value for v in votes], 32),
            "rounds": np.array([v.round for v in votes] or [0], np.uint64),
            "origins": cat([v.origin.value for v in votes], 32),
            "authors": cat([v.author.value for v in votes], 32),
            "sigs": cat([v.signature.flatten() for v in votes], 64)}


def verify_votes_many(committee: Committee, votes: Sequence[Vote] | dict) -> np.ndarray:
    """n x Vote::verify on the GPU -> status int32[n]."""
    p = votes if isinstance(votes, dict) else pack_votes(votes)
    n = len(votes) if not isinstance(votes, dict) else len(p["rounds"])
    st = np.zeros(max(n, 1), np.int32)
    cp = committee.packed()
    cc = committee_struct(cp)
    check(_lib.lib().nw_votes_verify_many(ctypes.byref(cc), _p(p["ids"]), _p(p["rounds"]),
                                          _p(p["origins"]), _p(p["authors"]), _p(p["sigs"]), n,
                                          _p(st)), "nw_votes_verify_many")
    return st[:n]


def raise_for_status(code: int, index: int, header: Header | None, vote: Vote | None,
                     votes: Sequence[tuple[PublicKey, Signature]] = ()) -> None:
    """Map an NW_DAG_* status to the reference's DagError (Ok = return)."""
    if code == 0:
        return
    if code == DAG_INVALID_HEADER_ID:
        raise InvalidHeaderId()
    if code == DAG_UNKNOWN_AUTHORITY:
        if vote is not None:
            raise UnknownAuthority(vote.author)
        raise UnknownAuthority(header.author if index == 2**64 - 1 else votes[index][0])
    if code == DAG_MALFORMED_HEADER:
        raise MalformedHeader(header.id)
    if code == DAG_AUTHORITY_REUSE:
        raise AuthorityReuse(votes[index][0])
    if code == DAG_REQUIRES_QUORUM:
        raise CertificateRequiresQuorum()
    if DAG_INVALID_VOTES < code < DAG_INVALID_VOTES + 16:
        raise InvalidSignature(CryptoError(code - DAG_INVALID_VOTES, index), code)
    if DAG_INVALID_SIGNATURE < code < DAG_INVALID_SIGNATURE + 16:
        raise InvalidSignature(CryptoError(code - DAG_INVALID_SIGNATURE), code)
    raise RuntimeError(f"unexpected status {code}")
