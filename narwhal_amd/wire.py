"""Narwhal's primary wire format, and verification of received frames on the engine.

``serialize`` mirrors ``bincode::serialize(&PrimaryMessage::...)`` as the reference's Core
sends it (primary/src/core.rs:129, 204, 234; enum primary/src/primary.rs:32-38; bincode
1.3 fixint little-endian with u64 lengths; ``PublicKey`` as its base64 string,
crypto/src/lib.rs:94-112; ``Digest`` and ``Signature`` as raw bytes; BTreeMap/BTreeSet in
key order). ``verify_primary_messages`` hands a batch of received frames to
``nw_primary_messages_verify_wire``, which decodes them natively and verifies each with
the check the primary applies (Header::verify / Vote::verify / Certificate::verify), as
``PrimaryReceiverHandler::dispatch`` (primary/src/primary.rs:224-240) followed by
``Core::sanitize_*`` (primary/src/core.rs:306-346, verification part) would.
"""
from __future__ import annotations

import base64
import ctypes
import struct
from typing import Sequence

import numpy as np

from . import _lib
from ._lib import check
from .crypto import PublicKey, Signature
from .messages import Certificate, Committee, Header, Vote, _p, committee_struct

MSG_HEADER, MSG_VOTE, MSG_CERTIFICATE, MSG_CERTIFICATES_REQUEST = 0, 1, 2, 3
DAG_SERIALIZATION = 21

__all__ = ["serialize", "serialize_certificates_request", "verify_primary_messages", "scan",
           "MSG_HEADER", "MSG_VOTE", "MSG_CERTIFICATE", "MSG_CERTIFICATES_REQUEST",
           "DAG_SERIALIZATION"]


def _pk(pk: PublicKey) -> bytes:
    s = base64.b64encode(pk.value)          # base64 0.13 `encode` = STANDARD, padded
    return struct.pack("<Q", len(s)) + s


def _header(h: Header) -> bytes:
    out = [_pk(h.author), struct.pack("<Q", h.round), struct.pack("<Q", len(h.payload))]
    for d in sorted(h.payload):
        out.append(d.value + struct.pack("<I", h.payload[d]))
    out.append(struct.pack("<Q", len(h.parents)))
    out.extend(d.value for d in sorted(h.parents))
    out.append(h.id.value)
    out.append(h.signature.flatten())
    return b"".join(out)


def serialize(msg: Header | Vote | Certificate) -> bytes:
    """bincode::serialize(&PrimaryMessage::{Header, Vote, Certificate}(msg))."""
    if isinstance(msg, Header):
        return struct.pack("<I", MSG_HEADER) + _header(msg)
    if isinstance(msg, Vote):
        return (struct.pack("<I", MSG_VOTE) + msg.id.value + struct.pack("<Q", msg.round)
                + _pk(msg.origin) + _pk(msg.author) + msg.signature.flatten())
    if isinstance(msg, Certificate):
        out = [struct.pack("<I", MSG_CERTIFICATE), _header(msg.header),
               struct.pack("<Q", len(msg.votes))]
        for pk, sig in msg.votes:
            out.append(_pk(pk) + sig.flatten())
        return b"".join(out)
    raise TypeError(type(msg))


def serialize_certificates_request(digests: Sequence, requestor: PublicKey) -> bytes:
    """bincode::serialize(&PrimaryMessage::CertificatesRequest(digests, requestor))."""
    return (struct.pack("<I", MSG_CERTIFICATES_REQUEST) + struct.pack("<Q", len(digests))
            + b"".join(d.value for d in digests) + _pk(requestor))


def frames_soa(frames: Sequence[bytes]) -> tuple[np.ndarray, np.ndarray]:
    offs = np.zeros(len(frames) + 1, np.uint64)
    offs[1:] = np.cumsum([len(f) for f in frames]) if frames else []
    data = np.frombuffer(b"".join(frames) or b"\0", np.uint8).copy()
    return data, offs


def verify_primary_messages(committee: Committee | dict, frames: Sequence[bytes] | tuple
                            ) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Decode + verify received PrimaryMessage frames on the engine.
    Returns (kind int32[n]: MSG_* or -1, status int32[n]: 0 / NW_DAG_*, index uint64[n])."""
    data, offs = frames if isinstance(frames, tuple) else frames_soa(frames)
    n = len(offs) - 1
    kind = np.zeros(max(n, 1), np.int32)
    st = np.zeros(max(n, 1), np.int32)
    ix = np.zeros(max(n, 1), np.uint64)
    cc = committee_struct(committee if isinstance(committee, dict) else committee.packed())
    check(_lib.lib().nw_primary_messages_verify_wire(ctypes.byref(cc), _p(data), _p(offs), n,
                                                     _p(kind), _p(st), _p(ix)),
          "nw_primary_messages_verify_wire")
    return kind[:n], st[:n], ix[:n]


def scan(frames: Sequence[bytes] | tuple) -> tuple[np.ndarray, np.ndarray]:
    """Decode only (host code, no device): (kind int32[n], counts uint64[n, 3]) — payload
    entries and parents after de-duplication and votes, per nw_primary_messages_scan."""
    data, offs = frames if isinstance(frames, tuple) else frames_soa(frames)
    n = len(offs) - 1
    kind = np.zeros(max(n, 1), np.int32)
    counts = np.zeros((max(n, 1), 3), np.uint64)
    rc = _lib.lib().nw_primary_messages_scan(_p(data), _p(offs), n, _p(kind), _p(counts))
    if rc < 0:
        raise _lib.EngineError(f"nw_primary_messages_scan: {_lib.E_NAMES.get(rc, rc)}")
    return kind[:n], counts[:n]


def frames_from_stream(s: dict) -> tuple[np.ndarray, np.ndarray]:
    """bincode PrimaryMessage::Certificate frames for an nw_certificates SoA stream (the
    layout of narwhal_amd.workloads.certificate_stream / messages.pack_certificates)."""
    hb = s["header_bytes"].tobytes()
    ho, vo = s["header_offsets"], s["vote_offsets"]
    pcs = s["payload_counts"]
    ids, hs = s["ids"], s["header_sigs"]
    vpk, vsg = s["vote_pks"], s["vote_sigs"]
    tag = struct.pack("<I", MSG_CERTIFICATE)
    pk_cache: dict[bytes, bytes] = {}

    def pk(b: bytes) -> bytes:
        e = pk_cache.get(b)
        if e is None:
            e = pk_cache[b] = _pk(PublicKey(b))
        return e

    frames = []
    for i in range(len(ho) - 1):
        h = hb[int(ho[i]):int(ho[i + 1])]
        np_ = int(pcs[i])
        parents = h[40 + 36 * np_:]
        a, b = int(vo[i]), int(vo[i + 1])
        frames.append(b"".join([
            tag, pk(h[:32]), h[32:40], struct.pack("<Q", np_), h[40:40 + 36 * np_],
            struct.pack("<Q", len(parents) // 32), parents, ids[i].tobytes(), hs[i].tobytes(),
            struct.pack("<Q", b - a)] + [pk(vpk[j].tobytes()) + vsg[j].tobytes()
                                          for j in range(a, b)]))
    return frames_soa(frames)
