"""Wire-format ingest (narwhal_amd/csrc/nw_wire.cpp): bincode
PrimaryMessage frames -> native decode -> Header/Vote/Certificate::verify.

The expectations come from an independent, test-only Python restatement of the serde +
bincode 1.3 semantics the reference's receiver applies (primary/src/primary.rs:230):
u32 variant, u64 lengths, base64 PublicKey strings (crypto/src/lib.rs:73-112, [..32]
slice), BTreeMap/BTreeSet re-sorting and de-duplication. Frames are built from the
certificate/vote corpora of tests/cert_cases.py plus wire-level mutations (truncation at
every byte, bad variants, base64 edge cases, duplicate/unsorted keys, trailing bytes).
Parity of the decode step is pinned only by this restatement (the reference holds no
serialized fixtures: "parity unpinned" beyond it); the verdicts after decoding are the
oracle's. CPU tests use the decode-only entry (nw_primary_messages_scan)."""
import base64
import hashlib
import struct

import numpy as np
import pytest

from narwhal_amd import wire as WI
from narwhal_amd.crypto import Digest, PublicKey, Signature
from narwhal_amd.messages import Certificate, Header, Vote
from oracle import oracle as O

from cert_cases import mutated_stream, pack, unpack, votes_case


# ------------------------------------------------------------------ test-only restatement
_B64 = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"


def ref_b64(s: bytes):
    """base64 0.13 STANDARD decode: padding optional, whole quads when padded, non-zero
    trailing bits rejected."""
    end, pad = len(s), 0
    while end and s[end - 1:end] == b"=" and pad < 2:
        end, pad = end - 1, pad + 1
    if (pad and len(s) % 4) or end % 4 == 1 or (pad and end % 4 + pad != 4):
        return None
    acc = bits = 0
    out = bytearray()
    for c in s[:end]:
        v = _B64.find(bytes([c]))
        if v < 0:
            return None
        acc, bits = (acc << 6) | v, bits + 6
        if bits >= 8:
            bits -= 8
            out.append(acc >> bits)
            acc &= (1 << bits) - 1
    return bytes(out) if acc == 0 else None


class _R:
    def __init__(self, b):
        self.b, self.p = b, 0

    def take(self, k):
        if k < 0 or self.p + k > len(self.b):
            raise ValueError("eof")
        r = self.b[self.p:self.p + k]
        self.p += k
        return r

    def u32(self):
        return struct.unpack("<I", self.take(4))[0]

    def u64(self):
        return struct.unpack("<Q", self.take(8))[0]

    def pk(self):
        d = ref_b64(self.take(self.u64()))
        if d is None or len(d) < 32:
            raise ValueError("pk")
        return d[:32]


def ref_decode(frame: bytes):
    """-> (kind, record) with record as tests/cert_cases.unpack produces, or (-1, None)."""
    r = _R(frame)
    try:
        v = r.u32()
        if v in (0, 2):
            author, rnd = r.pk(), r.u64()
            pay = {}
            for _ in range(r.u64()):
                d = r.take(32)
                pay[d] = r.u32()                       # BTreeMap: last value wins
            parents = {r.take(32) for _ in range(r.u64())}
            hid, sig = r.take(32), r.take(64)
            hb = (author + struct.pack("<Q", rnd)
                  + b"".join(d + struct.pack("<I", pay[d]) for d in sorted(pay))
                  + b"".join(sorted(parents)))
            rec = {"hb": hb, "np": len(pay), "id": hid, "sig": sig, "votes": [],
                   "nparents": len(parents)}
            if v == 2:
                rec["votes"] = [(r.pk(), r.take(64)) for _ in range(r.u64())]
            return v, rec
        if v == 1:
            hid, rnd = r.take(32), r.u64()
            origin, author, sig = r.pk(), r.pk(), r.take(64)
            return 1, {"id": hid, "round": rnd, "origin": origin, "author": author, "sig": sig}
        if v == 3:
            nd = r.u64()
            r.take(32 * nd)
            r.pk()
            return 3, {"nd": nd}
    except (ValueError, struct.error):
        pass
    return -1, None


# ------------------------------------------------------------------ frame builders
def _pk(b: bytes) -> bytes:
    s = base64.b64encode(b)
    return struct.pack("<Q", len(s)) + s


def cert_frame(rec, variant=2) -> bytes:
    hb, np_ = rec["hb"], rec["np"]
    parents = hb[40 + 36 * np_:]
    out = (struct.pack("<I", variant) + _pk(hb[:32]) + hb[32:40] + struct.pack("<Q", np_)
           + hb[40:40 + 36 * np_] + struct.pack("<Q", len(parents) // 32) + parents
           + rec["id"] + rec["sig"])
    if variant == 2:
        out += struct.pack("<Q", len(rec["votes"])) + b"".join(_pk(p) + s for p, s in rec["votes"])
    return out


def vote_frame(p, i) -> bytes:
    return (struct.pack("<I", 1) + p["ids"][i].tobytes() + struct.pack("<Q", int(p["rounds"][i]))
            + _pk(p["origins"][i].tobytes()) + _pk(p["authors"][i].tobytes())
            + p["sigs"][i].tobytes())


def _wire_mutations(rec):
    """Frames that must fail to decode, and frames that decode to something else."""
    good = cert_frame(rec)
    bad = [good[:k] for k in range(0, len(good), 7)]              # truncations
    bad.append(struct.pack("<I", 4) + good[4:])                     # unknown variant
    b64 = base64.b64encode(rec["hb"][:32])
    L = struct.pack("<Q", len(b64))
    last = _B64[_B64.index(b64[42:43]) | 1:][:1]
    for s in (b64[:42] + last + b"=",                                 # non-zero trailing bits
              b64.replace(b"=", b"") + b"==",                         # wrong padding
              b"!" + b64[1:],                                         # invalid symbol
              base64.b64encode(rec["hb"][:30]),                       # decodes to 30 bytes
              b64 + b"=",                                             # excess padding
              ):
        bad.append(struct.pack("<I", 2) + struct.pack("<Q", len(s)) + s + good[4 + 8 + len(b64):])
    odd = [good + b"\x00" * 5,                                        # trailing bytes: allowed
           struct.pack("<I", 2) + struct.pack("<Q", 43) + b64[:43] + good[4 + 8 + 44:],  # unpadded
           struct.pack("<I", 2) + _pk(rec["hb"][:32] + b"\x01\x02\x03\x04") + good[4 + 8 + 44:],
           struct.pack("<I", 2) + struct.pack("<Q", 44) + b64[:-1] + b"A"     # 33 bytes: [..32]
           + good[4 + 8 + 44:]]
    return bad, odd


def _dup_key_frame(rec):
    """Payload with a duplicate key (last value wins) and parents out of order."""
    hb = rec["hb"]
    parents = [hb[40 + 36 * rec["np"] + 32 * j:40 + 36 * rec["np"] + 32 * (j + 1)]
               for j in range((len(hb) - 40 - 36 * rec["np"]) // 32)]
    d = hashlib.sha512(b"dup").digest()[:32]
    pay = d + struct.pack("<I", 9) + d + struct.pack("<I", 0)
    out = (struct.pack("<I", 2) + _pk(hb[:32]) + hb[32:40] + struct.pack("<Q", 2) + pay
           + struct.pack("<Q", len(parents) + 1) + b"".join(parents[::-1] + parents[:1])
           + rec["id"] + rec["sig"] + struct.pack("<Q", len(rec["votes"]))
           + b"".join(_pk(p) + s for p, s in rec["votes"]))
    return out


def _corpus(N=4, copies=1, seed=11):
    com, s, _, _, _ = mutated_stream(N=N, copies=copies, seed=seed)
    recs = unpack(s)
    frames = [cert_frame(r) for r in recs] + [cert_frame(r, 0) for r in recs[:8]]
    vcom, vp, vn, _ = votes_case(N)
    frames += [vote_frame(vp, i) for i in range(vn)]
    bad, odd = _wire_mutations(recs[0])
    assert all(ref_decode(f)[0] == -1 for f in bad)
    assert all(ref_decode(f)[0] == 2 for f in odd)
    frames += bad + odd + [_dup_key_frame(recs[0])]
    frames.append(WI.serialize_certificates_request([Digest(bytes(32))] * 3,
                                                    PublicKey(recs[0]["hb"][:32])))
    return com, frames


# ------------------------------------------------------------------ CPU
def test_encoder_matches_restatement_and_appendix_b(golden):
    """serialize(header()) decodes (restatement) to the fixture whose id is SURVEY
    Appendix B's, and the scan agrees on kinds and counts."""
    keys = O.keys(4)
    author, secret = keys[-1]
    d32 = lambda b: hashlib.sha512(b).digest()[:32]
    genesis = {Digest(d32(bytes(32) + struct.pack("<Q", 0) + pk)) for pk, _ in keys}
    h = Header(author=PublicKey(author), round=1, parents=genesis)
    h.id = Digest(d32(h.digest_bytes()))
    h.signature = Signature.from_bytes(O.sign(secret, h.id.value))
    f = WI.serialize(h)
    kind, rec = ref_decode(f)
    assert kind == 0 and d32(rec["hb"]) == h.id.value
    assert base64.b64encode(h.id.value).decode() == golden["keys"]["appendix_b"]["header_id_b64"]
    assert len(f) == 4 + 52 + 8 + 8 + 8 + 32 * 4 + 32 + 64
    v = Vote(h.id, 1, h.author, PublicKey(keys[0][0]))
    c = Certificate(h, [(PublicKey(pk), Signature.from_bytes(bytes(64))) for pk, _ in keys])
    k, cnt = WI.scan([f, WI.serialize(v), WI.serialize(c)])
    assert k.tolist() == [0, 1, 2]
    assert cnt.tolist() == [[0, 4, 0], [0, 0, 0], [0, 4, 4]]


def test_scan_vs_restatement():
    _, frames = _corpus()
    kind, counts = WI.scan(frames)
    for i, f in enumerate(frames):
        k, rec = ref_decode(f)
        assert kind[i] == k, (i, k, kind[i])
        if k in (0, 2):
            assert counts[i].tolist() == [rec["np"], rec["nparents"], len(rec["votes"])], i
    assert (kind == -1).sum() >= 20 and (kind == 2).sum() >= 20


def test_scan_every_truncation_of_every_variant():
    _, frames = _corpus()
    for f in frames[:3] + frames[-40:-20]:
        cuts = [f[:k] for k in range(len(f))]
        kind, _ = WI.scan(cuts)
        assert kind.tolist() == [ref_decode(c)[0] for c in cuts]


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_verify_wire_vs_oracle():
    com, frames = _corpus(N=4, copies=2)
    kind, st, ix = WI.verify_primary_messages(com, frames)
    exp_st = np.zeros(len(frames), np.int32)
    exp_kind = np.zeros(len(frames), np.int32)
    certs, headers, votes = [], [], []
    for i, f in enumerate(frames):
        k, rec = ref_decode(f)
        exp_kind[i] = k
        if k == -1:
            exp_st[i] = WI.DAG_SERIALIZATION
        elif k == 2:
            certs.append((i, rec))
        elif k == 0:
            headers.append((i, rec))
        elif k == 1:
            votes.append((i, rec))
    assert kind.tolist() == exp_kind.tolist()
    if certs:
        # batch coefficients are random on the wire path: compare on the deterministic set
        ost, _ = O.certificates_verify_many(com, pack([r for _, r in certs]))
        for (i, _), e in zip(certs, ost):
            exp_st[i] = e
    if headers:
        ost, _ = O.certificates_verify_many(com, pack([r for _, r in headers]), headers_only=True)
        for (i, _), e in zip(headers, ost):
            exp_st[i] = e
    if votes:
        cat = lambda key, w: np.frombuffer(b"".join(r[key] for _, r in votes), np.uint8).reshape(-1, w)
        vp = {"ids": cat("id", 32), "rounds": np.array([r["round"] for _, r in votes], np.uint64),
              "origins": cat("origin", 32), "authors": cat("author", 32), "sigs": cat("sig", 64)}
        ost = O.votes_verify_many(com, vp, len(votes))
        for (i, _), e in zip(votes, ost):
            exp_st[i] = e
    bad = [(i, int(a), int(b)) for i, (a, b) in enumerate(zip(st, exp_st)) if a != b]
    assert not bad, bad


@pytest.mark.gpu
def test_verify_wire_multithreaded_decode():
    """> 4096 frames per call: the decode splits over threads and merges the parts in place
    (nw_wire.cpp decode_all). Tiling the small corpus must tile its statuses exactly."""
    com, frames = _corpus(N=4, copies=2)
    kind0, st0, _ = WI.verify_primary_messages(com, frames)
    reps = -(-9000 // len(frames))
    tiled = list(frames) * reps
    for _ in range(2):   # second call reuses the per-thread buffers
        kind, st, _ = WI.verify_primary_messages(com, tiled)
        assert kind.tolist() == np.tile(kind0, reps).tolist()
        assert st.tolist() == np.tile(st0, reps).tolist()


def test_frames_from_stream_round_trip():
    """The bench's frame builder (wire.frames_from_stream) against the restatement."""
    from narwhal_amd import workloads as W
    from cert_cases import oracle_digest_many, oracle_sign_many
    keys = O.keys(4)
    s = W.certificate_stream(10, keys, oracle_sign_many, oracle_digest_many, payload=2, seed=1)
    data, offs = WI.frames_from_stream(s)
    recs = unpack(s)
    b = data.tobytes()
    for i, r in enumerate(recs):
        k, d = ref_decode(b[int(offs[i]):int(offs[i + 1])])
        assert k == 2 and d["hb"] == r["hb"] and d["id"] == r["id"] and d["votes"] == r["votes"]
    kind, counts = WI.scan((data, offs))
    assert (kind == 2).all() and counts[:, 0].tolist() == [2] * 10
