"""Certificate / Header / Vote test streams built with the ORACLE (test infrastructure).

Honest certificates come from narwhal_amd.workloads.certificate_stream with the oracle as
signer and hasher; ``mutated_stream`` then applies every primary::DagError class
(primary/src/messages.rs:48-67, 189-215; error.rs:26-59) with the status and index the
reference's check order implies. Those expectations are written here by hand from the
reference code, so the oracle is pinned against them (tests/test_messages.py) before it
is used to check the GPU (tests/test_gpu_messages.py).
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np

from narwhal_amd import workloads as W
from oracle import oracle as O

L_ORDER = 2**252 + 27742317777372353535851937790883648493
MAX = 2**64 - 1


def oracle_sign_many(sks: np.ndarray, msgs: np.ndarray) -> np.ndarray:
    return np.array([np.frombuffer(O.sign(bytes(k), bytes(m)), np.uint8)
                     for k, m in zip(sks, msgs)]).reshape(-1, 64)


def oracle_digest_many(data: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    b = data.tobytes()
    return np.array([np.frombuffer(hashlib.sha512(b[int(offsets[i]):int(offsets[i + 1])])
                                   .digest()[:32], np.uint8) for i in range(len(offsets) - 1)]
                    ).reshape(-1, 32)


def d32(b: bytes) -> bytes:
    return hashlib.sha512(b).digest()[:32]


def unpack(s: dict) -> list[dict]:
    """SoA stream -> list of records {hb, np, id, sig, votes[(pk, sig)]}."""
    out = []
    hb = s["header_bytes"].tobytes()
    for i in range(len(s["header_offsets"]) - 1):
        a, b = int(s["header_offsets"][i]), int(s["header_offsets"][i + 1])
        va, vb = int(s["vote_offsets"][i]), int(s["vote_offsets"][i + 1])
        out.append({"hb": hb[a:b], "np": int(s["payload_counts"][i]),
                    "id": s["ids"][i].tobytes(), "sig": s["header_sigs"][i].tobytes(),
                    "votes": [(s["vote_pks"][j].tobytes(), s["vote_sigs"][j].tobytes())
                              for j in range(va, vb)]})
    return out


def pack(recs: list[dict]) -> dict:
    ho = np.zeros(len(recs) + 1, np.uint64)
    ho[1:] = np.cumsum([len(r["hb"]) for r in recs])
    vo = np.zeros(len(recs) + 1, np.uint64)
    vo[1:] = np.cumsum([len(r["votes"]) for r in recs])
    vp = b"".join(pk for r in recs for pk, _ in r["votes"]) or bytes(32)
    vs = b"".join(sg for r in recs for _, sg in r["votes"]) or bytes(64)
    return {"header_bytes": np.frombuffer(b"".join(r["hb"] for r in recs) or b"\0", np.uint8).copy(),
            "header_offsets": ho,
            "payload_counts": np.array([r["np"] for r in recs], np.uint32),
            "ids": np.frombuffer(b"".join(r["id"] for r in recs), np.uint8).reshape(-1, 32).copy(),
            "header_sigs": np.frombuffer(b"".join(r["sig"] for r in recs), np.uint8).reshape(-1, 64).copy(),
            "vote_offsets": vo,
            "vote_pks": np.frombuffer(vp, np.uint8).reshape(-1, 32).copy(),
            "vote_sigs": np.frombuffer(vs, np.uint8).reshape(-1, 64).copy()}


def committee_with_zero_stake(keys, zero_key):
    """Committee of ``keys`` (stake 1, worker 0) plus ``zero_key`` at stake 0."""
    entries = sorted([(pk, 1) for pk, _ in keys] + [(zero_key[0], 0)])
    return {"pks": np.array([np.frombuffer(pk, np.uint8) for pk, _ in entries]),
            "stakes": np.array([s for _, s in entries], np.uint32),
            "worker_offsets": np.arange(len(entries) + 1, dtype=np.uint64),
            "worker_ids": np.zeros(len(entries), np.uint32)}


def mutated_stream(N: int = 4, copies: int = 1, seed: int = 5):
    """Returns (committee, stream, expected_status[n], expected_index[n], classes[n])."""
    keys = O.keys(N)
    outsider = O.keypair_from_seed(bytes([0xA5]) * 32)
    zero = O.keypair_from_seed(bytes([0x5A]) * 32)
    sk_of = {pk: sk for pk, sk in keys + [outsider, zero]}
    classes = ["honest", "genesis", "genesis_outsider", "id_flip", "author_outsider",
               "author_zero_stake", "bad_worker_id", "header_sig_flip", "header_sig_high",
               "vote_reuse", "vote_outsider", "vote_zero_stake", "no_quorum", "vote_sig_flip",
               "vote_sig_high", "vote_R_undecodable", "vote_s_plus_l", "id_flip_and_bad_votes",
               "all_votes", "payload_ok"]
    n = len(classes) * copies
    base = W.certificate_stream(n, keys, oracle_sign_many, oracle_digest_many, seed=seed,
                                n_votes=N)
    recs = unpack(base)
    q = W.quorum(N)
    exp_st, exp_ix, cls_of = [], [], []

    def resign(r, author=None, payload=None):
        hb = bytearray(r["hb"])
        if author is not None:
            hb[:32] = author[0]
        if payload is not None:
            parents = bytes(hb[40 + 36 * r["np"]:])
            hb = bytearray(bytes(hb[:40]) + payload[0] + parents)
            r["np"] = payload[1]
        r["hb"] = bytes(hb)
        r["id"] = d32(r["hb"])
        r["sig"] = O.sign(sk_of[r["hb"][:32]], r["id"])
        cd = d32(r["id"] + r["hb"][32:40] + r["hb"][:32])
        r["votes"] = [(pk, O.sign(sk_of[pk], cd)) for pk, _ in r["votes"]]
        return cd

    def cert_digest(r):
        return d32(r["id"] + r["hb"][32:40] + r["hb"][:32])

    for i, r in enumerate(recs):
        c = classes[i % len(classes)]
        st, ix = 0, 0
        r["votes"] = r["votes"][:q]                      # exactly a quorum by default
        if c == "genesis":
            r["hb"] = keys[i % N][0] + bytes(8)
            r["np"], r["id"], r["sig"], r["votes"] = 0, bytes(32), bytes(64), []
        elif c == "genesis_outsider":
            r["hb"] = outsider[0] + bytes(8)
            r["np"], r["id"], r["sig"], r["votes"] = 0, bytes(32), bytes(64), []
            st = 16
        elif c == "id_flip":
            r["id"] = bytes([r["id"][0] ^ 1]) + r["id"][1:]
            st = 16
        elif c == "author_outsider":
            resign(r, author=outsider)
            st, ix = 17, MAX
        elif c == "author_zero_stake":
            resign(r, author=zero)
            st, ix = 17, MAX
        elif c == "bad_worker_id":
            ents = (bytes([1]) * 32 + struct.pack("<I", 0)) + (bytes([2]) * 32 + struct.pack("<I", 7))
            resign(r, payload=(ents, 2))
            st, ix = 18, 1
        elif c == "payload_ok":
            ents = (bytes([1]) * 32 + struct.pack("<I", 0)) + (bytes([2]) * 32 + struct.pack("<I", 0))
            resign(r, payload=(ents, 2))
        elif c == "header_sig_flip":
            s = bytearray(r["sig"]); s[40] ^= 4; r["sig"] = bytes(s)
            st = 32 + 7
        elif c == "header_sig_high":
            s = bytearray(r["sig"]); s[63] |= 0x40; r["sig"] = bytes(s)
            st = 32 + 1
        elif c == "vote_reuse":
            r["votes"] = r["votes"][:2] + [r["votes"][0]] + r["votes"][3:]
            st, ix = 19, 2
        elif c == "vote_outsider":
            r["votes"][1] = (outsider[0], O.sign(outsider[1], cert_digest(r)))
            st, ix = 17, 1
        elif c == "vote_zero_stake":
            r["votes"][-1] = (zero[0], O.sign(zero[1], cert_digest(r)))
            st, ix = 17, len(r["votes"]) - 1
        elif c == "no_quorum":
            r["votes"] = r["votes"][:q - 1]
            st = 20
        elif c == "vote_sig_flip":
            pk, s = r["votes"][1]; s = bytearray(s); s[45] ^= 8
            r["votes"][1] = (pk, bytes(s))
            st, ix = 48 + 7, len(r["votes"])
        elif c == "vote_sig_high":
            pk, s = r["votes"][-1]; s = bytearray(s); s[63] |= 0x80
            r["votes"][-1] = (pk, bytes(s))
            st, ix = 48 + 1, len(r["votes"]) - 1
        elif c == "vote_R_undecodable":
            pk, s = r["votes"][0]
            r["votes"][0] = (pk, (2).to_bytes(32, "little") + s[32:])   # y = 2: not on the curve
            st, ix = 48 + 4, 0
        elif c == "vote_s_plus_l":
            pk, s = r["votes"][1]
            v = int.from_bytes(s[32:], "little") + L_ORDER
            r["votes"][1] = (pk, s[:32] + v.to_bytes(32, "little"))
            st, ix = 48 + 2, 1
        elif c == "id_flip_and_bad_votes":
            r["id"] = bytes([r["id"][0] ^ 0x80]) + r["id"][1:]
            r["votes"] = r["votes"][:1]
            st = 16
        elif c == "all_votes":
            cd = cert_digest(r)
            r["votes"] = [(pk, O.sign(sk, cd)) for pk, sk in keys]
        exp_st.append(st)
        exp_ix.append(ix)
        cls_of.append(c)
    com = committee_with_zero_stake(keys, zero)
    return com, pack(recs), np.array(exp_st, np.int32), np.array(exp_ix, np.uint64), cls_of


def votes_case(N: int = 4, seed: int = 3, count: int = 24, keys=None):
    """Vote stream (Vote::verify): honest votes plus tampered / unknown-author ones.
    Returns (committee, packed votes, n, expected status). keys: the committee's
    (pk, sk) pairs (default: the first N fixture keys)."""
    keys = O.keys(N) if keys is None else keys
    outsider = O.keypair_from_seed(bytes([0xA5]) * 32)
    rng = np.random.Generator(np.random.PCG64(seed))
    ids, rounds, origins, authors, sigs, exp = [], [], [], [], [], []
    for i in range(count):
        hid = rng.bytes(32)
        rnd = int(rng.integers(0, 2**63))
        origin = keys[i % N][0]
        author_pk, author_sk = keys[(i + 1) % N]
        kind = i % 4
        if kind == 2:
            author_pk, author_sk = outsider
        d = d32(hid + struct.pack("<Q", rnd) + origin)
        sig = O.sign(author_sk, d)
        st = 0
        if kind == 1:
            sig = sig[:33] + bytes([sig[33] ^ 2]) + sig[34:]
            st = 32 + 7
        elif kind == 2:
            st = 17
        elif kind == 3 and i % 8 == 7:
            rnd ^= 1                       # signature over another round
            st = 32 + 7
        ids.append(hid); rounds.append(rnd); origins.append(origin); authors.append(author_pk)
        sigs.append(sig); exp.append(st)
    cat = lambda xs, w: np.frombuffer(b"".join(xs), np.uint8).reshape(-1, w).copy()
    p = {"ids": cat(ids, 32), "rounds": np.array(rounds, np.uint64), "origins": cat(origins, 32),
         "authors": cat(authors, 32), "sigs": cat(sigs, 64)}
    com = {"pks": np.array([np.frombuffer(pk, np.uint8) for pk in sorted(pk for pk, _ in keys)]),
           "stakes": np.ones(N, np.uint32), "worker_offsets": np.arange(N + 1, dtype=np.uint64),
           "worker_ids": np.zeros(N, np.uint32)}
    return com, p, len(exp), np.array(exp, np.int32)
