#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/gen_golden.py

Independent anchors (none of them is the oracle under test):
  * hashlib (OpenSSL 3.0.2)                     -> SHA-512 known answers
  * libsodium 1.0.18 (/opt/conda/lib)           -> key derivation, RFC 8032 signing,
                                                   ChaCha20 keystream, strict verdicts
  * RFC 8032 section 7.1 test vectors 1-3       -> literal values below
  * SURVEY.md Appendix B values                  -> literal values below
The oracle (oracle/libnw_oracle.so) is used only to CONSTRUCT inputs that need curve
arithmetic libsodium does not expose (torsion points, mixed-order keys, injected-z
batch residuals); every such construction is cross-checked against libsodium where
the Appendix A contract says the two agree, and the expected status codes follow the
Appendix A contract table (reference semantics, crypto/src/lib.rs:200-219).

The reference (Rust) holds no known-answer vectors for this path:
its tests are sign-then-verify properties, restated in tests/test_reference_scenarios.py.
"""
from __future__ import annotations

import base64
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O          # noqa: E402  (construction helper only)
from narwhal_amd import workloads as W  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493

so = ctypes.CDLL("/opt/conda/lib/libsodium.so")
assert so.sodium_init() >= 0


def sod_keypair(seed: bytes) -> tuple[bytes, bytes]:
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    assert so.crypto_sign_seed_keypair(pk, sk, seed) == 0
    return pk.raw, sk.raw


def sod_sign(sk: bytes, m: bytes) -> bytes:
    s = ctypes.create_string_buffer(64)
    so.crypto_sign_detached(s, None, m, ctypes.c_ulonglong(len(m)), sk)
    return s.raw


def sod_verify(sig: bytes, m: bytes, pk: bytes) -> bool:
    return so.crypto_sign_verify_detached(sig, m, ctypes.c_ulonglong(len(m)), pk) == 0


def sod_chacha(key: bytes, n: int) -> bytes:
    out = ctypes.create_string_buffer(n)
    so.crypto_stream_chacha20(out, ctypes.c_ulonglong(n), bytes(8), key)
    return out.raw


def le(x: int) -> bytes:
    return x.to_bytes(32, "little")


def enc_y(y: int, sign: int) -> bytes:
    b = bytearray(le(y))
    b[31] |= sign << 7
    return bytes(b)


def h(b: bytes) -> str:
    return b.hex()


# --------------------------------------------------------------------------------------
def gen_sha512():
    vecs = []
    rng = np.random.Generator(np.random.PCG64(7))
    for name, m in [("empty", b""), ("abc", b"abc"),
                    ("reference_serialized_batch_228", W.reference_serialized_batch())]:
        vecs.append({"name": name, "msg": h(m), "sha512": hashlib.sha512(m).hexdigest()})
    for n in [1, 55, 72, 96, 111, 112, 113, 127, 128, 129, 239, 240, 241, 255, 256, 1000, 3300]:
        m = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        vecs.append({"name": f"random_{n}", "msg": h(m), "sha512": hashlib.sha512(m).hexdigest()})
    big = []
    for bid in [0, 1, 65535]:
        m = W.worker_batch(bid).tobytes()
        assert len(m) == W.BATCH_BYTES == 508052
        big.append({"batch_id": bid, "seed": 0, "len": len(m),
                    "sha512": hashlib.sha512(m).hexdigest()})
    # worker serialized_batch() digest.
    assert base64.b64encode(hashlib.sha512(W.reference_serialized_batch()).digest()[:32]).decode() \
        == "JNAPdKB2fnSAjIVGYwkClyhT+iAOB55YK4t73s1zMdg="
    return {"vectors": vecs, "worker_batches": big}


# --------------------------------------------------------------------------------------
RFC8032 = [  # RFC 8032 section 7.1, TEST 1..3 (secret key = seed)
    ("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
     "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
     "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe24655141438e7a100b"),
    ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
     "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
     "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aeeb00d291612bb0c00"),
    ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
     "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
     "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28dc027beceea1ec40a"),
]


def gen_keys():
    seeds_ks = sod_chacha(bytes(32), 32 * 4)
    seeds = [seeds_ks[32 * i:32 * i + 32] for i in range(4)]
    assert [s[:8].hex() for s in seeds] == ["76b8e0ada0f13d90", "da41597c5157488d",
                                           "9f07e7be5551387a", "29b721769ce64e43"]
    pks = [sod_keypair(s)[0] for s in seeds]
    assert [base64.b64encode(p).decode() for p in pks] == [
        "IP26ybELdYe7p7W8FjvOaeeW1x5O1EwQ/LRIhon3oUQ=", "deQXTdWIIlSAhvF7A3zssO6GUWt9E0AKgMhWtL2vf+E=",
        "YxwVQfOkv0TU2JcGFWSqhJXXZvYZGj/2FWIAPxhLjGU=", "vq2gYSbHjZi0oaafbuYYlpTw9HUVONqCTxrcixShtWI="]
    digest = hashlib.sha512(b"Hello, world!").digest()[:32]
    assert base64.b64encode(digest).decode() == "wVJ82JPBJHc9gRkRlwyP5uhX1t9dySJr2KFgYUwM2WM="
    sig3 = sod_sign(sod_keypair(seeds[3])[1], digest)
    assert sig3.hex() == ("fd1017091c871c5feb5b171ada10a5b636522f10ce6a2c8cbec12dafe78455a5"
                          "693a194e5b7a3baa25fbd5b04dbfed62a3b766872435625f1d7aeeace9afcd07")
    rfc = []
    for sk, pk, m, sig in RFC8032:
        pk2, skf = sod_keypair(bytes.fromhex(sk))
        assert pk2.hex() == pk and sod_sign(skf, bytes.fromhex(m)).hex() == sig
        rfc.append({"seed": sk, "pk": pk, "msg": m, "sig": sig})
    return {
        "stdrng_zero_seed_keys": [{"seed": h(s), "pk": h(p)} for s, p in zip(seeds, pks)],
        "hello_digest": h(digest),
        "hello_sig_key3": h(sig3),
        "rfc8032": rfc,
        # SURVEY Appendix B (primary header() fixture values, derived in the survey container)
        "appendix_b": {
            "header_id_b64": "x9EEQngGDO7nM65hC8F/shrTrbm1yweqNaxLG/iBmFk=",
            "header_sig": "8d1ba7c6b3f186b879565990964ce88c21658712b793d6a406fbd249e39be2ffba6f17ee78f3b1cd0a134779c0faf7b42eec4cb318f8450608de121ec9e97107",
            "certificate_digest_b64": "SUtj4JGoXKMCr6o120L2B4+SJHHJFr7kQxFTp9hKA3M=",
        },
    }


# --------------------------------------------------------------------------------------
SMALL_ORDER_CANONICAL = [
    "0100000000000000000000000000000000000000000000000000000000000000",   # identity
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",   # order 2
    "0000000000000000000000000000000000000000000000000000000000000000",   # order 4
    "0000000000000000000000000000000000000000000000000000000000000080",   # order 4
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",   # order 8
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",   # order 8
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",   # order 8
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",   # order 8
]
SMALL_ORDER_NONCANONICAL = [
    h(enc_y(P, 0)), h(enc_y(P, 1)),            # y = p   (= 0)
    h(enc_y(P + 1, 0)), h(enc_y(P + 1, 1)),    # y = p+1 (= 1)
    h(enc_y(1, 1)),                            # identity, sign bit set (x = -0)
    h(enc_y(P - 1, 1)),                        # order 2, sign bit set
]


def gen_edge_corpus():
    """Strict-verify edge classes. Expected status codes are
    the reference's check order (crypto/src/lib.rs:200-204 -> dalek verify_strict)."""
    rng = np.random.Generator(np.random.PCG64(2024))
    seeds = [rng.bytes(32) for _ in range(8)]
    kp = [sod_keypair(s) for s in seeds]
    msg = hashlib.sha512(b"edge corpus message").digest()[:32]
    other = hashlib.sha512(b"a different message").digest()[:32]
    items = []

    def add(cls, m, pk, sig, expect, sodium_agrees=True):
        st = O.verify_strict(m, pk, sig)
        assert st == expect, (cls, st, expect)
        sv = sod_verify(sig, m, pk)
        if sodium_agrees:
            assert sv == (expect == 0), (cls, sv, expect)
        items.append({"class": cls, "msg": h(m), "pk": h(pk), "sig": h(sig), "status": expect,
                      "libsodium_valid": sv})

    for i, (pk, sk) in enumerate(kp):
        add("honest", msg, pk, sod_sign(sk, msg), 0)
    pk0, sk0 = kp[0]
    sig0 = sod_sign(sk0, msg)
    add("wrong_message", other, pk0, sig0, 7)
    for bit in [0, 77, 200, 254]:     # bit flips in R
        s = bytearray(sig0); s[bit // 8] ^= 1 << (bit % 8)
        exp = O.verify_strict(msg, pk0, bytes(s))
        assert exp in (4, 6, 7)
        add(f"flip_R_bit{bit}", msg, pk0, bytes(s), exp)
    for bit in [256, 300, 500]:       # bit flips in s (keep < l)
        s = bytearray(sig0); s[bit // 8] ^= 1 << (bit % 8)
        add(f"flip_s_bit{bit - 256}", msg, pk0, bytes(s), 7)
    for bit in [0, 100, 254]:         # bit flips in A
        p = bytearray(pk0); p[bit // 8] ^= 1 << (bit % 8)
        exp = O.verify_strict(msg, bytes(p), sig0)
        assert exp in (3, 5, 7)
        add(f"flip_A_bit{bit}", msg, bytes(p), sig0, exp)
    # s + l: non-canonical scalar (bits 253..255 still clear).
    s_int = int.from_bytes(sig0[32:], "little")
    add("s_plus_l", msg, pk0, sig0[:32] + le(s_int + L), 2)
    add("s_high_bit_255", msg, pk0, sig0[:63] + bytes([sig0[63] | 0x80]), 1)
    add("s_high_bit_253", msg, pk0, sig0[:63] + bytes([sig0[63] | 0x20]), 1)
    add("s_eq_l", msg, pk0, sig0[:32] + le(L), 2)
    add("s_eq_2^252", msg, pk0, sig0[:32] + le(2**252), 7)     # < l: canonical, wrong
    # Not on the curve (decode failure) for A and for R.
    bad = []
    for y in range(2, 200):
        if O.decompress(enc_y(y, 0)) is None:
            bad.append(y)
        if len(bad) >= 3:
            break
    for y in bad:
        add(f"A_not_on_curve_y{y}", msg, enc_y(y, 0), sig0, 3)
        add(f"R_not_on_curve_y{y}", msg, pk0, enc_y(y, 1) + sig0[32:], 4)
    for t in [2, 7]:
        y = P + t
        if O.decompress(enc_y(y, 0)) is None:
            add(f"A_noncanon_not_on_curve_p+{t}", msg, enc_y(y, 0), sig0, 3)
            add(f"R_noncanon_not_on_curve_p+{t}", msg, pk0, enc_y(y, 1) + sig0[32:], 4)
    # Small-order A and R, canonical and non-canonical encodings.
    for i, e in enumerate(SMALL_ORDER_CANONICAL + SMALL_ORDER_NONCANONICAL):
        eb = bytes.fromhex(e)
        assert O.is_small_order(eb) == 1, e
        add(f"A_small_order_{i}", msg, eb, sig0, 5)
        add(f"R_small_order_{i}", msg, pk0, eb + sig0[32:], 6)
    # Signature::default() (crypto_tests.rs:110-114): R = 0 (order 4) -> R small.
    add("signature_default", msg, pk0, bytes(64), 6)
    # Non-canonical large-order encodings y in p + {3,4,5,6,9,10,14,15,16,18}: dalek decodes
    # them (libsodium rejects as non-canonical); no valid signature exists -> equation.
    for t in [3, 4, 5, 6, 9, 10, 14, 15, 16, 18]:
        for sign in (0, 1):
            eb = enc_y(P + t, sign)
            assert O.decompress(eb) is not None and O.is_small_order(eb) == 0, t
            add(f"A_noncanon_large_order_p+{t}_s{sign}", msg, eb, sig0, 7)
            add(f"R_noncanon_large_order_p+{t}_s{sign}", msg, pk0, eb + sig0[32:], 7)
    # Mixed-order A = aB + T8: strict accepts iff k*T8 == 0 (k = 0 mod 8).
    T8 = bytes.fromhex(SMALL_ORDER_CANONICAL[4])
    a = (int.from_bytes(rng.bytes(32), "little") % L).to_bytes(32, "little")
    prefix = rng.bytes(32)
    A = O.point_add(O.scalarmult_base(a), T8)
    assert O.is_small_order(A) == 0
    got_acc = got_rej = 0
    for j in range(400):
        m = hashlib.sha512(b"mixed" + bytes([j % 256, j // 256])).digest()[:32]
        sig = O.sign_raw(a, prefix, A, m)
        k = int.from_bytes(O.hram(sig[:32], A, m), "little")
        if k % 8 == 0 and got_acc < 3:
            add("mixed_order_A_kT_zero", m, A, sig, 0)      # libsodium 1.0.18 accepts too
            got_acc += 1
        elif k % 8 != 0 and got_rej < 3:
            add("mixed_order_A_kT_nonzero", m, A, sig, 7)
            got_rej += 1
        if got_acc >= 3 and got_rej >= 3:
            break
    assert got_acc == 3 and got_rej == 3
    # Small-order A with R = [s]B: strict rejects (A small), cofactorless equation holds.
    s = (int.from_bytes(rng.bytes(32), "little") % L).to_bytes(32, "little")
    R = O.scalarmult_base(s)
    add("A_identity_R_eq_sB", msg, SMALL_ORDER_CANONICAL[0] and bytes.fromhex(SMALL_ORDER_CANONICAL[0]),
        R + s, 5)
    return {"items": items}


def gen_batches():
    """verify_batch scenarios with injected z (crypto/src/lib.rs:206-219 + dalek
    verify_batch). Status: 0 Ok, else the first failure in reference order."""
    rng = np.random.Generator(np.random.PCG64(99))
    digest = hashlib.sha512(b"Hello, world!").digest()[:32]
    ks = O.keys(4)
    batches = []

    def add(name, pks, sigs, expect, z=None, expect_idx=None):
        n = len(pks)
        if z is None:
            z = rng.bytes(16 * n)
        pa = np.frombuffer(b"".join(pks), dtype=np.uint8).reshape(-1, 32) if n else np.zeros((0, 32), np.uint8)
        sa = np.frombuffer(b"".join(sigs), dtype=np.uint8).reshape(-1, 64) if n else np.zeros((0, 64), np.uint8)
        za = np.frombuffer(z, dtype=np.uint8).reshape(-1, 16) if n else None
        st, idx = O.verify_batch(digest, pa, sa, za)
        assert st == expect, (name, st, expect)
        if expect_idx is not None:
            assert idx == expect_idx, (name, idx, expect_idx)
        batches.append({"name": name, "digest": h(digest), "pks": [h(p) for p in pks],
                        "sigs": [h(s) for s in sigs], "z": h(z), "status": st, "index": idx})

    # crypto_tests.rs:79-94 verify_valid_batch: 3 sigs from keys().pop() x3
    keys3 = list(reversed(ks))[:3]
    add("verify_valid_batch", [p for p, _ in keys3], [O.sign(sk, digest) for _, sk in keys3], 0)
    # crypto_tests.rs:96-115 verify_invalid_batch: 2 valid + Signature::default()
    keys2 = list(reversed(ks))[:2]
    add("verify_invalid_batch", [p for p, _ in keys2] + [ks[1][0]],
        [O.sign(sk, digest) for _, sk in keys2] + [bytes(64)], 7)
    add("empty", [], [], 0)
    # large honest batch
    seeds = O.stdrng_seeds(64)
    kp = [O.keypair_from_seed(s) for s in seeds]
    pks = [p for p, _ in kp]
    sigs = [O.sign(sk, digest) for _, sk in kp]
    add("honest_64", pks, sigs, 0)
    add("honest_64_last_default", pks, sigs[:-1] + [bytes(64)], 7)
    bad = bytearray(sigs[10]); bad[40] ^= 1
    add("honest_64_flip_s", pks, sigs[:10] + [bytes(bad)] + sigs[11:], 7)
    # ordering: high-bit s at 20, A decode failure at 5 -> crypto loop hits index 5 first
    s20 = sigs[20][:63] + bytes([sigs[20][63] | 0x80])
    add("order_A_decode_before_s_high", pks[:5] + [enc_y(2, 0)] + pks[6:],
        sigs[:20] + [s20] + sigs[21:], 3, expect_idx=5)
    add("s_high_bits", pks, sigs[:20] + [s20] + sigs[21:], 1, expect_idx=20)
    # non-canonical s at 30 is reported after all from_bytes passed
    s30 = sigs[30][:32] + le(int.from_bytes(sigs[30][32:], "little") + L)
    add("s_noncanonical", pks, sigs[:30] + [s30] + sigs[31:], 2, expect_idx=30)
    # R decode failure
    r40 = enc_y(2, 0) + sigs[40][32:]
    assert O.decompress(enc_y(2, 0)) is None
    add("R_decode", pks, sigs[:40] + [r40] + sigs[41:], 4, expect_idx=40)
    # Strict != batch: A = identity, R = [s]B satisfies the cofactorless equation.
    s = (int.from_bytes(rng.bytes(32), "little") % L).to_bytes(32, "little")
    R = O.scalarmult_base(s)
    ident = bytes.fromhex(SMALL_ORDER_CANONICAL[0])
    add("small_order_A_equation_holds", pks[:3] + [ident], sigs[:3] + [R + s], 0)
    # Torsion-only residual: mixed-order A with k*T8 != 0. Verdict depends on z: Ok iff
    # (z*k mod l)*T8 == identity, i.e. (z*k mod l) = 0 mod 8.
    T8 = bytes.fromhex(SMALL_ORDER_CANONICAL[4])
    a = (int.from_bytes(rng.bytes(32), "little") % L).to_bytes(32, "little")
    prefix = rng.bytes(32)
    A = O.point_add(O.scalarmult_base(a), T8)
    for j in range(100):
        sig = O.sign_raw(a, prefix, A, digest if j == 0 else digest)
        k = int.from_bytes(O.hram(sig[:32], A, digest), "little")
        if k % 8:
            break
        prefix = rng.bytes(32)
    assert k % 8
    z_ok = z_bad = None
    for _ in range(2000):
        zc = rng.bytes(16)
        zk = (int.from_bytes(zc, "little") * k) % L
        if zk % 8 == 0 and z_ok is None:
            z_ok = zc
        if zk % 8 != 0 and z_bad is None:
            z_bad = zc
        if z_ok and z_bad:
            break
    base_z = rng.bytes(16 * 3)
    add("torsion_residual_z_cancels", pks[:3] + [A], sigs[:3] + [sig], 0, z=base_z + z_ok)
    add("torsion_residual_z_exposes", pks[:3] + [A], sigs[:3] + [sig], 7, z=base_z + z_bad)
    return {"batches": batches}


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, fn in [("sha512.json", gen_sha512), ("keys.json", gen_keys),
                     ("edge_corpus.json", gen_edge_corpus), ("batches.json", gen_batches)]:
        data = fn()
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(data, f, indent=1)
        print("wrote", name)


if __name__ == "__main__":
    main()
