"""ctypes wrapper over oracle/libnw_oracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference's crypto path (see nw_oracle.h for the
reference file:line each function follows). Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker; the
product (narwhal_amd) never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libnw_oracle.so")

OK = 0
ERR_S_HIGH_BITS = 1
ERR_S_NONCANONICAL = 2
ERR_A_DECODE = 3
ERR_R_DECODE = 4
ERR_A_SMALL_ORDER = 5
ERR_R_SMALL_ORDER = 6
ERR_EQUATION = 7

_lib = None


def build() -> str:
    """Compile libnw_oracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        S = ctypes.c_size_t
        I = ctypes.c_int
        L.nwo_sha512.argtypes = [P, S, P]
        L.nwo_sha512_digest32_many.argtypes = [P, P, P, S, P, I]
        L.nwo_chacha20_keystream.argtypes = [P, P, ctypes.c_uint64, P, S]
        L.nwo_keypair_from_seed.argtypes = [P, P, P]
        L.nwo_sign.argtypes = [P, P, S, P]
        L.nwo_sign_raw.argtypes = [P, P, P, P, S, P]
        L.nwo_verify_strict.argtypes = [P, S, P, P]
        L.nwo_verify_strict.restype = I
        L.nwo_verify_strict_many.argtypes = [P, S, P, P, S, P, I]
        L.nwo_verify_batch.argtypes = [P, P, P, S, P, ctypes.POINTER(S)]
        L.nwo_verify_batch.restype = I
        L.nwo_verify_batch_many.argtypes = [P, P, P, P, S, P, P, I]
        L.nwo_decompress.argtypes = [P, P]
        L.nwo_decompress.restype = I
        L.nwo_is_small_order.argtypes = [P]
        L.nwo_is_small_order.restype = I
        L.nwo_hram.argtypes = [P, P, P, S, P]
        L.nwo_scalar_reduce64.argtypes = [P, P]
        L.nwo_scalar_mul.argtypes = [P, P, P]
        L.nwo_scalar_add.argtypes = [P, P, P]
        L.nwo_scalarmult_base.argtypes = [P, P]
        L.nwo_scalarmult.argtypes = [P, P, P]
        L.nwo_scalarmult.restype = I
        L.nwo_point_add.argtypes = [P, P, P]
        L.nwo_point_add.restype = I
        L.nwo_msm.argtypes = [P, P, S, P, ctypes.POINTER(I)]
        L.nwo_msm.restype = I
        L.nwo_digest_72.argtypes = [P, ctypes.c_uint64, P, P]
        L.nwo_certificates_verify_many.argtypes = [P, P, P, P, P, P, P, P, P, S, P, I, P, P, I]
        L.nwo_votes_verify_many.argtypes = [P, P, P, P, P, P, S, P]
        # the timed dalek-equivalent restatement (nw_dalek.c), same signatures
        L.nwd_verify_strict.argtypes = [P, S, P, P]
        L.nwd_verify_strict.restype = I
        L.nwd_verify_strict_many.argtypes = [P, S, P, P, S, P, I]
        L.nwd_verify_batch.argtypes = [P, P, P, S, P, ctypes.POINTER(S)]
        L.nwd_verify_batch.restype = I
        L.nwd_verify_batch_many.argtypes = [P, P, P, P, S, P, P, I]
        L.nwd_double_base.argtypes = [P, P, P, P]
        L.nwd_double_base.restype = I
        L.nwd_certificates_verify_many.argtypes = [P, P, P, P, P, P, P, P, P, S, P, I, P, P, I]
        _lib = L
    return _lib


# engine="check": the parity checker (nw_oracle.c); engine="dalek": the dalek-equivalent
# restatement (nw_dalek.c: NAF-5 / affine NAF-8 double-base, Straus / Pippenger MSM), which
# bench.py times as cpu_baseline. Same verdicts; tests/test_dalek_restatement.py checks it.
DALEK_ALGORITHM = ("dalek-equivalent restatement (ed25519-dalek 1.0.1 / curve25519-dalek 3 u64 "
                   "backend): radix-2^51 field, width-5 NAF of k over 8 cached odd multiples of "
                   "-A, width-8 NAF of s over 64 affine odd multiples of B; verify_batch: "
                   "vartime Straus (NAF-5) below 190 points, Pippenger w=6/7/8 (<500/<800/>=800)")


def _fn(name: str, engine: str):
    if engine not in ("check", "dalek"):
        raise ValueError(f"unknown oracle engine {engine!r}")
    return getattr(lib(), ("nwd_" if engine == "dalek" else "nwo_") + name)


def _buf(b: bytes):
    return ctypes.c_char_p(bytes(b))


def _np_ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def sha512(msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().nwo_sha512(_buf(msg), len(msg), out)
    return out.raw


def digest32(msg: bytes) -> bytes:
    """Digest(Sha512(msg)[..32]) — worker/src/processor.rs:38."""
    return sha512(msg)[:32]


def sha512_digest32_many(data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
                         nthreads: int = 0) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    n = len(offsets)
    out = np.zeros((n, 32), dtype=np.uint8)
    lib().nwo_sha512_digest32_many(_np_ptr(data), _np_ptr(offsets), _np_ptr(lengths), n,
                                   _np_ptr(out), nthreads)
    return out


def chacha20(key: bytes, nonce: bytes, counter: int, n: int) -> bytes:
    out = ctypes.create_string_buffer(n)
    lib().nwo_chacha20_keystream(_buf(key), _buf(nonce), counter, out, n)
    return out.raw


def stdrng_seeds(count: int, seed: bytes = bytes(32)) -> list[bytes]:
    """rand 0.7 StdRng::from_seed(seed) fill_bytes(32) x count (crypto_tests.rs:26-29)."""
    ks = chacha20(seed, bytes(8), 0, 32 * count)
    return [ks[32 * i:32 * i + 32] for i in range(count)]


def keypair_from_seed(seed: bytes) -> tuple[bytes, bytes]:
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    lib().nwo_keypair_from_seed(_buf(seed), pk, sk)
    return pk.raw, sk.raw


def keys(count: int = 4) -> list[tuple[bytes, bytes]]:
    """The reference's keys() fixture (crypto/src/tests/crypto_tests.rs:26-29)."""
    return [keypair_from_seed(s) for s in stdrng_seeds(count)]


def sign(sk: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().nwo_sign(_buf(sk), _buf(msg), len(msg), out)
    return out.raw


def sign_raw(a: bytes, prefix: bytes, A: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(64)
    lib().nwo_sign_raw(_buf(a), _buf(prefix), _buf(A), _buf(msg), len(msg), out)
    return out.raw


def verify_strict(msg: bytes, pk: bytes, sig: bytes, engine: str = "check") -> int:
    return _fn("verify_strict", engine)(_buf(msg), len(msg), _buf(pk), _buf(sig))


def verify_strict_many(msgs: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                       shared_msg: bool = False, nthreads: int = 0,
                       engine: str = "check") -> np.ndarray:
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    pks = np.ascontiguousarray(pks, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    n = pks.shape[0]
    st = np.zeros(n, dtype=np.int32)
    _fn("verify_strict_many", engine)(_np_ptr(msgs), 0 if shared_msg else 32, _np_ptr(pks),
                                      _np_ptr(sigs), n, _np_ptr(st), nthreads)
    return st


def verify_batch(digest: bytes, pks: np.ndarray, sigs: np.ndarray,
                 z16: np.ndarray | None = None, engine: str = "check") -> tuple[int, int]:
    pks = np.ascontiguousarray(pks, dtype=np.uint8).reshape(-1, 32)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(-1, 64)
    n = pks.shape[0]
    idx = ctypes.c_size_t(0)
    zp = None
    if z16 is not None:
        z16 = np.ascontiguousarray(z16, dtype=np.uint8).reshape(-1, 16)
        zp = _np_ptr(z16)
    st = _fn("verify_batch", engine)(_buf(digest), _np_ptr(pks), _np_ptr(sigs), n, zp,
                                     ctypes.byref(idx))
    return st, idx.value


def verify_batch_many(digests: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                      offsets: np.ndarray, z16: np.ndarray | None = None,
                      nthreads: int = 0, engine: str = "check") -> np.ndarray:
    digests = np.ascontiguousarray(digests, dtype=np.uint8)
    pks = np.ascontiguousarray(pks, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    nb = len(offsets) - 1
    st = np.zeros(nb, dtype=np.int32)
    zp = None
    if z16 is not None:
        z16 = np.ascontiguousarray(z16, dtype=np.uint8)
        zp = _np_ptr(z16)
    _fn("verify_batch_many", engine)(_np_ptr(digests), _np_ptr(pks), _np_ptr(sigs),
                                     _np_ptr(offsets), nb, zp, _np_ptr(st), nthreads)
    return st


def decompress(p: bytes) -> bytes | None:
    out = ctypes.create_string_buffer(32)
    ok = lib().nwo_decompress(_buf(p), out)
    return out.raw if ok else None


def is_small_order(p: bytes) -> int:
    return lib().nwo_is_small_order(_buf(p))


def hram(R: bytes, A: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().nwo_hram(_buf(R), _buf(A), _buf(msg), len(msg), out)
    return out.raw


def scalar_reduce64(x: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().nwo_scalar_reduce64(_buf(x), out)
    return out.raw


def scalar_mul(a: bytes, b: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().nwo_scalar_mul(_buf(a), _buf(b), out)
    return out.raw


def scalar_add(a: bytes, b: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().nwo_scalar_add(_buf(a), _buf(b), out)
    return out.raw


def scalarmult_base(s: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().nwo_scalarmult_base(_buf(s), out)
    return out.raw


def scalarmult(s: bytes, P: bytes) -> bytes | None:
    out = ctypes.create_string_buffer(32)
    return out.raw if lib().nwo_scalarmult(_buf(s), _buf(P), out) else None


def point_add(P: bytes, Q: bytes) -> bytes | None:
    out = ctypes.create_string_buffer(32)
    return out.raw if lib().nwo_point_add(_buf(P), _buf(Q), out) else None


def msm(scalars: list[bytes], points: list[bytes]) -> tuple[bytes, bool] | None:
    n = len(points)
    out = ctypes.create_string_buffer(32)
    ident = ctypes.c_int(0)
    ok = lib().nwo_msm(_buf(b"".join(scalars)), _buf(b"".join(points)), n, out,
                       ctypes.byref(ident))
    return (out.raw, bool(ident.value)) if ok else None


# ---- primary messages (primary/src/messages.rs:48-67, 131-153, 189-234) ----
class _Committee(ctypes.Structure):
    _fields_ = [("nauth", ctypes.c_size_t), ("pks", ctypes.c_void_p),
                ("stakes", ctypes.c_void_p), ("worker_offsets", ctypes.c_void_p),
                ("worker_ids", ctypes.c_void_p)]


def _committee(c: dict) -> _Committee:
    return _Committee(len(c["stakes"]), _np_ptr(c["pks"]), _np_ptr(c["stakes"]),
                      _np_ptr(c["worker_offsets"]), _np_ptr(c["worker_ids"]))


def double_base(a: bytes, A: bytes, b: bytes) -> bytes | None:
    """encode([a]A + [b]B) by the dalek-equivalent vartime_double_scalar_mul_basepoint."""
    out = ctypes.create_string_buffer(32)
    return out.raw if lib().nwd_double_base(_buf(a), _buf(A), _buf(b), out) else None


def digest_72(x: bytes, round_: int, y: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().nwo_digest_72(_buf(x), round_, _buf(y), out)
    return out.raw


def certificates_verify_many(committee: dict, p: dict, z16: np.ndarray | None = None,
                             headers_only: bool = False, nthreads: int = 0,
                             engine: str = "check") -> tuple[np.ndarray, np.ndarray]:
    """Certificate::verify (or Header::verify) over a packed stream (same SoA layout as
    narwhal_amd.messages.pack_certificates / pack_committee)."""
    n = len(p["header_offsets"]) - 1
    st = np.zeros(max(n, 1), np.int32)
    ix = np.zeros(max(n, 1), np.uint64)
    cc = _committee(committee)
    zp = None
    if z16 is not None:
        z16 = np.ascontiguousarray(z16, np.uint8)
        zp = _np_ptr(z16)
    _fn("certificates_verify_many", engine)(
        ctypes.byref(cc), _np_ptr(p["header_bytes"]), _np_ptr(p["header_offsets"]),
        _np_ptr(p["payload_counts"]), _np_ptr(p["ids"]), _np_ptr(p["header_sigs"]),
        _np_ptr(p["vote_offsets"]), _np_ptr(p["vote_pks"]), _np_ptr(p["vote_sigs"]), n, zp,
        1 if headers_only else 0, _np_ptr(st), _np_ptr(ix), nthreads)
    return st[:n], ix[:n]


def votes_verify_many(committee: dict, p: dict, n: int) -> np.ndarray:
    st = np.zeros(max(n, 1), np.int32)
    cc = _committee(committee)
    lib().nwo_votes_verify_many(ctypes.byref(cc), _np_ptr(p["ids"]), _np_ptr(p["rounds"]),
                                _np_ptr(p["origins"]), _np_ptr(p["authors"]), _np_ptr(p["sigs"]),
                                n, _np_ptr(st))
    return st[:n]
