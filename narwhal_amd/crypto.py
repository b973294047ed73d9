"""Host-side mirror of the reference's ``crypto`` crate surface over the MI355X engine.

Reference: /root/reference/crypto/src/lib.rs. Same names, argument meaning and error
behaviour, so code (and tests) written against the Rust crate read the same here:

    Digest(bytes32)                       lib.rs:20-57   (Ord = lexicographic bytes)
    Hash protocol (.digest() -> Digest)   lib.rs:59-62
    PublicKey(bytes32), base64 helpers    lib.rs:64-118
    Signature(part1, part2), flatten      lib.rs:177-198
    Signature.verify(digest, pk)          lib.rs:200-204  -> raises CryptoError
    Signature.verify_batch(digest, votes) lib.rs:206-219  -> raises CryptoError
    CryptoError                           lib.rs:18 (ed25519::Error, opaque)

Every check runs in the gfx950 kernels through the C ABI (include/narwhal_amd.h); there
is no CPU path. Runtime/device failures raise EngineError, never CryptoError.
Bulk helpers (verify_strict_many, verify_batch_many, sha512_digest32_many) expose the
batched entry points the aggregation service uses.
"""
from __future__ import annotations

import base64
import ctypes
from dataclasses import dataclass, field
from typing import Iterable, Protocol

import numpy as np

from . import _lib
from ._lib import EngineError, check

__all__ = ["Digest", "Hash", "PublicKey", "SecretKey", "Signature", "CryptoError",
           "EngineError", "generate_keypair", "keypair_from_seed_many", "sign_many",
           "sha512_digest", "sha512_digest32_many", "verify_strict_many",
           "verify_batch_many"]


class CryptoError(Exception):
    """Opaque verification failure (the reference's ed25519::Error). ``code`` names the
    first failing check (NW_ERR_*), for diagnostics only."""

    def __init__(self, code: int, index: int | None = None):
        self.code = code
        self.index = index
        super().__init__(f"signature error: {_lib.ERR_NAMES.get(code, code)}"
                         + ("" if index is None else f" (item {index})"))


@dataclass(frozen=True, order=True)
class Digest:
    """32-byte hash digest; ordering is lexicographic on the bytes (derive(Ord))."""
    value: bytes = bytes(32)

    def __post_init__(self):
        if len(self.value) != 32:
            raise ValueError("Digest must be 32 bytes")

    def to_vec(self) -> bytes:
        return self.value

    def size(self) -> int:
        return 32

    def __repr__(self) -> str:       # Debug: base64
        return base64.b64encode(self.value).decode()

    def __str__(self) -> str:        # Display: first 16 base64 chars
        return base64.b64encode(self.value).decode()[:16]


class Hash(Protocol):
    def digest(self) -> Digest: ...


@dataclass(frozen=True, order=True)
class PublicKey:
    value: bytes = bytes(32)

    def __post_init__(self):
        if len(self.value) != 32:
            raise ValueError("PublicKey must be 32 bytes")

    def encode_base64(self) -> str:
        return base64.b64encode(self.value).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "PublicKey":
        raw = base64.b64decode(s)
        if len(raw) < 32:
            raise ValueError("InvalidLength")
        return cls(raw[:32])

    def __repr__(self) -> str:
        return self.encode_base64()


class SecretKey:
    """crypto::SecretKey (lib.rs:120-161): seed || public key, zeroised on drop."""

    def __init__(self, raw: bytes):
        if len(raw) != 64:
            raise ValueError("SecretKey must be 64 bytes")
        self._raw = bytearray(raw)

    def encode_base64(self) -> str:
        return base64.b64encode(bytes(self._raw)).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "SecretKey":
        raw = base64.b64decode(s)
        if len(raw) < 64:
            raise ValueError("InvalidLength")
        return cls(raw[:64])

    def __bytes__(self) -> bytes:
        return bytes(self._raw)

    def __eq__(self, other) -> bool:
        return isinstance(other, SecretKey) and self._raw == other._raw

    def __del__(self):
        for i in range(len(self._raw)):
            self._raw[i] = 0


def keypair_from_seed_many(seeds: np.ndarray) -> np.ndarray:
    """Public keys for n 32-byte seeds (dalek Keypair::generate given the RNG output)."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
    out = np.zeros_like(seeds)
    if len(seeds):
        check(_lib.lib().nw_keypair_from_seed_many(_ptr(seeds), len(seeds), _ptr(out)),
              "nw_keypair_from_seed_many")
    return out


def generate_keypair(fill_bytes) -> tuple[PublicKey, SecretKey]:
    """crypto::generate_keypair(csprng) (lib.rs:167-175); fill_bytes(n) -> n random bytes
    plays the RNG (e.g. oracle.stdrng_seeds-compatible ChaCha20, or os.urandom)."""
    seed = bytes(fill_bytes(32))
    pk = keypair_from_seed_many(np.frombuffer(seed, np.uint8))[0].tobytes()
    return PublicKey(pk), SecretKey(seed + pk)


def sign_many(sks: np.ndarray, digests: np.ndarray, shared_key: bool = False,
              shared_digest: bool = False) -> np.ndarray:
    """n x Signature::new (RFC 8032 deterministic). Returns n x 64 bytes."""
    sks = np.ascontiguousarray(sks, dtype=np.uint8)
    digests = np.ascontiguousarray(digests, dtype=np.uint8)
    n = max(1 if shared_key else sks.size // 64, 1 if shared_digest else digests.size // 32)
    out = np.zeros((n, 64), np.uint8)
    check(_lib.lib().nw_sign_many(_ptr(sks), 0 if shared_key else 64, _ptr(digests),
                                  0 if shared_digest else 32, n, _ptr(out)), "nw_sign_many")
    return out


@dataclass(frozen=True)
class Signature:
    part1: bytes = bytes(32)   # R
    part2: bytes = bytes(32)   # s

    @classmethod
    def from_bytes(cls, b: bytes) -> "Signature":
        if len(b) != 64:
            raise ValueError("signature must be 64 bytes")
        return cls(bytes(b[:32]), bytes(b[32:]))

    @classmethod
    def new(cls, digest: Digest, secret: SecretKey) -> "Signature":
        """crypto::Signature::new (lib.rs:185-191)."""
        sig = sign_many(np.frombuffer(bytes(secret), np.uint8),
                        np.frombuffer(digest.value, np.uint8), shared_key=True,
                        shared_digest=True)[0].tobytes()
        return cls.from_bytes(sig)

    def flatten(self) -> bytes:
        return self.part1 + self.part2

    def verify(self, digest: Digest, public_key: PublicKey) -> None:
        """crypto::Signature::verify -> dalek verify_strict semantics."""
        L = _lib.lib()
        rc = check(L.nw_signature_verify(_cbuf(self.flatten()), _cbuf(digest.value),
                                         _cbuf(public_key.value)), "nw_signature_verify")
        if rc != _lib.NW_OK:
            raise CryptoError(rc)

    @staticmethod
    def verify_batch(digest: Digest, votes: Iterable[tuple[PublicKey, "Signature"]],
                     z16: bytes | None = None) -> None:
        """crypto::Signature::verify_batch (empty -> Ok). z16 injects the 128-bit
        coefficients (n x 16 bytes) for deterministic tests; default = fresh CSPRNG."""
        votes = list(votes)
        n = len(votes)
        pks = b"".join(pk.value for pk, _ in votes)
        sigs = b"".join(s.flatten() for _, s in votes)
        idx = ctypes.c_size_t(0)
        L = _lib.lib()
        rc = check(L.nw_signature_verify_batch(_cbuf(digest.value), _cbuf(pks), _cbuf(sigs), n,
                                               None if z16 is None else _cbuf(z16),
                                               ctypes.byref(idx)),
                   "nw_signature_verify_batch")
        if rc != _lib.NW_OK:
            raise CryptoError(rc, idx.value)


def _cbuf(b: bytes):
    return ctypes.c_char_p(bytes(b)) if b else ctypes.c_char_p(b"\0")


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def sha512_digest(data: bytes) -> Digest:
    """Digest(Sha512::digest(data)[..32]) on the GPU (worker/src/processor.rs:38)."""
    out = sha512_digest32_many(np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8),
                               np.array([0], np.uint64), np.array([len(data)], np.uint64))
    return Digest(out[0].tobytes())


def sha512_digest32_many(data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    n = len(offsets)
    out = np.zeros((n, 32), dtype=np.uint8)
    check(_lib.lib().nw_sha512_digest32_many(_ptr(data), _ptr(offsets), _ptr(lengths), n,
                                             _ptr(out)), "nw_sha512_digest32_many")
    return out


def verify_strict_many(digests: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                       shared_digest: bool = False) -> tuple[np.ndarray, np.ndarray]:
    """Bulk Signature::verify. Returns (status int32[n], bitmap uint8[ceil(n/8)])."""
    digests = np.ascontiguousarray(digests, dtype=np.uint8)
    pks = np.ascontiguousarray(pks, dtype=np.uint8).reshape(-1, 32)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(-1, 64)
    n = pks.shape[0]
    st = np.zeros(n, dtype=np.int32)
    bm = np.zeros((n + 7) // 8, dtype=np.uint8)
    if n:
        check(_lib.lib().nw_verify_strict_many(_ptr(digests), 0 if shared_digest else 32,
                                               _ptr(pks), _ptr(sigs), n, _ptr(st), _ptr(bm)),
              "nw_verify_strict_many")
    return st, bm


def verify_batch_many(digests: np.ndarray, pks: np.ndarray, sigs: np.ndarray,
                      offsets: np.ndarray, z16: np.ndarray | None = None) -> np.ndarray:
    """Bulk Signature::verify_batch: batch b = items offsets[b]..offsets[b+1]."""
    digests = np.ascontiguousarray(digests, dtype=np.uint8)
    pks = np.ascontiguousarray(pks, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    nb = len(offsets) - 1
    st = np.zeros(nb, dtype=np.int32)
    zp = None
    if z16 is not None:
        z16 = np.ascontiguousarray(z16, dtype=np.uint8)
        zp = _ptr(z16)
    check(_lib.lib().nw_verify_batch_many(_ptr(digests), _ptr(pks), _ptr(sigs), _ptr(offsets),
                                          nb, zp, _ptr(st)), "nw_verify_batch_many")
    return st
