"""Loader for the in-tree C-ABI library narwhal_amd/libnarwhal_amd.so (gfx950 kernels).

There is deliberately no fallback: if the library is missing, or no gfx950 device is
visible, every compute call raises. Building: ``make`` at the repo root (or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnarwhal_amd.so")
# NW_LIB: an alternative build of the same library (compiler-flag experiments); the
# default is always the in-tree build.
LIB_PATH = os.environ.get("NW_LIB", LIB_PATH)
HEADER = os.path.join(os.path.dirname(_HERE), "include", "narwhal_amd.h")

NW_OK = 0
ERR_NAMES = {1: "S_HIGH_BITS", 2: "S_NONCANONICAL", 3: "A_DECODE", 4: "R_DECODE",
             5: "A_SMALL_ORDER", 6: "R_SMALL_ORDER", 7: "EQUATION"}
DAG_NAMES = {16: "InvalidHeaderId", 17: "UnknownAuthority", 18: "MalformedHeader",
             19: "AuthorityReuse", 20: "CertificateRequiresQuorum"}
E_NAMES = {-1: "NW_E_INVALID_ARG", -2: "NW_E_NO_DEVICE", -3: "NW_E_DEVICE",
           -4: "NW_E_OUT_OF_MEMORY"}

_lib = None

# void (*fn)(void*) for nw_job_notify
NOTIFY_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
# void (*fn)(void* arg, int32_t status, uint64_t index) for the nw_service_* requests
VERDICT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64)


class EngineError(RuntimeError):
    """A runtime/device failure (negative NW_E_* code) — never an 'invalid signature'."""


def header_symbols() -> list[str]:
    """Every nw_* function declared in include/narwhal_amd.h."""
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(nw_[a-z0-9_]+)\s*\(", txt)))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"{LIB_PATH} not built (run `make` at the repo root); "
                          "narwhal_amd has no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    sig = {
        "nw_init": ([], I), "nw_device_count": ([], I), "nw_set_device": ([I], I),
        "nw_get_device": ([], I), "nw_last_error": ([], ctypes.c_char_p),
        "nw_version": ([], ctypes.c_char_p), "nw_synchronize": ([], I), "nw_prepare": ([], I),
        "nw_sha512_digest32_many": ([P, P, P, S, P], I),
        "nw_signature_verify": ([P, P, P], I),
        "nw_verify_strict_many": ([P, S, P, P, S, P, P], I),
        "nw_signature_verify_batch": ([P, P, P, S, P, ctypes.POINTER(S)], I),
        "nw_verify_batch_many": ([P, P, P, P, S, P, P], I),
        "nw_dev_sha512_digest32_many": ([P, P, P, S, P, P], I),
        "nw_dev_verify_strict_many": ([P, S, P, P, S, P, P, P], I),
        "nw_keypair_from_seed_many": ([P, S, P], I),
        "nw_sign_many": ([P, S, P, S, S, P], I),
        "nw_dev_keypair_from_seed_many": ([P, S, P, P], I),
        "nw_dev_sign_many": ([P, S, P, S, S, P, P], I),
        "nw_dev_verify_batch_workspace": ([S, S], S),
        "nw_dev_verify_batch_many": ([P, P, P, P, P, S, S, P, P, P, P, P, P], I),
        "nw_certificates_verify_many": ([P, P, P, P, P], I),
        "nw_headers_verify_many": ([P, P, P, P], I),
        "nw_votes_verify_many": ([P, P, P, P, P, P, S, P], I),
        "nw_dev_certificates_workspace": ([S, S], S),
        "nw_dev_certificates_verify_many": ([P, P, I, P, P, P, P, P, P], I),
        "nw_submit_verify_strict": ([P, S, P, P, S, P, P, ctypes.POINTER(P)], I),
        "nw_submit_verify_batch_many": ([P, P, P, P, S, P, P, P, ctypes.POINTER(P)], I),
        "nw_submit_sha512_digest32_many": ([P, P, P, S, P, ctypes.POINTER(P)], I),
        "nw_submit_certificates_verify_many": ([P, P, P, P, P, ctypes.POINTER(P)], I),
        "nw_submit_headers_verify_many": ([P, P, P, P, ctypes.POINTER(P)], I),
        "nw_submit_votes_verify_many": ([P, P, P, P, P, P, S, P, ctypes.POINTER(P)], I),
        "nw_job_poll": ([P], I), "nw_job_wait": ([P], I),
        "nw_job_notify": ([P, NOTIFY_FN, P], I), "nw_job_release": ([P], None),
        "nw_path_stats": ([P, P], I),
        "nw_primary_messages_verify_wire": ([P, P, P, S, P, P, P], I),
        "nw_primary_messages_scan": ([P, P, S, P, P], I),
        "nw_service_create": ([P, S, ctypes.c_uint32, S, ctypes.POINTER(P)], I),
        "nw_service_certificate": ([P, P, S, ctypes.c_uint32, P, P, P, P, S, VERDICT_FN, P], I),
        "nw_service_header": ([P, P, S, ctypes.c_uint32, P, P, VERDICT_FN, P], I),
        "nw_service_vote": ([P, P, ctypes.c_uint64, P, P, P, VERDICT_FN, P], I),
        "nw_service_verify": ([P, P, P, P, VERDICT_FN, P], I),
        "nw_service_verify_batch": ([P, P, P, P, S, VERDICT_FN, P], I),
        "nw_service_flush": ([P], I), "nw_service_drain": ([P], I),
        "nw_service_stats": ([P, P, P], I), "nw_service_destroy": ([P], None),
        "nw_service_set_hedge": ([P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64], I),
        "nw_service_hedge_stats": ([P, P, P, P, P], I),
        "nw_host_verify_strict_many": ([P, S, P, P, S, P], I),
        "nw_host_verify_batch_many": ([P, P, P, P, S, P, P, P], I),
        "nw_host_certificates_verify_many": ([P, P, P, I, P, P], I),
        "nw_host_votes_verify_many": ([P, P, P, P, P, P, S, P], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def path_stats() -> tuple[int, int]:
    """(small-job launches, bulk-pipeline jobs) of Header / Vote / Certificate host calls so
    far (nw_path_stats)."""
    a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
    lib().nw_path_stats(ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def check(rc: int, what: str) -> int:
    """Raise EngineError for negative (runtime) codes; pass verdicts (>= 0) through."""
    if rc < 0:
        msg = lib().nw_last_error().decode(errors="replace")
        raise EngineError(f"{what}: {E_NAMES.get(rc, rc)}: {msg}")
    return rc
