"""CPU-side checks of the C ABI boundary: the in-tree library loads, exports every symbol
include/narwhal_amd.h declares, and — with no GPU — fails loudly (negative NW_E_* codes,
EngineError), never silently computing on the CPU."""
import ctypes

import numpy as np
import pytest
import torch

from narwhal_amd import _lib
from narwhal_amd import crypto as C


def test_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s


def test_version():
    assert b"gfx950" in _lib.lib().nw_version()


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only behaviour")
def test_no_device_fails_loudly():
    L = _lib.lib()
    assert L.nw_init() == -2            # NW_E_NO_DEVICE
    assert L.nw_device_count() == 0
    assert L.nw_prepare() == -2
    with pytest.raises(_lib.EngineError):
        C.Signature(bytes(32), bytes(32)).verify(C.Digest(bytes(32)), C.PublicKey(bytes(32)))
    with pytest.raises(_lib.EngineError):
        C.sha512_digest(b"abc")
    st = ctypes.c_int32(0)
    assert L.nw_verify_strict_many(b"\0" * 32, 32, b"\0" * 32, b"\0" * 64, 1,
                                   ctypes.byref(st), None) == -2
    assert b"gfx950" in L.nw_last_error()
    # the fan-out mode fails the same way (no silent CPU path behind NW_ALL_DEVICES)
    assert L.nw_set_device(-1) == -2
    assert L.nw_submit_verify_strict(b"\0" * 32, 32, b"\0" * 32, b"\0" * 64, 1, None, None,
                                     ctypes.byref(ctypes.c_void_p())) == -2


def test_header_status_codes_match_oracle():
    from oracle import oracle as O
    txt = open(_lib.HEADER).read()
    for name, val in [("NW_OK", O.OK), ("NW_ERR_S_HIGH_BITS", O.ERR_S_HIGH_BITS),
                      ("NW_ERR_S_NONCANONICAL", O.ERR_S_NONCANONICAL),
                      ("NW_ERR_A_DECODE", O.ERR_A_DECODE), ("NW_ERR_R_DECODE", O.ERR_R_DECODE),
                      ("NW_ERR_A_SMALL_ORDER", O.ERR_A_SMALL_ORDER),
                      ("NW_ERR_R_SMALL_ORDER", O.ERR_R_SMALL_ORDER),
                      ("NW_ERR_EQUATION", O.ERR_EQUATION)]:
        assert f"#define {name} {val}" in txt, name


def test_digest_semantics():
    a, b = C.Digest(bytes([1] + [0] * 31)), C.Digest(bytes([0] * 31 + [2]))
    assert b < a                                  # lexicographic (derive(Ord))
    pk = C.PublicKey(bytes(range(32)))
    assert C.PublicKey.decode_base64(pk.encode_base64()) == pk
    assert C.Signature.from_bytes(bytes(64)).flatten() == bytes(64)
