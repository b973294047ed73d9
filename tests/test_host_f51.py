"""The host path's field in five 51-bit limbs (narwhal_amd/csrc/nw_host_f51.hpp, used by the
service hedge's comb checks) against Python integers mod p = 2^255 - 19: products, squares
and biased differences at the limb bounds the header states (mul / sq inputs up to 2^54 per
limb, sub's subtrahend loose < 2^52), canonical encoding of every residue class edge
(0, p - 1, p, 2^255 - 1, values >= p), decoding with bit 255 ignored, inversion. Through a
test shim (tools/f51_check.cpp) built here with g++. No GPU."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 2**255 - 19
M51 = 2**51 - 1


@pytest.fixture(scope="module")
def f51():
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = os.path.join(ROOT, "tools", "libnw_f51check.so")
    src = [os.path.join(ROOT, "tools", "f51_check.cpp"),
           os.path.join(ROOT, "narwhal_amd", "csrc", "nw_host_f51.hpp")]
    if not os.path.exists(out) or os.path.getmtime(out) < max(map(os.path.getmtime, src)):
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I",
                        os.path.join(ROOT, "narwhal_amd", "csrc"), src[0], "-o", out], check=True)
    L = ctypes.CDLL(out)
    for n in ("f51_mul", "f51_mul_limbs", "f51_sq", "f51_sub", "f51_tobytes", "f51_frombytes",
              "f51_invert", "f51_eq"):
        getattr(L, n).restype = ctypes.c_int if n == "f51_eq" else None
    return L


def limbs(x):
    return np.array([(x >> (51 * i)) & M51 for i in range(5)], np.uint64)


def value(l):
    return sum(int(v) << (51 * i) for i, v in enumerate(l))


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def tob(L, l):
    out = np.zeros(32, np.uint8)
    L.f51_tobytes(ptr(np.ascontiguousarray(l, np.uint64)), ptr(out))
    return int.from_bytes(out.tobytes(), "little")


EDGES = [0, 1, 2, 18, 19, 20, P - 2, P - 1, P, P + 1, P + 18, 2**255 - 1, 2**254, 2**51 - 1,
         2**51, 2**102 + 5]


def rand_limbs(rng, top):
    """Raw limbs uniformly below `top` each (the unreduced forms the formulas produce)."""
    return np.array([int(rng.integers(0, top)) for _ in range(5)], np.uint64)


def test_tobytes_canonical_edges(f51):
    for x in EDGES:
        assert tob(f51, limbs(x)) == x % P, x


def test_tobytes_unreduced_limbs(f51):
    rng = np.random.Generator(np.random.PCG64(1))
    for top in (2**51, 2**52, 2**53, 2**54):
        for _ in range(400):
            l = rand_limbs(rng, top)
            assert tob(f51, l) == value(l) % P
    for l in ([2**54 - 1] * 5, [0, 0, 0, 0, 2**54 - 1], [2**54 - 1, 0, 0, 0, 0]):
        assert tob(f51, np.array(l, np.uint64)) == value(l) % P


def test_mul_sq_at_bounds(f51):
    rng = np.random.Generator(np.random.PCG64(2))
    out = np.zeros(32, np.uint8)
    ol = np.zeros(5, np.uint64)
    cases = [np.array([2**54 - 1] * 5, np.uint64), limbs(P - 1), limbs(0), limbs(1)]
    cases += [rand_limbs(rng, t) for t in (2**51, 2**52, 2**53, 2**54) for _ in range(150)]
    for i, a in enumerate(cases):
        b = cases[(7 * i + 3) % len(cases)]
        f51.f51_mul(ptr(a), ptr(b), ptr(out))
        assert int.from_bytes(out.tobytes(), "little") == value(a) * value(b) % P, i
        f51.f51_mul_limbs(ptr(a), ptr(b), ptr(ol))
        assert all(int(v) < 2**52 for v in ol), ol            # "loose" output
        assert value(ol) % P == value(a) * value(b) % P
        f51.f51_sq(ptr(a), ptr(out))
        assert int.from_bytes(out.tobytes(), "little") == value(a) ** 2 % P, i


def test_sub_bias(f51):
    rng = np.random.Generator(np.random.PCG64(3))
    ol = np.zeros(5, np.uint64)
    for _ in range(600):
        a = rand_limbs(rng, 2**53)
        b = rand_limbs(rng, 2**52)          # sub's subtrahend is loose
        f51.f51_sub(ptr(a), ptr(b), ptr(ol))
        assert all(int(v) < 2**54 for v in ol)
        assert value(ol) % P == (value(a) - value(b)) % P


def test_frombytes_ignores_bit255_and_invert(f51):
    rng = np.random.Generator(np.random.PCG64(4))
    ol = np.zeros(5, np.uint64)
    out = np.zeros(32, np.uint8)
    for x in EDGES + [int.from_bytes(rng.bytes(32), "little") for _ in range(300)]:
        b = np.frombuffer(x.to_bytes(32, "little"), np.uint8).copy()
        f51.f51_frombytes(ptr(b), ptr(ol))
        assert value(ol) == x & (2**255 - 1)
        if (x & (2**255 - 1)) % P:
            f51.f51_invert(ptr(b), ptr(out))
            y = int.from_bytes(out.tobytes(), "little")
            assert y * (x & (2**255 - 1)) % P == 1
