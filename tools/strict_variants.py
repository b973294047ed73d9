#!/usr/bin/env python3
"""A/B timing of k_verify_strict builds in ONE process (GPU box).

    python tools/strict_variants.py [--items N] [--reps R] [--steps K] LIB [LIB ...]

Each LIB is a build of libnarwhal_amd.so (the in-tree one, or exp/<v>/libnarwhal_amd.so
built here with one kernel change). All are loaded side by side (ctypes, RTLD_LOCAL: every
copy has its own HIP module and constants), the config-4 corpus is built once (bench.py's
build_strict_corpus with the in-tree library), and the variants are timed interleaved
round-robin over R rounds of K launches, so clock drift hits all of them alike. Every
variant's statuses must equal the in-tree build's. One JSON line per variant.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    P, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.nw_init.restype = I
    L.nw_set_device.argtypes = [I]
    L.nw_last_error.restype = ctypes.c_char_p
    L.nw_dev_verify_strict_many.argtypes = [P, S, P, P, S, P, P, P]
    L.nw_dev_verify_strict_many.restype = I
    assert L.nw_init() > 0, L.nw_last_error()
    assert L.nw_set_device(0) == 0
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--items", type=int, default=12_500_000)
    ap.add_argument("--unique", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--all-valid", action="store_true",
                    help="tile only the corpus's valid items (no early-decided statuses)")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ts = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(ts)
    stream = ctypes.c_void_p(ts.cuda_stream)
    from narwhal_amd import _lib
    assert _lib.lib().nw_init() > 0
    m_u, p_u, s_u, valid = bench.build_strict_corpus(dev, stream, a.unique, 4096, seed=1000)
    n = a.items
    if a.all_valid:
        good = torch.from_numpy(np.nonzero(valid)[0]).to(dev)
        idx = good[torch.arange(n, dtype=torch.int64, device=dev) % good.numel()]
        valid = np.ones(good.numel(), dtype=bool)
    else:
        idx = torch.arange(n, dtype=torch.int64, device=dev) % a.unique
    m, p, s = (t.index_select(0, idx).contiguous() for t in (m_u, p_u, s_u))
    del idx
    exp = np.resize(valid, n)
    libs = [load(x) for x in a.libs]
    st = torch.empty(n, dtype=torch.int32, device=dev)
    bm = torch.zeros((n + 63) // 64 * 8, dtype=torch.uint8, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    times = {x: [] for x in a.libs}
    ok = {}
    for rep in range(a.reps):
        for name, L in zip(a.libs, libs):
            def launch():
                rc = L.nw_dev_verify_strict_many(P(m), 32, P(p), P(s), n, P(st), P(bm), stream)
                assert rc == 0, L.nw_last_error()
            launch()
            torch.cuda.synchronize()
            if rep == 0:
                ok[name] = bool(np.array_equal(st.cpu().numpy() == 0, exp))
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(a.steps)]
            for e0, e1 in evs:
                e0.record()
                launch()
                e1.record()
            torch.cuda.synchronize()
            times[name] += [e0.elapsed_time(e1) for e0, e1 in evs]
    for name in a.libs:
        ms = float(np.median(times[name]))
        print(json.dumps({"lib": name, "median_ms": ms, "verifies_per_s": n / ms * 1e3,
                          "min_ms": float(np.min(times[name])), "parity": ok[name]}), flush=True)


if __name__ == "__main__":
    main()
