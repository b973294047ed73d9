#!/usr/bin/env python3
"""Config 1's one call (crypto::Signature::verify_batch over 10,000 pairs, the bench's inputs)
timed alone: N calls through the C entry point, median and p10 in microseconds, one JSON line.
The environment picks the variant (NW_BATCH_GATE, NW_GATE_CHUNK, ...; read once per process).

    python tools/r06/c1_ab.py 300
"""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from narwhal_amd import _lib, crypto as C, workloads as W  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    L = _lib.lib()
    n = 10_000
    seeds = W.fixture_seeds(n)
    pks = C.keypair_from_seed_many(seeds)
    sks = np.concatenate([seeds, pks], axis=1)
    digest = np.frombuffer(hashlib.sha512(b"Hello, world!").digest()[:32], np.uint8)
    sigs = C.sign_many(sks, digest, shared_digest=True)
    idx = ctypes.c_size_t(0)
    args = [a.ctypes.data_as(ctypes.c_void_p) for a in (digest, pks, sigs)]
    fn = L.nw_signature_verify_batch
    ok = True
    for _ in range(5):
        ok &= fn(args[0], args[1], args[2], n, None, ctypes.byref(idx)) == 0
    t = []
    for _ in range(calls):
        t0 = time.perf_counter()
        r = fn(args[0], args[1], args[2], n, None, ctypes.byref(idx))
        t.append(time.perf_counter() - t0)
        ok &= r == 0
    t = np.array(t) * 1e6
    env = {k: v for k, v in os.environ.items() if k.startswith("NW_")}
    print(json.dumps({"env": env, "calls": calls, "median_us": round(float(np.median(t)), 1),
                      "p10_us": round(float(np.percentile(t, 10)), 1),
                      "p90_us": round(float(np.percentile(t, 90)), 1), "ok": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
