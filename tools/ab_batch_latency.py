"""Median one-call latency of a 10k verify_batch through the host entry point (config 1),
over many calls: A/B helper for host-path changes (run once per setting). Streaming the
staging memcpy into 256 KB H2D pieces measured slower (0.386-0.394 vs 0.372 ms: each
hipMemcpyAsync costs more than the overlap saves), so the job path keeps one H2D."""
import ctypes, hashlib, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from narwhal_amd import _lib, crypto as C, workloads as W

L = _lib.lib()
n = 10_000
seeds = W.fixture_seeds(n)
pks = C.keypair_from_seed_many(seeds)
sks = np.concatenate([seeds, pks], axis=1)
digest = np.frombuffer(hashlib.sha512(b"Hello, world!").digest()[:32], np.uint8)
sigs = C.sign_many(sks, digest, shared_digest=True)
idx = ctypes.c_size_t(0)
vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)
lat = []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 300):
    t = time.perf_counter()
    rc = L.nw_signature_verify_batch(vp(digest), vp(pks), vp(sigs), n, None, ctypes.byref(idx))
    lat.append(time.perf_counter() - t)
    assert rc == 0, rc
lat = np.array(lat[20:]) * 1e3
print(f"median {np.median(lat):.4f} ms "
      f"p10 {np.percentile(lat, 10):.4f} p90 {np.percentile(lat, 90):.4f}")
