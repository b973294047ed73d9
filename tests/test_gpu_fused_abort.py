"""a lone fused verify_batch whose job fails AFTER its launches were queued
must not leave the job's pooled completion counters (dfz) non-zero for the next call.
NW_TEST_FUSE_ABORT=1 (nw_jobs.cpp submit_batch test hook) fails the first such call after
its kernels ran and leaves its counters set to garbage; job_abort marks them dirty. The next
calls on the same pooled job must clear them and give the oracle's verdicts, without the
fused kernels' 2 s spin budget running out (a stale ticket would make them wait for
counters that never arrive). Runs in a child process (the hook is read once)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys, time
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from narwhal_amd import crypto as C
from oracle import oracle as O
from test_gpu_batch import _corpus_sizes, _mutate
rng = np.random.Generator(np.random.PCG64(5))
dig, pk, sigs, off, z16 = _corpus_sizes(np.array([10000]), rng, every=0)
bad = sigs.copy()
_mutate(bad, pk, 4321, 0)
d = C.Digest(dig[0].tobytes())
def call(s):
    votes = [(C.PublicKey(pk[i].tobytes()), C.Signature.from_bytes(s[i].tobytes())) for i in range(len(pk))]
    t = time.perf_counter()
    try:
        C.Signature.verify_batch(d, votes, z16=z16.tobytes())
        r = (0, None)
    except C.CryptoError as e:
        r = (e.code, e.index)
    except Exception as e:
        r = ("error", str(e))
    return r, time.perf_counter() - t
r0, _ = call(sigs)
assert r0[0] == "error" and "NW_TEST_FUSE_ABORT" in r0[1], r0
want_bad = O.verify_batch(dig[0].tobytes(), pk, bad, z16)
for s, want in ((sigs, (0, None)), (bad, want_bad), (sigs, (0, None))):
    r, dt = call(s)
    assert r[0] == want[0] and (want[0] == 0 or r[1] == want[1]), (r, want)
    assert dt < 1.0, dt
print("ABORT_OK")
"""


def test_fused_counters_cleared_after_failed_call():
    env = dict(os.environ, NW_TEST_FUSE_ABORT="1")
    r = subprocess.run([sys.executable, "-u", "-c", f"ROOT = {ROOT!r}\n" + _CHILD], env=env,
                       capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and "ABORT_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
