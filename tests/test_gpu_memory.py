"""Device memory: the engine's large per-device tables (strict B tables 2.15 GB, keyed B comb
11.8 GB, committee key tables 67 MB per key) and what happens without room for them.
NW_DEVICE_MEM_LIMIT (test hook, nw_kernels.hip table_malloc) makes every table allocation
above the limit fail as on a smaller device; the run is a child process so that its tables
are not the test session's."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from narwhal_amd import _lib
from narwhal_amd import messages as M
from oracle import oracle as O
from cert_cases import mutated_stream, votes_case

class Com:
    def __init__(self, p):
        self.p = p
    def packed(self):
        return self.p

L = _lib.lib()
rc = L.nw_prepare()
assert rc == -4, (rc, L.nw_last_error())          # NW_E_OUT_OF_MEMORY, reported cleanly
assert b"keyed B comb" in L.nw_last_error(), L.nw_last_error()
for N in (4, 10):
    com, s, exp_st, exp_ix, cls = mutated_stream(N=N, copies=1, seed=N + 7)
    z16 = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(len(s["vote_pks"]), 16),
                                                           dtype=np.uint8)
    for _ in range(2):                               # twice: no small-job path without tables
        st, ix = M.verify_certificates_many(Com(com), s, z16)
        ost, oix = O.certificates_verify_many(com, s, z16)
        assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist(), N
    st, ix = M.verify_certificates_many(Com(com), s, None)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist()
    hst, hix = M.verify_headers_many(Com(com), s)
    ohst, ohix = O.certificates_verify_many(com, s, headers_only=True)
    assert hst.tolist() == ohst.tolist() and hix.tolist() == ohix.tolist()
vcom, vp, vn, vexp = votes_case(N=8, seed=5, count=64)
assert M.verify_votes_many(Com(vcom), vp).tolist() == vexp.tolist()
small, pipe = _lib.path_stats()
assert small == 0 and pipe > 0, (small, pipe)
print("FALLBACK_OK")
"""


def test_no_room_for_keyed_tables_falls_back_unkeyed():
    """With 3 GB per table allocation the strict tables fit but the keyed B comb does not:
    nw_prepare returns NW_E_OUT_OF_MEMORY with the reason, and every Header / Vote /
    Certificate check still runs (unkeyed: the strict ladder and each certificate's own
    verify_batch), statuses and indices equal to the oracle's."""
    env = dict(os.environ, NW_DEVICE_MEM_LIMIT=str(3 * 10**9))
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + _CHILD], env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and "FALLBACK_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


_CHILD_W16 = r"""
import sys
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
from narwhal_amd import _lib
from narwhal_amd import messages as M
from oracle import oracle as O
from cert_cases import mutated_stream

class Com:
    def __init__(self, p):
        self.p = p
    def packed(self):
        return self.p

for N in (4, 10, 4):
    com, s, exp_st, exp_ix, cls = mutated_stream(N=N, copies=1, seed=N + 7)
    z16 = np.random.Generator(np.random.PCG64(N)).integers(0, 256, size=(len(s["vote_pks"]), 16),
                                                           dtype=np.uint8)
    st, ix = M.verify_certificates_many(Com(com), s, z16)
    ost, oix = O.certificates_verify_many(com, s, z16)
    assert st.tolist() == ost.tolist() and ix.tolist() == oix.tolist(), N
    st, ix = M.verify_certificates_many(Com(com), s, None)
    assert st.tolist() == exp_st.tolist() and ix.tolist() == exp_ix.tolist(), N
print("W16_OK")
"""


def test_no_room_for_20bit_key_combs_uses_16bit():
    """a committee of <= 64 keys prefers 20-bit key combs (940 MB per key). When
    that allocation fails (NW_KEYTAB_LIMIT = 2 GB: 3.8 GB for 4 keys), the keyed checks run
    on 16-bit combs (1.07 GB for 16 keys) instead of the unkeyed fallback; the 16-bit tables
    are then kept for the 10-key and the next 4-key committee (no reallocation per switch).
    Statuses and indices equal the oracle's."""
    env = dict(os.environ, NW_KEYTAB_LIMIT=str(2 * 10**9), NW_KEYTAB_LOG="1")
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + _CHILD_W16], env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and "W16_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
    log = [x for x in r.stderr.splitlines() if x.startswith("[keytab]")]
    assert len(log) == 2, log
    assert "width 20" in log[0] and "FAILED" in log[0], log
    assert "width 16" in log[1] and "-> ok" in log[1], log
