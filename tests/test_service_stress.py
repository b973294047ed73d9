"""The aggregation service's host logic (narwhal_amd/csrc/nw_service.cpp) on the CPU: lock-
free request ingest, batch sealing when full, growth of the next batch, the flusher's
choices and the completer, driven by tools/service_stress.cpp with test doubles in place of
the device entry points (each answers a request with a fingerprint of exactly the bytes
that request supplied, and checks every batch's offsets). Several producer threads submit
random certificates (0 .. 3,000 votes), headers, votes, Signature::verify and verify_batch
requests; every request must get exactly one verdict and it must be its own. One job in 16
is 3 ms late, so the hedge (nw_service_set_hedge: host doubles answering with the same
fingerprints) delivers part of the verdicts, racing the completer for each request. Also
under ThreadSanitizer. No GPU."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(target):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    r = subprocess.run(["make", "-s", target], cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(ROOT, target)


@pytest.mark.parametrize("producers,requests,max_items", [(1, 3000, 64), (4, 8000, 4096),
                                                          (8, 4000, 1 << 20)])
def test_service_stress(producers, requests, max_items):
    exe = _build("tools/service_stress")
    r = subprocess.run([exe, str(producers), str(requests), str(max_items)],
                       capture_output=True, text=True, timeout=300)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0, out
    assert out["accepted"] == producers * requests
    assert out["missing"] == out["duplicate"] == out["wrong"] == out["bad_shape"] == 0
    assert out["hedged"] > 0 and 0 < out["host_first"] <= out["host_calls"]


def test_service_stress_tsan():
    exe = _build("tools/service_stress_tsan")
    # (built with -DNW_SERVICE_SYSTEM_CLOCK_WAIT: this image's libtsan does not intercept the
    # pthread_cond_clockwait that steady-clock waits use, see nw_service.cpp wait_ns)
    r = subprocess.run([exe, "6", "2000", "2048"], capture_output=True, text=True, timeout=600,
                       env={**os.environ, "TSAN_OPTIONS": "halt_on_error=1"})
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
