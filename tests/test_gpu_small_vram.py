"""Job inputs in device memory written by the CPU (nw_jobs.cpp job_reserve_vram): with
NW_SMALL_VRAM=1 the small-job kernel's inputs, with NW_BATCH_VRAM=1 a lone fused
verify_batch's inputs travel as the CPU's writes into host-mapped fine-grained device memory
instead of pinned host memory (read across the bus, or copied by an H2D). The small-job
parity file (tests/test_gpu_small.py: headers, votes, certificates, irregular committees) and
the batch parity file (tests/test_gpu_batch.py: lone batches on both sides of the fused
limit, every failure class) run in child processes against the oracle: small jobs with the
opt-in staging (the library must report it), lone batches with the default staging turned
OFF (NW_BATCH_VRAM=0: the pinned buffer and H2D path keeps its coverage; the default path is
the one tests/test_gpu_batch.py runs in the suite itself), lone batches with the input
gate (NW_BATCH_GATE=1: the kernels queued before the votes are written, chunk flags), and
lone batches that wait for the launch's completion event instead of the tail's done word
(NW_BATCH_SPIN=0; the default spin path is the suite's own), also under the injected
post-launch failure of tests/test_gpu_fused_abort.py; and small jobs that wait for their
completion event instead of their workgroups' done flags (NW_SMALL_DONE=0); and small jobs
whose flag words arrive holding the job's own sequence number (NW_TEST_STALE_FLAGS=1, what a
recycled pinned buffer can hold: the host must clear them before the launch, profiles/r06aa)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NOTICE = "NW_SMALL_VRAM: small jobs' inputs written into host-mapped fine-grained device memory"


GATE = "NW_BATCH_GATE: lone batches launched before their votes are written"
STALE = "NW_TEST_STALE_FLAGS: small-job flag words poisoned"


@pytest.mark.parametrize("env,value,test,notice", [
    ("NW_SMALL_VRAM", "1", "test_gpu_small.py", NOTICE),   # opt-in for small jobs
    ("NW_BATCH_VRAM", "0", "test_gpu_batch.py", None),     # lone batches: on by default
    ("NW_BATCH_GATE", "1", "test_gpu_batch.py", GATE),     # votes written after the launch
    ("NW_BATCH_SPIN", "0", "test_gpu_batch.py", None),     # the completion event only
    ("NW_BATCH_SPIN", "0", "test_gpu_fused_abort.py", None),
    ("NW_SMALL_DONE", "0", "test_gpu_small.py", None),     # small jobs: the event only
    ("NW_TEST_STALE_FLAGS", "1", "test_gpu_small.py", STALE),   # poisoned flag words
])
def test_inputs_in_device_memory(env, value, test, notice):
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-s", "-p",
                        "no:cacheprovider", os.path.join(ROOT, "tests", test)],
                       cwd=ROOT, env=dict(os.environ, **{env: value}), capture_output=True,
                       text=True, timeout=280)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    out = r.stdout + r.stderr
    if notice:
        assert notice in out
    else:
        assert NOTICE not in out and GATE not in out and STALE not in out
