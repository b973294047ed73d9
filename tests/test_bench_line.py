"""bench.py's output contract (the driver left a ~30 KB line unparsed).

CPU: the line assembly over a canned full result (round 4's round-end record) stays under
the driver's size limit, parses, and carries the contract keys, a roofline and a
cpu_baseline; `--gpus N` disagreeing with the launcher's WORLD_SIZE exits non-zero before
any GPU work. GPU: `bench.py --gpus 2` with no launcher starts two ranks itself (gloo,
sharing the box's one GPU) and reports n_gpus 2 with parity ok."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CANNED = os.path.join(ROOT, "profiles", "r04j", "bench_full.json")
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "parity")


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _check_line(line):
    text = json.dumps(line, separators=(",", ":"))
    assert len(text) < 16384, len(text)
    back = json.loads(text)
    for k in CONTRACT:
        assert k in back, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in back["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in back["cpu_baseline"], k
    return back


def test_compact_line_from_round4_record():
    B = _bench()
    full = json.load(open(CANNED))
    assert len(json.dumps(full)) > 16384          # the record the driver could not parse
    full["summary"] = B.summary(full)
    back = _check_line(B.compact_line(full, os.path.join(ROOT, "gpurun_out", "d.json")))
    assert back["value"] == full["value"] and back["parity"] == "ok"
    assert back["detail"] == os.path.join("gpurun_out", "d.json")
    s = back["summary"]
    assert s["batch10k"]["latency_ms"] == round(full["verify_batch_10k"]["latency_ms"], 3)
    assert set(s["cert_stream_Mcerts_s"]) == {"N4", "N10", "N50", "N100"}
    # the service tail is reported with p90 and max, not only the good percentiles, and with
    # the load generator's own lateness and the hedge's host answers beside them
    row = s["service"]["N50"]["offered_achieved_p50_p90_p99_max_lagmax_ms_hostfirst"][0]
    assert len(row) == 8 and row[6] is not None


def test_compact_line_bounded_when_legs_grow():
    B = _bench()
    full = json.load(open(CANNED))
    full["summary"] = B.summary(full)
    # many more committees and rates than the default bench runs
    full["summary"]["service"] = {f"N{n}": full["summary"]["service"]["N50"] for n in range(200)}
    full["summary"]["worker"]["offered_achieved_p50ms_p99ms"] *= 100
    back = _check_line(B.compact_line(full))
    assert "service" not in back["summary"] and back["summary"]["batch10k"]


def test_gpus_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "WORLD_SIZE=2" in p.stderr
    assert p.stdout.strip() == ""


@pytest.mark.gpu
def test_bench_gpus2_spawns_ranks():
    env = dict(os.environ, NW_BENCH_BACKEND="gloo",
               NW_BENCH_DETAIL=os.path.join(ROOT, "gpurun_out", "bench_n2_detail.json"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    # every leg the driver's N > 1 run times (strict, SHA-512, certificates, verify_batch,
    # wire ingest) at toy sizes; the latency legs (service, worker) are per-process
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--items-per-gpu", "65536",
                        "--unique", "8192", "--sha-batches", "256", "--sha-unique", "16",
                        "--certs", "2048", "--cert-unique", "512", "--committees", "4",
                        "--cert-payload-committees", "", "--batch-many", "2",
                        "--wire-frames", "512", "--wire-steps", "1",
                        "--no-worker", "--no-service", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["parity"] == "ok", r
    assert r["config"]["items_total"] == 2 * 65536
    s = r["summary"]
    assert s["sha512"]["GB_s"] > 0 and s["cert_stream_Mcerts_s"]["N4"] > 0
    assert s["batch10k"]["resident_M_s"] > 0 and s["wire_Mcerts_s"] > 0


@pytest.mark.gpu
def test_bench_gpus8_gloo_rehearsal():
    """The driver's 8-GPU run rehearsed by process on the one-GPU box: `bench.py --gpus 8`
    starts 8 ranks (all on device 0 over gloo), each verifies its shard of every timed leg
    (strict, SHA-512, certificates, verify_batch, wire ingest) at toy sizes, and rank 0 checks
    the gathered 8-shard verdict bitmap bit for bit."""
    env = dict(os.environ, NW_BENCH_BACKEND="gloo",
               NW_BENCH_DETAIL=os.path.join(ROOT, "gpurun_out", "bench_n8_detail.json"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    # one 8 x 4096-item corpus, 8 shards; ragged / empty shards: tests/test_distributed.py
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8",
                        "--steps", "2", "--warmup", "1", "--items-per-gpu", "4096",
                        "--unique", "2048", "--sha-batches", "64", "--sha-unique", "8",
                        "--certs", "512", "--cert-unique", "256", "--committees", "4",
                        "--cert-invalid", "0", "--cert-payload-committees", "",
                        "--batch-many", "1", "--wire-frames", "256", "--wire-steps", "1",
                        "--no-worker", "--no-service", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 8 and r["parity"] == "ok", r
    assert r["config"]["items_total"] == 8 * 4096 and r["config"]["parallelism"] == "shard8"
    s = r["summary"]
    assert s["sha512"]["GB_s"] > 0 and s["cert_stream_Mcerts_s"]["N4"] > 0
    assert s["batch10k"]["resident_M_s"] > 0 and s["wire_Mcerts_s"] > 0
