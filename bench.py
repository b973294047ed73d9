#!/usr/bin/env python3
"""bench.py — Narwhal crypto hot path on MI355X: Ed25519 verifies/s (+ SHA-512 GB/s).

    python bench.py [--gpus N --steps K --warmup W --workload strict|sha]

One process per GPU (torch.distributed.run for N > 1; RCCL only for the barrier and the
max-over-ranks timing: the path shards, there is no data-path collective). Inputs are
synthetic, generated on the device with the engine's own keygen/signing kernels, and are
resident in HBM before the timed region; every timed step is one pass of the hot path
over one batch of inputs through the C ABI (nw_dev_*), launched on torch's current
stream so torch.cuda.Event brackets exactly the kernel launches.

Workloads (BASELINE.json configs):
  strict (default)  config 4: mixed corpus, 12.5M items per GPU (100M over 8 GPUs), 10%
                    invalid / non-canonical / small-order. crypto::Signature::verify
                    semantics per item; bitmap checked against the construction.
  sha               config 3: 65,536 worker batches x 508,052 B (977 x 512 B txs,
                    bincode layout), SHA-512 digests; checked against hashlib.
The SHA-512 rate (config 3) is also reported as a secondary field of the strict line.

Roofline work constants are SURVEY.md 8(d) (see DESIGN.md "Measurement").
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from narwhal_amd import _lib                 # noqa: E402
from narwhal_amd import crypto as C          # noqa: E402
from narwhal_amd import messages as M        # noqa: E402
from narwhal_amd import workloads as W       # noqa: E402

METRIC = "Ed25519 verifies/sec (1/2/4/8 MI355X) + SHA-512 GB/s vs dalek on host cores"
L_ORDER = 2**252 + 27742317777372353535851937790883648493
P_FIELD = 2**255 - 19

# implementation-independent work per unit.
MAC_PER_STRICT_VERIFY = 3200 * 64          # 204,800 32x32->64 MACs
MAC_PER_BATCH_ITEM_LARGE = 1000 * 64       # batch item, n >= 10k (64,000 MACs)
MAC_PER_BATCH_ITEM_SMALL = 2000 * 64       # batch item, small n (certificate votes)
# Keyed vote check: 27 table additions (16 from the committee key's 16-bit
# combs, 11 from the 24-bit B comb; ~7.5 F_p mults each) + one product for the y comparison
# + a share of the batched inversion ~ 215 F_p mults, no R decompression; the SURVEY small-n
# constant above describes per-certificate Straus, not this algorithm.
MAC_PER_KEYED_VOTE = 215 * 64              # 13,760 MACs
# Keyed strict verification (Header::verify by a committee key): R's
# decompression (~265 F_p mults) + 27 table additions (~7.5 each) ~ 470 F_p mults;
# SURVEY's 204,800 describes an unkeyed ladder verification.
MAC_PER_KEYED_STRICT = 470 * 64            # 30,080 MACs
SHA_OPS_PER_BLOCK = 4800                   # int32 ops per 128-B block
# Peaks (DESIGN.md "Measurement"): v_mad_u64_u32 issues at half rate on gfx950, so the spec
# MAC peak = 256 CU x 4 SIMD x 16 lanes x 2.4 GHz; the measured one is the microbenchmark's
# v_mad_u64_u32 issue rate at 4 waves/SIMD (profiles/r01_ubench_valu_4wps.txt).
PEAK_TMAC = 256 * 4 * 16 * 2.4e9 / 1e12    # 39.32 TMAC/s (spec)
PEAK_TMAC_MEASURED = 32.39                 # TMAC/s (measured, v_mad_u64_u32)
PEAK_TOPS_FULL = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.64 T int32 lane-ops/s (full-rate ops)
PEAK_HBM_GBS = 8000.0

SMALL_ORDER = [
    "0100000000000000000000000000000000000000000000000000000000000000",
    "ecffffffffffffffffffffffffffffffffffffffffffffffffffffffffffff7f",
    "0000000000000000000000000000000000000000000000000000000000000000",
    "0000000000000000000000000000000000000000000000000000000000000080",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05",
    "26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc85",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a",
    "c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac03fa",
]


def pmc_traffic(kernel: str, units: int):
    """Per-launch HBM bytes of `kernel` from the committed PMC passes (profiles/traffic.json,
    written by tools/profile_summary.py from FETCH_SIZE x 2 + WRITE_SIZE of a bench-size
    launch), scaled to `units` per launch. None when no profile exists for it."""
    try:
        e = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))[kernel]
    except (OSError, KeyError, ValueError):
        return None, None
    return e["hbm_bytes"] * units / e["units"], e["source"]


def cert_traffic(N: int):
    """HBM bytes per vote of one config-2 certificate call at committee size N (the call's
    kernels, FETCH_SIZE x 2 + WRITE_SIZE from tools/pmc_cert.sh, summarised by
    tools/pmc_cert_summary.py into profiles/cert_traffic.json). None when absent."""
    try:
        e = json.load(open(os.path.join(ROOT, "profiles", "cert_traffic.json")))[f"N{N}"]
    except (OSError, KeyError, ValueError):
        return None, None
    return e["hbm_bytes_per_vote"], e["source"]


# Algorithmic HBM bytes of one keyed vote check: the vote's key and signature (96 B) and its
# 27 table entries (affine niels, 128-B slots: 16 from the key's combs, 11 from the B comb).
ALG_BYTES_PER_KEYED_VOTE = 96 + 27 * 128


def pmc_issue_peak():
    """Issue-bound peak of k_verify_strict (verifies/s) from its committed PMC instruction mix
    (the newest of profiles/r06as/pmc_mix.json — round 6's final two-pass launch (r06ap, r06ak before it), k_strict_triage +
    k_verify_strict_pre —, r06m's — the one-pass kernel — and r02d's, written by
    tools/pmc_mix.sh + tools/pmc_strict_json.py): per-verify 64-bit / 32-bit integer and
    other VALU lane-ops, each priced at its microbenchmarked issue rate
    (profiles/r01_ubench_valu_4wps.txt; 32-bit integer ops at the half rate, an upper bound
    on their cost). None when no profile is present."""
    tags = ("r06m", "r02d") if os.environ.get("NW_STRICT_TRIAGE") == "0" else ("r06as", "r06ap", "r06ak", "r06m", "r02d")
    for tag in tags:
        rel = os.path.join("profiles", tag, "pmc_mix.json")
        try:
            m = json.load(open(os.path.join(ROOT, rel)))
        except (OSError, ValueError):
            continue
        return m["issue_peak_verifies_per_s"], rel
    return None, None


# One wave per SIMD (config 3: 65,536 messages = 1,024 waves): a lone wave issues one VALU
# instruction per 4 cycles whatever its rate (MI355X_MICROARCH.md, "one wave alone: 4"), so
# 1,024 SIMDs x 64 lanes / 4 cycles x 2.4 GHz = 39.3 T lane-ops/s; the dependent-chain
# microbenchmark at one wave per SIMD measured 27-30 T (profiles/r01_ubench_valu_1wps.txt:
# alignbit 29.9, bitop3 28.9, lshl_add_u64 27.2 - the SHA-512 kernel's three main ops).
PEAK_TOPS_ONE_WAVE = 256 * 4 * 64 / 4 * 2.4e9 / 1e12
UBENCH_TOPS_ONE_WAVE = (29.85 + 28.94 + 27.17) / 3


def pmc_sha_valu(units: int):
    """VALU lane-ops of one config-3 k_sha512_digest32 launch from the committed PMC pass
    (SQ_INSTS_VALU x 64, profiles/<tag>/pmc.json via profiles/traffic.json), scaled to
    `units` messages. None when absent."""
    try:
        src = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))[
            "k_sha512_digest32"]["source"]
        d = json.load(open(os.path.join(ROOT, src)))
        e = next(v for k, v in d.items() if k.startswith("k_sha512_digest32@grid65536"))
        return e["SQ_INSTS_VALU"] * 64 * units / 65536, src
    except (OSError, KeyError, ValueError, StopIteration):
        return None, None


def enc_y(y: int, sign: int) -> bytes:
    b = bytearray(y.to_bytes(32, "little"))
    b[31] |= sign << 7
    return bytes(b)


def log(msg: str) -> None:
    print(f"[bench r{os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def host_cores() -> dict:
    """CPU threads the baselines may use: the affinity mask (what nproc reports), capped by
    the cgroup CPU quota when one is set (the GPU box grants a CPU share smaller than the
    machine) and by OMP_NUM_THREADS when the environment sets it."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:                                                    # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        try:                                                # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = aff
    for cap in (quota, int(omp) if omp and omp.isdigit() else None):
        if cap:
            threads = min(threads, cap)
    return {"threads": threads, "affinity_cpus": aff, "cgroup_quota_cpus": quota,
            "omp_num_threads": omp}


def oracle_module():
    """The CPU oracle (test infrastructure, used only by the cpu_baseline legs), loaded with
    its OpenMP threads pinned one per core (OMP_PROC_BIND / OMP_PLACES are read when libgomp
    initialises, i.e. on first load)."""
    os.environ.setdefault("OMP_PROC_BIND", "close")
    os.environ.setdefault("OMP_PLACES", "cores")
    from oracle import oracle as O
    return O


def median_rate(fn, units: int, runs: int = 5) -> tuple[float, list[float]]:
    """Median over ``runs`` wall-clock runs of fn() (warm: one untimed run first) as
    units/s; returns (median rate, per-run seconds)."""
    fn()
    secs = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        secs.append(time.perf_counter() - t0)
    return units / float(np.median(secs)), secs


def ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def ptr_np(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: rc={rc} {_lib.lib().nw_last_error().decode()}")


# ------------------------------------------------------------------------ corpus (config 4)
def build_strict_corpus(dev, stream, uniq: int, nkeys: int, seed: int):
    """Unique corpus on the device: keys and signatures by the engine's kernels, then 10%
    of items turned into the Appendix A edge classes on the host (byte edits only).
    Returns device tensors (msgs, pks, sigs) and the expected validity mask."""
    L = _lib.lib()
    rng = np.random.Generator(np.random.PCG64(seed))
    seeds = torch.from_numpy(rng.integers(0, 256, size=(nkeys, 32), dtype=np.uint8)).to(dev)
    pks_k = torch.empty((nkeys, 32), dtype=torch.uint8, device=dev)
    check(L.nw_dev_keypair_from_seed_many(ptr(seeds), nkeys, ptr(pks_k), stream), "keygen")
    sks_k = torch.cat([seeds, pks_k], dim=1).contiguous()
    key_of = torch.from_numpy(rng.integers(0, nkeys, size=uniq)).to(dev)
    sks = sks_k.index_select(0, key_of).contiguous()
    msgs = torch.from_numpy(rng.integers(0, 256, size=(uniq, 32), dtype=np.uint8)).to(dev)
    sigs = torch.empty((uniq, 64), dtype=torch.uint8, device=dev)
    check(L.nw_dev_sign_many(ptr(sks), 64, ptr(msgs), 32, uniq, ptr(sigs), stream), "sign")
    torch.cuda.synchronize()
    m = msgs.cpu().numpy().copy()
    p = sks[:, 32:].cpu().numpy().copy()
    s = sigs.cpu().numpy().copy()
    valid = np.ones(uniq, dtype=bool)
    bad = rng.choice(uniq, uniq // 10, replace=False)
    classes = 12
    for j, i in enumerate(bad):
        c = j % classes
        if c == 0:     # wrong message
            m[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
        elif c == 1:   # bit flip in R
            s[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
        elif c == 2:   # bit flip in s (low 31 bytes: stays < 2^253)
            s[i, 32 + rng.integers(0, 31)] ^= np.uint8(1 << rng.integers(0, 8))
        elif c == 3:   # bit flip in A
            p[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
        elif c == 4:   # s + l (non-canonical scalar)
            v = int.from_bytes(s[i, 32:].tobytes(), "little") + L_ORDER
            s[i, 32:] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
        elif c == 5:   # s with high bits set
            s[i, 63] |= np.uint8(0x80 >> rng.integers(0, 3))
        elif c == 6:   # small-order A (canonical / non-canonical encodings)
            enc = SMALL_ORDER + [enc_y(P_FIELD, 0).hex(), enc_y(P_FIELD + 1, 1).hex(), enc_y(1, 1).hex()]
            p[i] = np.frombuffer(bytes.fromhex(enc[j % len(enc)]), np.uint8)
        elif c == 7:   # small-order R
            s[i, :32] = np.frombuffer(bytes.fromhex(SMALL_ORDER[j % 8]), np.uint8)
        elif c == 8:   # non-canonical large-order A (y = p + t): dalek decodes, no valid sig
            t = [3, 4, 5, 6, 9, 10, 14, 15, 16, 18][j % 10]
            p[i] = np.frombuffer(enc_y(P_FIELD + t, j & 1), np.uint8)
        elif c == 9:   # Signature::default()
            s[i] = 0
        elif c == 10:  # A not on the curve
            p[i] = np.frombuffer(enc_y([2, 7, 8][j % 3], j & 1), np.uint8)
        else:          # R not on the curve
            s[i, :32] = np.frombuffer(enc_y([2, 7, 8][j % 3], j & 1), np.uint8)
        valid[i] = False
    return (torch.from_numpy(m).to(dev), torch.from_numpy(p).to(dev), torch.from_numpy(s).to(dev),
            valid)


def tile(t: torch.Tensor, total: int) -> torch.Tensor:
    reps = (total + t.shape[0] - 1) // t.shape[0]
    return t.repeat((reps,) + (1,) * (t.dim() - 1))[:total].contiguous()


# ------------------------------------------------------------------------ timing helpers
def max_over_ranks(x: float) -> float:
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(launch, steps: int, warmup: int, world: int):
    for _ in range(warmup):
        launch()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record()
        launch()
        e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    if world > 1:
        elapsed = max_over_ranks(elapsed)
    return elapsed, kernel_ms


# ------------------------------------------------------------------------ workloads
def run_strict(args, dev, stream, rank, world):
    """Config 4: ONE global corpus of items_per_gpu x world items (the same seeded unique
    corpus on every rank, item g = unique[g mod U]); rank r verifies its contiguous shard
    (narwhal_amd.shard.shard_range, 64-item aligned) and the verdict bitmaps are gathered
    with one all_gather (RCCL) into the global 100M-bit bitmap, which rank 0 compares bit
    for bit with the construction."""
    from narwhal_amd.shard import gather_bitmaps, shard_range
    L = _lib.lib()
    n_total = args.items_per_gpu * world
    s0, e0 = shard_range(n_total, rank, world)
    n = e0 - s0
    log(f"building corpus: {args.unique} unique items; global {n_total}, shard [{s0}, {e0})")
    msgs_u, pks_u, sigs_u, valid_u = build_strict_corpus(dev, stream, args.unique, 4096, seed=1000)
    idx = torch.arange(s0, e0, dtype=torch.int64, device=dev) % args.unique
    msgs, pks, sigs = (t.index_select(0, idx).contiguous() for t in (msgs_u, pks_u, sigs_u))
    del idx
    status = torch.empty(n, dtype=torch.int32, device=dev)
    bitmap = torch.zeros((n + 63) // 64 * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def launch():
        check(L.nw_dev_verify_strict_many(ptr(msgs), 32, ptr(pks), ptr(sigs), n, ptr(status),
                                          ptr(bitmap), stream), "verify_strict")

    elapsed, kernel_ms = timed_steps(launch, args.steps, args.warmup, world)
    # the exchange step: one gather of every shard's verdict bitmap (ceil(n/8) bytes each)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    words = bitmap.view(torch.int64)
    if world > 1 and dist.get_backend() != "nccl":
        words = words.cpu()
    full = gather_bitmaps(words, n_total, world)
    gather_ms = (time.perf_counter() - t0) * 1e3
    # parity: local statuses vs the construction, then the global bitmap on rank 0
    exp_local = np.resize(valid_u, args.unique)[(np.arange(s0, e0) % args.unique)]
    st = status.cpu().numpy()
    ok = bool(np.array_equal(st == 0, exp_local))
    if rank == 0:
        bits = np.unpackbits(full.cpu().numpy(), bitorder="little")[:n_total].astype(bool)
        ok &= bool(np.array_equal(bits, np.resize(valid_u, n_total)))
    if world > 1:
        t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item() == 1.0)
    del msgs, pks, sigs
    return dict(n=n, n_total=n_total, elapsed=elapsed, kernel_ms=kernel_ms, parity=ok,
                gather_ms=gather_ms, sample=(msgs_u, pks_u, sigs_u, st[: args.unique]))


def run_sha(args, dev, stream, rank, world):
    L = _lib.lib()
    nb = args.sha_batches
    uniq = min(args.sha_unique, nb)
    log(f"building {uniq} unique worker batches ({W.BATCH_BYTES} B), tiled to {nb}")
    ub = np.stack([W.worker_batch(i, seed=rank) for i in range(uniq)])
    expect = [hashlib.sha512(ub[i].tobytes()).digest()[:32] for i in range(uniq)]
    data_u = torch.from_numpy(ub).to(dev)
    data = tile(data_u, nb).view(-1)
    offs = torch.arange(nb, dtype=torch.int64, device=dev) * W.BATCH_BYTES
    lens = torch.full((nb,), W.BATCH_BYTES, dtype=torch.int64, device=dev)
    out = torch.empty((nb, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def launch():
        check(L.nw_dev_sha512_digest32_many(ptr(data), ptr(offs), ptr(lens), nb, ptr(out),
                                            stream), "sha512")

    elapsed, kernel_ms = timed_steps(launch, args.steps, args.warmup, world)
    o = out.cpu().numpy()
    ok = all(o[i].tobytes() == expect[i % uniq] for i in range(0, nb, max(1, nb // 997)))
    ok &= all(o[i].tobytes() == expect[i % uniq] for i in range(uniq))
    del data, data_u
    return dict(n=nb, bytes=nb * W.BATCH_BYTES, elapsed=elapsed, kernel_ms=kernel_ms, parity=ok,
                sample=(ub, expect))


def cpu_baseline_sha(sample, seconds: float):
    """sha2-equivalent SHA-512 on the host cores: the oracle's C restatement
    (oracle/nw_oracle.c, 'port') over the unique config-3 worker batches, one batch per
    thread, passes until about ``seconds``; digests checked against hashlib. OpenSSL's
    SHA-512 (hashlib, one batch per thread) is timed beside it for context."""
    from concurrent.futures import ThreadPoolExecutor
    O = oracle_module()
    ub, expect = sample
    threads = host_cores()["threads"]
    n = len(ub)
    data = np.ascontiguousarray(ub).reshape(-1)
    offs = np.arange(n, dtype=np.uint64) * W.BATCH_BYTES
    lens = np.full(n, W.BATCH_BYTES, dtype=np.uint64)
    t0 = time.perf_counter()
    out = O.sha512_digest32_many(data, offs, lens, nthreads=threads)
    ok = all(out[i].tobytes() == expect[i] for i in range(n))
    passes = 1
    while time.perf_counter() - t0 < seconds:
        O.sha512_digest32_many(data, offs, lens, nthreads=threads)
        passes += 1
    dt = time.perf_counter() - t0
    msgs = [ub[i].tobytes() for i in range(n)]
    t1, op = time.perf_counter(), 0
    with ThreadPoolExecutor(threads) as ex:
        while time.perf_counter() - t1 < seconds / 2:
            list(ex.map(lambda b: hashlib.sha512(b).digest(), msgs))
            op += 1
    dt1 = time.perf_counter() - t1
    return dict(value=passes * n * W.BATCH_BYTES / dt / 1e9, unit="GB/s", cores=threads,
                kind="port", sample=f"{passes} passes over {n} unique {W.BATCH_BYTES}-B worker "
                                    f"batches, oracle sha512_digest32_many, {threads} threads, "
                                    f"{dt:.1f} s",
                openssl_GB_per_s=op * n * W.BATCH_BYTES / dt1 / 1e9,
                parity="ok" if ok else "FAIL")


def cert_stream_for(args, rank, N: int, stream_cache=None, payload: int = 0):
    """65,536 unique honest certificates for committee N (signed on the GPU), cached;
    payload = (digest, worker id) entries per header (SURVEY 8(d) config 2's P = 32 variant:
    +1,152 header bytes, primary/src/messages.rs:70-84)."""
    uniq = min(args.cert_unique, args.certs)
    key = N if payload == 0 else (N, payload)
    if stream_cache is not None and key in stream_cache:
        return stream_cache[key]
    keys = [(bytes(pk), bytes(sd) + bytes(pk)) for sd, pk in
            zip(W.fixture_seeds(N), C.keypair_from_seed_many(W.fixture_seeds(N)))]
    log(f"cert stream N={N} P={payload}: building {uniq} unique certificates, tiled to "
        f"{args.certs}")
    s = W.certificate_stream(uniq, keys, lambda sk, m: C.sign_many(sk, m),
                             lambda d, o: C.sha512_digest32_many(d, o[:-1], np.diff(o)),
                             payload=payload, seed=rank)
    if stream_cache is not None:
        stream_cache[key] = s
    return s


class ResidentCerts:
    """A certificate stream tiled to `n` certificates in HBM with the nw_certificates /
    nw_committee views and the device workspace of nw_dev_certificates_verify_many, plus
    the expected status / index of every certificate (the construction)."""

    def __init__(self, L, dev, s, exp_st_u, exp_ix_u, n, ws=None):
        uniq = len(s["header_offsets"]) - 1
        q = s["q"]
        Lh = int(s["header_offsets"][1])
        reps = (n + uniq - 1) // uniq

        def dev_tile(a, rows):
            t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
            return t.repeat((reps,) + (1,) * (t.dim() - 1))[:rows].contiguous()
        self.T = {"header_bytes": dev_tile(s["header_bytes"].reshape(uniq, Lh), n).view(-1),
                  "ids": dev_tile(s["ids"], n), "header_sigs": dev_tile(s["header_sigs"], n),
                  "vote_pks": dev_tile(s["vote_pks"].reshape(uniq, q * 32), n).view(-1, 32),
                  "vote_sigs": dev_tile(s["vote_sigs"].reshape(uniq, q * 64), n).view(-1, 64),
                  "payload_counts": dev_tile(s["payload_counts"].astype(np.int32), n),
                  "header_offsets": torch.arange(n + 1, dtype=torch.int64, device=dev) * Lh,
                  "vote_offsets": torch.arange(n + 1, dtype=torch.int64, device=dev) * q}
        self.Cm = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev)
                   for k, v in s["committee"].items()}
        nv = n * q
        self.host_vo = np.arange(n + 1, dtype=np.uint64) * q
        self.ws = ws if ws is not None else torch.empty(L.nw_dev_certificates_workspace(n, nv),
                                                        dtype=torch.uint8, device=dev)
        self.st = torch.empty(n, dtype=torch.int32, device=dev)
        self.ix = torch.empty(n, dtype=torch.int64, device=dev)
        P = lambda t: t.data_ptr()
        self.cc = M._CCommittee(len(s["committee"]["stakes"]), P(self.Cm["pks"]),
                                P(self.Cm["stakes"]), P(self.Cm["worker_offsets"]),
                                P(self.Cm["worker_ids"]))
        self.cs = M._CCertificates(n, P(self.T["header_bytes"]), P(self.T["header_offsets"]),
                                   P(self.T["payload_counts"]), P(self.T["ids"]),
                                   P(self.T["header_sigs"]), P(self.T["vote_offsets"]),
                                   P(self.T["vote_pks"]), P(self.T["vote_sigs"]), Lh * n, nv,
                                   self.host_vo.ctypes.data)
        self.exp_st = torch.from_numpy(exp_st_u).to(dev).repeat(reps)[:n]
        self.exp_ix = torch.from_numpy(exp_ix_u.astype(np.int64)).to(dev).repeat(reps)[:n]
        self.L, self.n, self.q = L, n, q

    def launch(self, stream):
        check(self.L.nw_dev_certificates_verify_many(ctypes.byref(self.cc), ctypes.byref(self.cs),
                                                     0, None, None, ptr(self.ws), ptr(self.st),
                                                     ptr(self.ix), stream), "certificates")

    def parity(self) -> bool:
        return bool(torch.equal(self.st, self.exp_st) and torch.equal(self.ix, self.exp_ix))


def run_cert(args, dev, stream, rank, world, N: int, invalid: float = 0.0, stream_cache=None,
             payload: int = 0):
    """Config 2: Certificate::verify stream, committee N, q = 2N/3 + 1 votes per cert.
    65,536 unique certificates (signed on the GPU), tiled to --certs; no dedup/caching.
    invalid > 0: that fraction of the unique certificates (evenly spaced, so every merged
    group holds some) carries one invalid vote (workloads.mutate_votes: equation, s high
    bits, R not on the curve); statuses AND indices are checked against the construction
    for every certificate of the tiled stream."""
    L = _lib.lib()
    s = cert_stream_for(args, rank, N, stream_cache, payload)
    uniq = len(s["header_offsets"]) - 1
    exp_st_u = np.zeros(uniq, np.int32)
    exp_ix_u = np.zeros(uniq, np.uint64)
    if invalid > 0:
        step = max(1, int(round(1 / invalid)))
        s, exp_st_u, exp_ix_u = W.mutate_votes(s, np.arange(step // 2, uniq, step), seed=N)
    q, n = s["q"], args.certs
    rc = ResidentCerts(L, dev, s, exp_st_u, exp_ix_u, n)
    torch.cuda.synchronize()
    elapsed, kernel_ms = timed_steps(lambda: rc.launch(stream), args.cert_steps, 1, world)
    ok = rc.parity()
    sec = elapsed / args.cert_steps
    mac_survey = MAC_PER_STRICT_VERIFY + q * MAC_PER_BATCH_ITEM_SMALL
    mac_keyed = MAC_PER_KEYED_STRICT + q * MAC_PER_KEYED_VOTE
    ach = n * mac_keyed / (kernel_ms * 1e-3) / 1e12
    res = {"committee": N, "quorum": q, "payload_entries": payload,
           "header_bytes": int(s["header_offsets"][1]), "certs_per_gpu": n, "unique_certs": uniq,
           "invalid_fraction": float((exp_st_u != 0).mean()),
           "certs_per_s": n * world / sec, "sig_checks_per_s": n * (q + 1) * world / sec,
           "ms_per_step": sec * 1e3,
           "achieved_TMAC_s": ach, "frac": ach / PEAK_TMAC, "frac_measured": ach / PEAK_TMAC_MEASURED,
           "work_per_cert": f"{mac_keyed} MAC (keyed strict header {MAC_PER_KEYED_STRICT} + q x "
                            f"{MAC_PER_KEYED_VOTE} per keyed vote check: 27 table additions, no "
                            f"R decompression)",
           "roofline": cert_roofline(N, n, q, ach),
           "survey_TMAC_s": n * mac_survey / (kernel_ms * 1e-3) / 1e12,
           "survey_work_note": "SURVEY 8(d) small-n constant (per-certificate Straus, 128,000 "
                               "MAC/vote) overstates the keyed algorithm's work; not a roofline",
           "parity": "ok" if ok else "FAIL",
           "parity_check": "status and index of every certificate == construction"}
    del rc
    torch.cuda.empty_cache()
    return res, (s, exp_st_u, exp_ix_u)


def cert_roofline(N: int, n: int, q: int, ach: float):
    """The certificate call's roofline: VALU-bound (integer field arithmetic), achieved
    keyed-algorithm TMAC/s against the spec MAC peak, with the call's measured HBM traffic
    (committed PMC, per vote x the call's votes) beside its algorithmic bytes."""
    bpv, src = cert_traffic(N)
    votes = n * q
    return {"bound": "valu", "achieved": ach, "peak": PEAK_TMAC, "unit": "TMAC/s",
            "frac": ach / PEAK_TMAC,
            "traffic": bpv * votes if bpv is not None else None,
            "traffic_per_vote": bpv, "traffic_unit": "HBM bytes per call",
            "traffic_source": src,
            "algorithmic_bytes": ALG_BYTES_PER_KEYED_VOTE * votes,
            "algorithmic_bytes_per_vote": ALG_BYTES_PER_KEYED_VOTE}


def run_cert_alternating(args, dev, stream, rank, world, N: int, invalid: float,
                         stream_cache=None):
    """Arrival pattern that alternates honest and invalid calls: the
    all-valid stream and the same stream with `invalid` of its certificates carrying one bad
    vote, both resident, called H, I, H, I, ... on one stream; per-call kernel time by
    events; reported as the worst per-call rate relative to the mean all-valid call. Every
    call's statuses and indices are checked."""
    L = _lib.lib()
    s = cert_stream_for(args, rank, N, stream_cache)
    uniq = len(s["header_offsets"]) - 1
    step = max(1, int(round(1 / invalid)))
    sb, bst, bix = W.mutate_votes(s, np.arange(step // 2, uniq, step), seed=N)
    n = args.certs
    good = ResidentCerts(L, dev, s, np.zeros(uniq, np.int32), np.zeros(uniq, np.uint64), n)
    bad = ResidentCerts(L, dev, sb, bst, bix, n, ws=good.ws)
    torch.cuda.synchronize()
    good.launch(stream)
    bad.launch(stream)
    torch.cuda.synchronize()
    ms = {"good": [], "bad": []}
    ok = True
    for k in range(2 * max(2, args.cert_steps)):
        which = good if k % 2 == 0 else bad
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        which.launch(stream)
        e1.record()
        torch.cuda.synchronize()
        ms["good" if which is good else "bad"].append(e0.elapsed_time(e1))
        ok &= which.parity()
    mean_good = float(np.mean(ms["good"]))
    res = {"committee": N, "pattern": "honest, invalid, honest, invalid, ...",
           "invalid_fraction": float((bst != 0).mean()), "honest_call_ms": ms["good"],
           "invalid_call_ms": ms["bad"],
           "worst_call_vs_all_valid": mean_good / max(ms["good"] + ms["bad"]),
           "certs_per_s": 2 * n * world / ((sum(ms["good"]) + sum(ms["bad"])) * 1e-3 /
                                           len(ms["good"])),
           "parity": "ok" if ok else "FAIL"}
    del good, bad
    torch.cuda.empty_cache()
    return res


def cpu_baseline_cert(sample, N: int, seconds: float):
    """Config 2 on the host cores: Certificate::verify with the
    dalek-equivalent signature checks (oracle/nw_dalek.c: Header::verify strict +
    Signature::verify_batch per certificate, the reference's per-certificate algorithm,
    primary/src/messages.rs:189-215) over a bounded prefix of the same unique stream, all
    threads, pinned, median of 5 runs; statuses and indices compared with the construction
    (= the GPU's)."""
    O = oracle_module()
    s, exp_st, exp_ix = sample
    cores = host_cores()
    T = cores["threads"]

    def prefix(m):
        ho, vo = s["header_offsets"], s["vote_offsets"]
        return {"header_bytes": s["header_bytes"][: int(ho[m])], "header_offsets": ho[: m + 1],
                "payload_counts": s["payload_counts"][:m], "ids": s["ids"][:m],
                "header_sigs": s["header_sigs"][:m], "vote_offsets": vo[: m + 1],
                "vote_pks": s["vote_pks"][: int(vo[m])], "vote_sigs": s["vote_sigs"][: int(vo[m])]}

    m = min(len(exp_st), 256)
    t0 = time.perf_counter()
    O.certificates_verify_many(s["committee"], prefix(m), nthreads=T, engine="dalek")
    per = (time.perf_counter() - t0) / m
    m = int(min(len(exp_st), max(m, seconds / 6 / max(per, 1e-9))))
    p = prefix(m)
    st, ix = O.certificates_verify_many(s["committee"], p, nthreads=T, engine="dalek")
    agree = bool(np.array_equal(st, exp_st[:m]) and np.array_equal(ix, exp_ix[:m]))
    rate, secs = median_rate(lambda: O.certificates_verify_many(s["committee"], p, nthreads=T,
                                                                engine="dalek"), m)
    return {"value": rate, "unit": "certs/s", "cores": T, "kind": "port", "engine": "dalek",
            "host": cores, "pinned": os.environ.get("OMP_PROC_BIND"),
            "sample": f"dalek-equivalent restatement; median of {len(secs)} runs over the first "
                      f"{m} unique N={N} certificates, certificates_verify_many "
                      f"(per-certificate verify_batch), {T} threads",
            "algorithm": O.DALEK_ALGORITHM,
            "run_s": secs, "statuses_match": agree}


def run_batch10k(args, dev, stream, rank, world):
    """Config 1: crypto::Signature::verify_batch over 10,000 (PublicKey, Signature) pairs on
    one digest (SHA-512("Hello, world!")[..32], crypto_tests.rs:55-56), keys = the StdRng
    zero-seed fixture stream. Latency of one call through the host entry point (H2D +
    kernels + D2H), plus device throughput with 64 such batches resident in HBM."""
    L = _lib.lib()
    n = 10_000
    seeds = W.fixture_seeds(n)
    pks = C.keypair_from_seed_many(seeds)
    sks = np.concatenate([seeds, pks], axis=1)
    digest = np.frombuffer(hashlib.sha512(b"Hello, world!").digest()[:32], np.uint8)
    sigs = C.sign_many(sks, digest, shared_digest=True)
    bad = sigs.copy()
    bad[-1] = 0                                    # crypto_tests.rs:110-114: Signature::default()
    idx = ctypes.c_size_t(0)
    # the argument pointers are built once: numpy's .ctypes.data_as costs a few us of Python per
    # argument, which a native caller (crypto::Signature::verify_batch's binding) never pays
    p_dig, p_pks = (a.ctypes.data_as(ctypes.c_void_p) for a in (digest, pks))
    p_sig = {id(a): a.ctypes.data_as(ctypes.c_void_p) for a in (sigs, bad)}
    p_idx = ctypes.byref(idx)
    fn = L.nw_signature_verify_batch

    def call(sg):
        return _lib.check(fn(p_dig, p_pks, p_sig[id(sg)], n, None, p_idx), "verify_batch")
    ok = call(sigs) == 0 and call(bad) != 0
    for _ in range(2):
        call(sigs)
    # median of 50 timed calls (the mean of a few is at the mercy of one slow wake-up)
    times = []
    for _ in range(50):
        t0 = time.perf_counter()
        ok &= call(sigs) == 0
        times.append(time.perf_counter() - t0)
    lat = float(np.median(times))
    lat_mean = float(np.mean(times))
    # throughput: nb independent 10k batches resident on the device
    nb = args.batch_many
    d_pk = torch.from_numpy(pks).to(dev).repeat(nb, 1).contiguous()
    d_sig = torch.from_numpy(sigs).to(dev).repeat(nb, 1).contiguous()
    d_dig = torch.from_numpy(digest).to(dev).repeat(nb).contiguous()
    d_off = torch.arange(nb + 1, dtype=torch.int64, device=dev) * n
    host_off = np.arange(nb + 1, dtype=np.uint64) * n
    # a quarter of the resident batches carry one bad vote: every 8th (from 3) a flipped bit in
    # s (equation failure: status 7, index n), every 8th (from 6) s with a high bit set
    # (Signature::from_bytes failure: status 1 at that vote's index)
    exp_st = np.zeros(nb, np.int32)
    exp_ix = np.zeros(nb, np.int64)
    for b in range(nb):
        if b % 8 == 3:
            j = (b * 997) % n
            d_sig[b * n + j, 32] ^= 1
            exp_st[b], exp_ix[b] = 7, n
        elif b % 8 == 6:
            j = (b * 1237) % n
            d_sig[b * n + j, 63] |= 0x80
            exp_st[b], exp_ix[b] = 1, j
    ws = torch.empty(L.nw_dev_verify_batch_workspace(nb, nb * n), dtype=torch.uint8, device=dev)
    d_st = torch.empty(nb, dtype=torch.int32, device=dev)
    d_fi = torch.empty(nb, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    def launch():
        check(L.nw_dev_verify_batch_many(ptr(d_dig), ptr(d_pk), ptr(d_sig), ptr(d_off),
                                         host_off.ctypes.data_as(ctypes.c_void_p), nb,
                                         nb * n, None, None, ptr(ws), ptr(d_st), ptr(d_fi),
                                         stream),
              "verify_batch_many")
    elapsed, kernel_ms = timed_steps(launch, args.steps, 1, world)
    ok &= bool(np.array_equal(d_st.cpu().numpy(), exp_st) and
               np.array_equal(d_fi.cpu().numpy()[exp_st != 0], exp_ix[exp_st != 0]))
    sec = elapsed / args.steps
    res = {"items": n, "latency_ms": lat * 1e3, "latency_ms_mean": lat_mean * 1e3,
           "latency_stat": "median of 50 calls (the C call; argument pointers built once)", "verifies_per_s_one_call": n / lat,
           "batches_resident": nb, "verifies_per_s_resident": nb * n * world / sec,
           "resident_invalid_batches": int((exp_st != 0).sum()),
           "parity_check": "one-call: valid Ok, Signature::default() Err; resident: status of "
                           "every batch and index of every failing one == construction",
           "achieved_TMAC_s": nb * n * MAC_PER_BATCH_ITEM_LARGE / (kernel_ms * 1e-3) / 1e12,
           "work_per_item": f"{MAC_PER_BATCH_ITEM_LARGE} MAC (SURVEY 8d, n >= 10k)",
           "parity": "ok" if ok else "FAIL"}
    del d_pk, d_sig, ws
    torch.cuda.empty_cache()
    return res, (digest, pks, sigs)


def run_wire(args, dev, stream, rank, world, N: int = 4):
    """received bincode PrimaryMessage::Certificate frames -> native
    decode -> Certificate::verify, through the blocking host entry point
    (nw_primary_messages_verify_wire). Frames/s includes host decode, H2D, kernels, D2H."""
    from narwhal_amd import wire as WI
    L = _lib.lib()
    n = args.wire_frames
    keys = [(bytes(pk), bytes(sd) + bytes(pk)) for sd, pk in
            zip(W.fixture_seeds(N), C.keypair_from_seed_many(W.fixture_seeds(N)))]
    s = W.certificate_stream(n, keys, lambda sk, m: C.sign_many(sk, m),
                             lambda d, o: C.sha512_digest32_many(d, o[:-1], np.diff(o)),
                             seed=100 + rank)
    # 1 % of the certificates carry one invalid vote (as the config-2 invalid leg)
    s, exp_st, exp_ix = W.mutate_votes(s, np.arange(50, n, 100), seed=N + 7)
    data, offs = WI.frames_from_stream(s)
    com = M.committee_struct(s["committee"])
    kind = np.zeros(n, np.int32)
    st = np.zeros(n, np.int32)
    ix = np.zeros(n, np.uint64)

    def call():
        check(L.nw_primary_messages_verify_wire(ctypes.byref(com), M._p(data), M._p(offs), n,
                                                M._p(kind), M._p(st), M._p(ix)), "wire")
    call()
    ok = bool(np.array_equal(st, exp_st) and np.array_equal(ix, exp_ix) and
              (kind == WI.MSG_CERTIFICATE).all())
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.wire_steps):
        call()
    el = time.perf_counter() - t0
    if world > 1:
        el = max_over_ranks(el)
    sec = el / args.wire_steps
    return {"committee": N, "frames_per_call": n, "frame_bytes": int(offs[-1]),
            "certs_per_s": n * world / sec, "ms_per_call": sec * 1e3,
            "path": "host frames -> nw_primary_messages_verify_wire (decode + H2D + kernels + D2H)",
            "invalid_fraction": float((exp_st != 0).mean()),
            "parity": "ok" if ok else "FAIL",
            "parity_check": "status and index of every frame's certificate == construction"}


def cgroup_cpu_stat():
    """usage_usec / nr_throttled / throttled_usec of this process's cgroup (v2), or None."""
    try:
        rel = [ln[3:] for ln in open("/proc/self/cgroup").read().split("\n") if ln.startswith("0::")]
    except OSError:
        rel = []
    for path in [os.path.join("/sys/fs/cgroup", r.lstrip("/"), "cpu.stat") for r in rel] + \
            ["/sys/fs/cgroup/cpu.stat"]:
        try:
            with open(path) as f:
                st = dict(line.split()[:2] for line in f if line.strip())
            return {k: int(st[k]) for k in ("usage_usec", "nr_throttled", "throttled_usec")}
        except (OSError, KeyError, ValueError):
            continue
    return None


def loadgen_lib():
    """tools/libnw_loadgen.so (bench tooling over the public C ABI, tools/nw_loadgen.cpp)."""
    path = os.path.join(ROOT, "tools", "libnw_loadgen.so")
    L = ctypes.CDLL(path)
    P = ctypes.c_void_p
    L.nw_loadgen_certificates.argtypes = [P, P, P, P, ctypes.c_double, ctypes.c_uint64,
                                          ctypes.c_size_t, ctypes.c_uint32, ctypes.c_size_t,
                                          ctypes.c_uint32, P, P]
    L.nw_loadgen_certificates.restype = ctypes.c_int
    L.nw_loadgen_certificates_on.argtypes = [P, P, P, P, ctypes.c_double, ctypes.c_uint64,
                                             ctypes.c_uint32, P, P]
    L.nw_loadgen_certificates_on.restype = ctypes.c_int
    return L


def run_service_latency(args, rank, world, N: int, cache=None):
    """the primary's Core::sanitize_certificate calls
    Certificate::verify one certificate at a time (primary/src/core.rs:338-346). Single
    certificates arrive at a fixed offered rate (1k .. 1M per second, open loop) and go
    through the library's native aggregation service (nw_service_certificate: coalesced per
    max_delay / max_items into nw_submit_certificates_verify_many jobs, verdicts by
    callback), driven by tools/nw_loadgen.cpp from `producers` threads, as a Rust crate's
    tokio tasks would call it; latency = verdict time - scheduled arrival time, per
    certificate. Beside it, the asyncio front end (narwhal_amd/service.py NativeService) at
    the rates Python itself can issue. 1 % of the certificates carry one invalid vote; every
    (status, index) is checked against the construction. CPU reference point: the oracle's
    single-certificate Certificate::verify latency and rate on 1 thread (the reference
    verifies inline on the single Core task)."""
    import asyncio
    from narwhal_amd import service as SV
    from narwhal_amd.messages import certificates_struct, committee_struct
    uniq = args.service_unique
    keys = [(bytes(pk), bytes(sd) + bytes(pk)) for sd, pk in
            zip(W.fixture_seeds(N), C.keypair_from_seed_many(W.fixture_seeds(N)))]
    s = W.certificate_stream(uniq, keys, lambda sk, m: C.sign_many(sk, m),
                             lambda d, o: C.sha512_digest32_many(d, o[:-1], np.diff(o)),
                             seed=300 + rank)
    s, exp_st, exp_ix = W.mutate_votes(s, np.arange(50, uniq, 100), seed=N + 11)
    exp_st = np.ascontiguousarray(exp_st, np.int32)
    exp_ix = np.ascontiguousarray(exp_ix, np.uint64)
    hb, ho, vo = s["header_bytes"].tobytes(), s["header_offsets"], s["vote_offsets"]
    LG = loadgen_lib()
    cc, cs = committee_struct(s["committee"]), certificates_struct(s, uniq)
    delay_us = int(args.service_delay * 1e6)
    # the service's hedge (nw_service_set_hedge), read by nw_service_create in the loadgen
    os.environ["NW_SERVICE_HEDGE_US"] = str(args.service_hedge_us)
    os.environ["NW_SERVICE_HEDGE_THREADS"] = str(args.service_hedge_threads)
    os.environ["NW_SERVICE_HEDGE_QUEUED"] = str(args.service_hedge_queued)

    def native_load(rate: float, seconds: float):
        total = max(1, int(rate * seconds))
        lat = np.zeros(total)
        out3 = np.zeros(16)
        cg0, t_cg0 = cgroup_cpu_stat(), time.perf_counter()
        rc = LG.nw_loadgen_certificates(ctypes.byref(cc), ctypes.byref(cs), ptr_np(exp_st),
                                        ptr_np(exp_ix), rate, total, args.service_max_items,
                                        delay_us, args.service_inflight, args.service_producers,
                                        ptr_np(lat), ptr_np(out3))
        cg1, t_cg1 = cgroup_cpu_stat(), time.perf_counter()
        check(rc, "nw_loadgen_certificates")
        el, jobs, bad = float(out3[0]), int(out3[1]), int(out3[2])
        # the process's cgroup over the load: CFS quota throttling stalls every thread of it
        cg = ({"cgroup_cpus_used": (cg1["usage_usec"] - cg0["usage_usec"]) / 1e6 / (t_cg1 - t_cg0),
               "cgroup_throttled_periods": cg1["nr_throttled"] - cg0["nr_throttled"],
               "cgroup_throttled_ms": (cg1["throttled_usec"] - cg0["throttled_usec"]) / 1e3}
              if cg0 and cg1 else {})
        lag = {"producer_lag_max_ms": float(out3[3] * 1e3),
               "producer_lag_mean_ms": float(out3[4] * 1e3),
               "producer_cpu_per_wall": float(out3[5]), "producer_vcsw": int(out3[6]),
               "producer_ivcsw": int(out3[7]), "call_mean_us": float(out3[8] * 1e6),
               "call_max_us": float(out3[9] * 1e6), "calls_over_20us": int(out3[10]),
               "small_jobs": int(out3[11]), "pipeline_jobs": int(out3[12]),
               "hedged": int(out3[13]), "host_first": int(out3[14]),
               "host_only_batches": int(out3[15])}
        inval = exp_st[np.arange(total) % uniq] != 0
        slow = np.argsort(lat)[-max(1, total // 100):]   # the slowest 1 %: where in the run
        diag = {"p99_valid_ms": float(np.percentile(lat[~inval], 99) * 1e3),
                "p99_invalid_ms": float(np.percentile(lat[inval], 99) * 1e3) if inval.any() else None,
                "slowest1pct_in_first_tenth": float(np.mean(slow < total // 10)),
                "slowest1pct_invalid_frac": float(np.mean(inval[slow]))}
        return {**diag, **lag, **cg, "offered_certs_per_s": rate, "certs": total,
                "achieved_certs_per_s": total / el if el > 0 else None,
                "p50_ms": float(np.percentile(lat, 50) * 1e3),
                "p90_ms": float(np.percentile(lat, 90) * 1e3),
                "p99_ms": float(np.percentile(lat, 99) * 1e3),
                "max_ms": float(lat.max() * 1e3), "jobs": jobs,
                "certs_per_job": total / max(1, jobs),
                "parity": "ok" if bad == 0 else f"FAIL ({bad} verdicts differ)"}

    rows = [SV.CertRow(hb[int(ho[i]):int(ho[i + 1])], int(s["payload_counts"][i]),
                       s["ids"][i].tobytes(), s["header_sigs"][i].tobytes(),
                       s["vote_pks"][int(vo[i]):int(vo[i + 1])].tobytes(),
                       s["vote_sigs"][int(vo[i]):int(vo[i + 1])].tobytes(),
                       int(vo[i + 1] - vo[i])) for i in range(uniq)]
    expect = [(int(a), int(b)) for a, b in zip(exp_st, exp_ix)]

    async def asyncio_load(rate: float, seconds: float):
        svc = SV.NativeService(s["committee"], max_items=args.service_max_items,
                               max_delay=args.service_delay, max_inflight=args.service_inflight)
        loop = asyncio.get_running_loop()
        total = max(1, int(rate * seconds))
        lat = np.zeros(total)
        bad = [0]
        bad_first = []   # (request, got, expected) of the first mismatches
        done = loop.create_future()
        left = [total]

        def make_cb(i, t_arr):
            def cb(f):
                lat[i] = loop.time() - t_arr
                if f.result() != expect[i % uniq]:
                    bad[0] += 1
                    if len(bad_first) < 10:
                        bad_first.append([i, list(f.result()), list(expect[i % uniq])])
                left[0] -= 1
                if left[0] == 0:
                    done.set_result(None)
            return cb
        await asyncio.gather(*[svc.certificate_status(rows[i]) for i in range(64)])   # warm
        jobs0 = svc.stats()[1]
        t0 = loop.time()
        i = 0
        while i < total:
            now = loop.time()
            while i < total and t0 + i / rate <= now:
                (lp, fut), f = svc._future()
                svc.submit_certificate(rows[i % uniq], (lp, fut))
                f.add_done_callback(make_cb(i, t0 + i / rate))
                i += 1
            await asyncio.sleep(min(0.0002, max(0.0, t0 + i / rate - loop.time())))
        await done
        el = loop.time() - t0
        jobs = svc.stats()[1] - jobs0
        svc.close()
        return {"offered_certs_per_s": rate, "certs": total, "achieved_certs_per_s": total / el,
                "p50_ms": float(np.percentile(lat, 50) * 1e3),
                "p99_ms": float(np.percentile(lat, 99) * 1e3),
                "max_ms": float(lat.max() * 1e3), "jobs": jobs,
                "certs_per_job": total / max(1, jobs),
                "parity": "ok" if bad[0] == 0 else "FAIL",
                **({"mismatches": bad[0], "first_mismatches": bad_first} if bad[0] else {})}

    rates = [float(x) for x in args.service_rates.split(",") if x]
    loads = [native_load(r, min(args.service_seconds, args.service_max_certs / r)) for r in rates]
    py_loads = [asyncio.run(asyncio_load(r, min(args.service_seconds, 20_000 / r)))
                for r in (1_000.0, 10_000.0)]
    res = {"committee": N, "quorum": int(W.quorum(N)), "max_delay_ms": args.service_delay * 1e3,
           "hedge_us": args.service_hedge_us, "hedge_threads": args.service_hedge_threads,
           "hedge_max_queued": args.service_hedge_queued,
           "max_items": args.service_max_items, "max_inflight": args.service_inflight,
           "producers": args.service_producers,
           "invalid_fraction": float((exp_st != 0).mean()), "loads": loads,
           "path": "nw_service_certificate (native aggregation, tools/nw_loadgen.cpp producers) "
                   "-> nw_submit_certificates_verify_many jobs -> verdict callbacks",
           "python_asyncio": {"path": "asyncio NativeService.submit_certificate -> "
                                      "nw_service_certificate, futures resolved by callback",
                              "loads": py_loads},
           "parity": "ok" if all(x["parity"] == "ok" for x in loads + py_loads) else "FAIL"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        O = oracle_module()

        def prefix(a, m):
            return {"header_bytes": s["header_bytes"][int(ho[a]):int(ho[m])],
                    "header_offsets": ho[a:m + 1] - ho[a], "payload_counts": s["payload_counts"][a:m],
                    "ids": s["ids"][a:m], "header_sigs": s["header_sigs"][a:m],
                    "vote_offsets": vo[a:m + 1] - vo[a],
                    "vote_pks": s["vote_pks"][int(vo[a]):int(vo[m])],
                    "vote_sigs": s["vote_sigs"][int(vo[a]):int(vo[m])]}
        singles = [prefix(i, i + 1) for i in range(200)]
        for p1 in singles[:5]:
            O.certificates_verify_many(s["committee"], p1, nthreads=1, engine="dalek")
        secs = []
        for p1 in singles:
            t = time.perf_counter()
            O.certificates_verify_many(s["committee"], p1, nthreads=1, engine="dalek")
            secs.append(time.perf_counter() - t)
        res["cpu_oracle_one_thread"] = {
            "p50_ms": float(np.percentile(secs, 50) * 1e3),
            "p99_ms": float(np.percentile(secs, 99) * 1e3),
            "certs_per_s": 1.0 / float(np.mean(secs)), "cores": 1, "kind": "port",
            "engine": "dalek",
            "sample": "dalek-equivalent restatement; 200 single Certificate::verify calls "
                      "(certificates_verify_many, 1 thread, per-certificate verify_batch as the "
                      "reference)"}
    return res


def run_worker_latency(args, rank, world):
    """the worker Processor (worker/src/processor.rs:36-54, here
    narwhal_amd/worker.py over the aggregating VerificationService) hashing 508,052-B batches
    that arrive at a fixed offered rate (open loop; latency = the digest message's arrival on
    tx_digest - the batch's scheduled arrival), next to the host's SHA-512 on the same batches
    (OpenSSL via hashlib = sha2-equivalent: one batch on 1 thread; 16 batches at once on 16
    threads). A GPU digest is one lane walking the batch's ~3,970 blocks, so a
    lone batch takes ~30 ms against ~0.35 ms on one core: the GPU path loses on latency at
    every rate and on throughput unless hundreds of batches are in flight (the --worker-deep
    load)."""
    import asyncio
    from concurrent.futures import ThreadPoolExecutor
    from narwhal_amd import service as SV
    from narwhal_amd import worker as WK
    uniq = 32
    ub = [W.worker_batch(i, seed=11 + rank).tobytes() for i in range(uniq)]
    expect = [hashlib.sha512(b).digest()[:32] for b in ub]

    async def load(rate: float, total: int, lookahead: int, hash_on: str = "device"):
        svc = SV.VerificationService(max_delay=args.worker_delay)
        store, rx, tx = WK.Store(), asyncio.Queue(), asyncio.Queue()
        task = WK.Processor.spawn(0, store, rx, tx, True, svc, max_in_flight=lookahead,
                                  hash_on=hash_on)
        loop = asyncio.get_running_loop()
        for i in range(4):                                   # warm: pool, first job
            await rx.put(ub[i])
            await tx.get()
        jobs0 = svc.jobs_submitted
        due, lat, bad = [], [], [0]

        async def produce():
            t0 = loop.time() + 0.002
            for i in range(total):
                d = t0 + i / rate - loop.time()
                if d > 0:
                    await asyncio.sleep(d)
                due.append(t0 + i / rate)
                await rx.put(ub[i % uniq])
            await rx.put(None)

        async def consume():
            for i in range(total):
                msg = await tx.get()
                lat.append(loop.time() - due[i])
                if msg[4:36] != expect[i % uniq]:
                    bad[0] += 1
        t_start = loop.time()
        await asyncio.gather(produce(), consume(), task)
        el = loop.time() - t_start
        a = np.array(lat) * 1e3
        return {"hash_on": hash_on, "offered_batches_per_s": rate, "batches": total,
                "lookahead": lookahead, "achieved_batches_per_s": total / el,
                "p50_ms": float(np.percentile(a, 50)), "p99_ms": float(np.percentile(a, 99)),
                "max_ms": float(a.max()), "jobs": svc.jobs_submitted - jobs0,
                "batches_per_job": total / max(1, svc.jobs_submitted - jobs0),
                "parity": "ok" if bad[0] == 0 else f"FAIL ({bad[0]} digests differ)"}

    rates = [float(x) for x in args.worker_rates.split(",") if x]
    plan = [(r, WK.Processor.MAX_IN_FLIGHT) for r in rates]
    # the GPU's capacity needs hundreds of batches in flight (one lane per batch): one load
    # with a deep lookahead shows the throughput the device can take, at its latency
    for x in args.worker_deep.split(","):
        if x:
            r, la = x.split(":")
            plan.append((float(r), int(la)))
    def count(r):
        return max(20, int(min(args.worker_seconds, args.worker_max_batches / r) * r))
    loads = [asyncio.run(load(r, count(r), la)) for r, la in plan]
    # the shipped default (Processor hash_on="host", as processor.rs:38): one batch at a time
    # on the event loop's thread
    host = [asyncio.run(load(float(x), count(float(x)), 1, "host"))
            for x in args.worker_host_rates.split(",") if x]
    res = {"batch_bytes": W.BATCH_BYTES, "max_delay_ms": args.worker_delay * 1e3, "loads": loads,
           "host_loads": host,
           "path": "worker.Processor(hash_on='device') -> VerificationService.digest -> "
                   "nw_submit_sha512_digest32_many (one lane per batch); host_loads: the "
                   "default hash_on='host' (hashlib on the loop thread)",
           "parity": "ok" if all(x["parity"] == "ok" for x in loads + host) else "FAIL"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        one = []
        for i in range(100):
            t = time.perf_counter()
            hashlib.sha512(ub[i % uniq]).digest()
            one.append(time.perf_counter() - t)
        T = 16

        def timed(b):
            t = time.perf_counter()
            hashlib.sha512(b).digest()
            return time.perf_counter() - t
        with ThreadPoolExecutor(T) as ex:
            list(ex.map(timed, ub[:T]))
            per, t0, n = [], time.perf_counter(), 0
            while time.perf_counter() - t0 < 1.0:
                per += list(ex.map(timed, ub[:T]))
                n += T
            dt = time.perf_counter() - t0
        res["cpu_sha2_equivalent"] = {
            "one_thread_p50_ms": float(np.percentile(one, 50) * 1e3),
            "one_thread_p99_ms": float(np.percentile(one, 99) * 1e3),
            "threads16_batch_p50_ms": float(np.percentile(per, 50) * 1e3),
            "threads16_batches_per_s": n / dt, "kind": "OpenSSL SHA-512 (hashlib)",
            "sample": "100 single batches on 1 thread; 16 batches at a time on 16 threads for 1 s"}
    return res


def cpu_baseline_batch(sample, seconds: float):
    """Config 1 on the host: the dalek-equivalent verify_batch
    (oracle/nw_dalek.c: Pippenger w = 8 over 20,001 points, crypto/src/lib.rs:206-219) on
    the same 10k batch --
    1 thread (dalek's verify_batch is single-threaded; one call = one batch) and all threads
    with one 10k batch per thread concurrently; pinned; median of 5 runs each."""
    O = oracle_module()
    digest, pks, sigs = sample
    cores = host_cores()
    T = cores["threads"]
    st, _ = O.verify_batch(digest.tobytes(), pks, sigs, engine="dalek")
    assert st == 0
    n = len(pks)
    r1, s1 = median_rate(lambda: O.verify_batch(digest.tobytes(), pks, sigs, engine="dalek"), n)
    dg = np.tile(digest, (T, 1))
    pk_t, sg_t = np.tile(pks, (T, 1)), np.tile(sigs, (T, 1))
    off = (np.arange(T + 1) * n).astype(np.uint64)
    stT = O.verify_batch_many(dg, pk_t, sg_t, off, nthreads=T, engine="dalek")
    assert (stT == 0).all()
    rT, sT = median_rate(lambda: O.verify_batch_many(dg, pk_t, sg_t, off, nthreads=T,
                                                     engine="dalek"), T * n)
    return {"value": rT, "unit": "verifies/s", "cores": T, "kind": "port", "engine": "dalek",
            "host": cores, "pinned": os.environ.get("OMP_PROC_BIND"),
            "sample": f"dalek-equivalent restatement; median of 5 runs: {T} concurrent "
                      f"verify_batch calls over the 10k config-1 batch (one per thread), "
                      f"verify_batch_many", "algorithm": O.DALEK_ALGORITHM,
            "run_s": sT, "one_thread": {"value": r1, "unit": "verifies/s", "cores": 1,
                                        "sample": "median of 5 single verify_batch calls "
                                                  "(one 10k batch, 1 thread)", "run_s": s1}}


def cpu_baseline_strict(sample, seconds: float):
    """The dalek-equivalent restatement ('port', oracle/nw_dalek.c: ed25519-dalek 1.0.1
    verify_strict's NAF-5 / affine NAF-8 double-base chain over curve25519-dalek's u64
    field) on the host cores, pinned, bounded: a prefix of the unique corpus sized to
    ~seconds/6 per run, median of 5 runs; the prefix's statuses are compared with the
    GPU's."""
    O = oracle_module()
    msgs_u, pks_u, sigs_u, gpu_st = sample
    cores = host_cores()
    T = cores["threads"]
    m, p, s = (t.cpu().numpy() for t in (msgs_u, pks_u, sigs_u))
    k = min(len(m), 4096)
    t0 = time.perf_counter()
    O.verify_strict_many(m[:k], p[:k], s[:k], nthreads=T, engine="dalek")
    per = (time.perf_counter() - t0) / k
    k = int(min(len(m), max(k, seconds / 6 / max(per, 1e-9))))
    m, p, s = m[:k], p[:k], s[:k]
    st = O.verify_strict_many(m, p, s, nthreads=T, engine="dalek")
    agree = bool(np.array_equal(st, gpu_st[:k]))
    rate, secs = median_rate(lambda: O.verify_strict_many(m, p, s, nthreads=T, engine="dalek"), k)
    # the checker (nw_oracle.c, fixed 4-bit windows) on the same prefix, for the record
    kc = min(k, 16384)
    rc, _ = median_rate(lambda: O.verify_strict_many(m[:kc], p[:kc], s[:kc], nthreads=T), kc, runs=3)
    return dict(value=rate, unit="verifies/s", cores=T, kind="port", engine="dalek", host=cores,
                pinned=os.environ.get("OMP_PROC_BIND"),
                sample=f"dalek-equivalent restatement (NAF-5 A / affine NAF-8 B double-base); "
                       f"median of {len(secs)} runs over the first {k} items of the unique mixed "
                       f"corpus, verify_strict_many, {T} threads, statuses == GPU's",
                algorithm=O.DALEK_ALGORITHM, statuses_match=agree, checker_value=rc,
                run_s=secs), agree


def summary(r: dict) -> dict:
    """Compact digest of every leg, printed LAST in the JSON line (the driver keeps the
    line's tail): headline, SHA-512, config 2 per committee (all-valid and 1 % invalid),
    config 1, wire ingest and the certificate service's latency."""
    def g(d, *ks):
        for k in ks:
            if not isinstance(d, dict) or k not in d:
                return None
            d = d[k]
        return d

    def rnd(x, n=3):
        return None if x is None else round(float(x), n)
    out = {"value": rnd(r.get("value"), 0), "unit": r.get("unit"), "parity": r.get("parity"),
           "roofline_frac": rnd(g(r, "roofline", "frac")),
           "issue_frac": rnd(g(r, "roofline", "issue_frac")),
           "cpu_baseline": rnd(g(r, "cpu_baseline", "value"), 0)}
    if "sha512" in r:
        out["sha512"] = {"GB_s": rnd(g(r, "sha512", "GB_per_s"), 1),
                         "hbm_frac": rnd(g(r, "sha512", "hbm_frac")),
                         "issue_frac": rnd(g(r, "sha512", "issue_frac")),
                         "cpu_GB_s": rnd(g(r, "sha512", "cpu_baseline", "value"), 2)}
    for leg in ("cert_stream", "cert_stream_invalid", "cert_stream_p32"):
        if r.get(leg):
            out[leg + "_Mcerts_s"] = {k: rnd(v.get("certs_per_s", 0) / 1e6, 2)
                                      for k, v in r[leg].items()}
    if r.get("cert_stream_invalid"):
        out["cert_invalid_vs_all_valid"] = {k: rnd(v.get("vs_all_valid"))
                                            for k, v in r["cert_stream_invalid"].items()}
    if r.get("cert_stream_alternating"):
        out["cert_alternating_worst_vs_all_valid"] = {
            k: rnd(v.get("worst_call_vs_all_valid")) for k, v in r["cert_stream_alternating"].items()}
    if r.get("cert_stream"):
        out["cert_cpu_certs_s"] = {k: rnd(g(v, "cpu_baseline", "value"), 0)
                                   for k, v in r["cert_stream"].items()}
    if "verify_batch_10k" in r:
        b = r["verify_batch_10k"]
        out["batch10k"] = {"latency_ms": rnd(b.get("latency_ms")),
                           "resident_M_s": rnd(b.get("verifies_per_s_resident", 0) / 1e6, 1),
                           "cpu_1thread_k_s": rnd(g(b, "cpu_baseline", "one_thread", "value")
                                                  and g(b, "cpu_baseline", "one_thread", "value") / 1e3, 1)}
    if "wire_ingest" in r:
        out["wire_Mcerts_s"] = rnd(r["wire_ingest"].get("certs_per_s", 0) / 1e6, 2)
    if r.get("worker_latency"):
        wl = r["worker_latency"]
        out["worker"] = {"offered_achieved_p50ms_p99ms": [
                             [int(x["offered_batches_per_s"]), int(x["achieved_batches_per_s"]),
                              rnd(x["p50_ms"], 2), rnd(x["p99_ms"], 2)] for x in wl["loads"]],
                         "host_default": [
                             [int(x["offered_batches_per_s"]), int(x["achieved_batches_per_s"]),
                              rnd(x["p50_ms"], 3), rnd(x["p99_ms"], 3)]
                             for x in wl.get("host_loads", [])],
                         "cpu_1thread_ms": rnd(g(wl, "cpu_sha2_equivalent", "one_thread_p50_ms"), 3),
                         "cpu16_batches_s": rnd(g(wl, "cpu_sha2_equivalent",
                                                  "threads16_batches_per_s"), 0)}
    if r.get("service_latency"):
        # per offered rate: achieved, latency percentiles, the load generator's own lateness
        # (producer_lag_max_ms: a producer preempted off-schedule shows here, not as a service
        # stall) and the requests the hedge's host threads answered first
        out["service"] = {k: {"offered_achieved_p50_p90_p99_max_lagmax_ms_hostfirst": [
                                  [int(x["offered_certs_per_s"]),
                                   int(x["achieved_certs_per_s"] or 0), rnd(x["p50_ms"], 2),
                                   rnd(x.get("p90_ms"), 2), rnd(x["p99_ms"], 2),
                                   rnd(x["max_ms"], 2), rnd(x.get("producer_lag_max_ms"), 2),
                                   x.get("host_first")] for x in v["loads"]],
                              "hedge_us": v.get("hedge_us"),
                              "cpu_1cert_ms": rnd(g(v, "cpu_oracle_one_thread", "p50_ms"), 2)}
                          for k, v in r["service_latency"].items()}
    return out


# The driver parses bench.py's last stdout line; round 4's ~30 KB line was not parsed, so the
# line is kept well below this and the per-leg detail goes to a side file.
LINE_LIMIT = 16384
LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
             "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "parity")
ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_unit",
                 "traffic_source", "algorithmic_bytes", "kernel", "kernel_ms", "work_per_unit",
                 "peak_measured", "frac_measured", "issue_peak", "issue_frac")
CPU_KEYS = ("value", "unit", "cores", "kind", "engine", "sample")


def compact_line(result: dict, detail_path: str | None = None) -> dict:
    """The one JSON object printed on stdout: the contract's keys, a trimmed roofline and
    cpu_baseline, and the summary of every other leg; everything else lives in the detail
    file. Optional parts are dropped (least important first) if the line would not fit."""
    line = {k: result[k] for k in LINE_KEYS if k in result}
    if isinstance(result.get("roofline"), dict):
        line["roofline"] = {k: result["roofline"][k] for k in ROOFLINE_KEYS
                            if k in result["roofline"]}
    if isinstance(result.get("cpu_baseline"), dict):
        line["cpu_baseline"] = {k: result["cpu_baseline"][k] for k in CPU_KEYS
                                if k in result["cpu_baseline"]}
    if "summary" in result:
        line["summary"] = dict(result["summary"])
    if detail_path:
        line["detail"] = os.path.relpath(detail_path, ROOT)
    for drop in ("worker", "service", "cert_alternating_worst_vs_all_valid",
                 "cert_cpu_certs_s", "cert_stream_p32_Mcerts_s"):
        if len(json.dumps(line, separators=(",", ":"))) < LINE_LIMIT // 2:
            break
        line.get("summary", {}).pop(drop, None)
    return line


def write_detail(result: dict) -> str | None:
    """Every leg's full record (NW_BENCH_DETAIL, default gpurun_out/bench_detail.json)."""
    path = os.environ.get("NW_BENCH_DETAIL", os.path.join(ROOT, "gpurun_out", "bench_detail.json"))
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(result, f)
        return path
    except OSError as e:
        log(f"could not write {path}: {e}")
        return None


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks (one per GPU) as the driver's
    torch.distributed.run command would, as a child process of this one (this process never
    touches a GPU), and return its exit code. Rank 0's JSON line reaches stdout unchanged."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["strict", "sha", "cert", "batch", "service", "worker"],
                    default="strict")
    ap.add_argument("--items-per-gpu", type=int, default=12_500_000)
    ap.add_argument("--unique", type=int, default=1 << 18)
    ap.add_argument("--sha-batches", type=int, default=65536)
    ap.add_argument("--sha-unique", type=int, default=256)
    ap.add_argument("--no-sha", action="store_true", help="skip the secondary SHA-512 leg")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--certs", type=int, default=1_000_000)
    ap.add_argument("--cert-unique", type=int, default=65536)
    ap.add_argument("--cert-steps", type=int, default=4)
    ap.add_argument("--cert-invalid", type=float, default=0.01,
                    help="extra config-2 leg with this fraction of certificates carrying a bad "
                         "vote (0 = skip)")
    ap.add_argument("--committees", default="4,10,50,100")
    ap.add_argument("--cert-payload", type=int, default=32,
                    help="payload entries per header of the config-2 P variant")
    ap.add_argument("--cert-payload-committees", default="4,100",
                    help="committees of the P variant leg (empty = skip)")
    ap.add_argument("--no-cert", action="store_true", help="skip the config-2 certificate leg")
    ap.add_argument("--no-batch", action="store_true", help="skip the config-1 verify_batch leg")
    ap.add_argument("--batch-many", type=int, default=64)
    ap.add_argument("--no-wire", action="store_true", help="skip the wire-ingest leg")
    ap.add_argument("--wire-frames", type=int, default=65536)
    ap.add_argument("--wire-steps", type=int, default=3)
    ap.add_argument("--no-service", action="store_true",
                    help="skip the certificate service latency leg")
    ap.add_argument("--service-committees", default="4,50")
    ap.add_argument("--service-unique", type=int, default=8192)
    ap.add_argument("--service-seconds", type=float, default=1.0)
    ap.add_argument("--service-rates", default="1000,10000,100000,1000000")
    ap.add_argument("--service-max-certs", type=float, default=400_000,
                    help="certificates per offered-load run at most (runs shorter than "
                         "--service-seconds at high rates)")
    ap.add_argument("--service-max-items", type=int, default=1 << 20)
    ap.add_argument("--service-inflight", type=int, default=4)
    ap.add_argument("--service-producers", type=int, default=4)
    ap.add_argument("--service-delay", type=float, default=0.0005,
                    help="VerificationService max_delay (s)")
    ap.add_argument("--service-hedge-us", type=int, default=1000,
                    help="service hedge deadline (us; 0 = off): late requests are also "
                         "verified on host threads, first verdict wins")
    ap.add_argument("--service-hedge-threads", type=int, default=6)
    ap.add_argument("--service-hedge-queued", type=int, default=512,
                    help="units a batch still waiting for a job slot may join the host "
                         "queue with (taken for the host alone)")
    ap.add_argument("--no-worker", action="store_true",
                    help="skip the worker Processor latency leg")
    ap.add_argument("--worker-rates", default="50,500,5000")
    ap.add_argument("--worker-seconds", type=float, default=2.0)
    ap.add_argument("--worker-max-batches", type=float, default=2000)
    ap.add_argument("--worker-host-rates", default="50,500,2000",
                    help="offered rates of the default host-hashing Processor (empty = skip)")
    ap.add_argument("--worker-deep", default="10000:1024",
                    help="extra worker loads rate:lookahead (Processor max_in_flight)")
    ap.add_argument("--worker-delay", type=float, default=0.0005,
                    help="VerificationService max_delay (s) for the worker leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        log(f"--gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')}: one rank per "
            "GPU is the contract; refusing to report a mismatched n_gpus")
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NW_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks sharing the GPUs
    # of a smaller box (rank -> device local % device_count); the driver's runs use RCCL.
    backend = os.environ.get("NW_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    L = _lib.lib()
    ndev = L.nw_init()
    if ndev <= 0:
        raise RuntimeError(f"nw_init failed: {ndev} {L.nw_last_error().decode()}")
    check(L.nw_set_device(local), "nw_set_device")
    # A dedicated (non-null) stream: the kernels launch on it and torch.cuda.Event records
    # on it, so the events bracket exactly the kernel launches.
    tstream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(tstream)
    stream = ctypes.c_void_p(tstream.cuda_stream)
    assert stream.value, "expected a non-null HIP stream"

    result = {}
    if args.workload == "strict":
        r = run_strict(args, dev, stream, rank, world)
        units = r["n_total"]
        value = units / r["elapsed"] * args.steps
        achieved = r["n"] * MAC_PER_STRICT_VERIFY / (r["kernel_ms"] * 1e-3) / 1e12
        traffic, tsrc = pmc_traffic("k_verify_strict", r["n"])
        issue_peak, issue_src = pmc_issue_peak()
        result = {
            "metric": METRIC, "value": value, "unit": "verifies/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": r["elapsed"] / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "config4_mixed_corpus_strict_verify",
                       "items_per_gpu": r["n"], "items_total": r["n_total"],
                       "unique_items": args.unique,
                       "invalid_fraction": 0.1, "semantics": "crypto::Signature::verify (dalek verify_strict)",
                       "parallelism": f"shard{world}",
                       "exchange": "all_gather of the per-shard verdict bitmaps",
                       "gather_ms": r["gather_ms"]},
            "roofline": {"bound": "valu", "achieved": achieved, "peak": PEAK_TMAC,
                         "unit": "TMAC/s", "frac": achieved / PEAK_TMAC,
                         "peak_measured": PEAK_TMAC_MEASURED,
                         "frac_measured": achieved / PEAK_TMAC_MEASURED,
                         "peak_source": "spec 256 CU x 4 SIMD x 16 MAC/clk x 2.4 GHz; measured "
                                        "v_mad_u64_u32 rate, profiles/r01_ubench_valu_4wps.txt",
                         "traffic": traffic,
                         "traffic_unit": "HBM bytes per launch", "traffic_source": tsrc,
                         "algorithmic_bytes": r["n"] * (32 + 32 + 64 + 4) + r["n"] / 8,
                         "kernel": ("k_verify_strict" if os.environ.get("NW_STRICT_TRIAGE") == "0"
                                    else "k_strict_triage + k_verify_strict_pre + k_status_bitmap"),
                         "kernel_ms": r["kernel_ms"],
                         "work_per_unit": f"{MAC_PER_STRICT_VERIFY} MAC/verify (SURVEY 8d)",
                         "issue_peak": issue_peak, "issue_unit": "verifies/s",
                         "issue_frac": (r["n"] / (r["kernel_ms"] * 1e-3) / issue_peak
                                        if issue_peak else None),
                         "issue_source": issue_src},
            "parity": "ok" if r["parity"] else "FAIL",
        }
        sample = r["sample"]
        del r
        torch.cuda.empty_cache()
        if not args.no_sha:
            s = run_sha(args, dev, stream, rank, world)
            gbs = s["bytes"] * world / (s["elapsed"] / args.steps) / 1e9
            kgbs = s["bytes"] / (s["kernel_ms"] * 1e-3) / 1e9
            blocks = s["n"] * ((W.BATCH_BYTES + 17 + 127) // 128)
            tops = blocks * SHA_OPS_PER_BLOCK / (s["kernel_ms"] * 1e-3) / 1e12
            straffic, ssrc = pmc_traffic("k_sha512_digest32", s["n"])
            result["sha512"] = {"workload": "config3_worker_batch_digests",
                                "batches_per_gpu": s["n"], "batch_bytes": W.BATCH_BYTES,
                                "GB_per_s": gbs, "kernel_GB_per_s": kgbs,
                                "hbm_frac": kgbs / PEAK_HBM_GBS,
                                "valu_Tops": tops, "valu_frac": tops / PEAK_TOPS_FULL,
                                "valu_note": "valu_* use SURVEY's 4,800 ops/block against the "
                                             "full-rate peak; issue_* use the kernel's PMC "
                                             "VALU count against one wave per SIMD's rate",
                                "kernel_ms": s["kernel_ms"],
                                "traffic": straffic, "traffic_source": ssrc,
                                "algorithmic_bytes": s["bytes"] + 32 * s["n"],
                                "parity": "ok" if s["parity"] else "FAIL"}
            lops, lsrc = pmc_sha_valu(s["n"])
            if lops:
                iss = lops / (s["kernel_ms"] * 1e-3) / 1e12
                result["sha512"].update({"issue_Tops": iss, "issue_peak_Tops": PEAK_TOPS_ONE_WAVE,
                                         "issue_frac": iss / PEAK_TOPS_ONE_WAVE,
                                         "issue_ubench_one_wave_Tops": UBENCH_TOPS_ONE_WAVE,
                                         "issue_source": f"{lsrc} (SQ_INSTS_VALU) / "
                                                         "profiles/r01_ubench_valu_1wps.txt"})
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                result["sha512"]["cpu_baseline"] = cpu_baseline_sha(s["sample"],
                                                                    min(3.0, args.cpu_seconds))
            if not s["parity"]:
                result["parity"] = "FAIL"
        if not args.no_cert:
            result["cert_stream"] = {}
            result["cert_stream_invalid"] = {}
            cache = {}
            for N in [int(x) for x in args.committees.split(",") if x]:
                r2, csample = run_cert(args, dev, stream, rank, world, N, stream_cache=cache)
                result["cert_stream"][f"N{N}"] = r2
                if r2["parity"] != "ok":
                    result["parity"] = "FAIL"
                if rank == 0 and world == 1 and not args.no_cpu_baseline:
                    r2["cpu_baseline"] = cpu_baseline_cert(csample, N, min(6.0, args.cpu_seconds))
                    if not r2["cpu_baseline"]["statuses_match"]:
                        result["parity"] = "FAIL"
                if args.cert_invalid > 0:
                    r3, _ = run_cert(args, dev, stream, rank, world, N, invalid=args.cert_invalid,
                                     stream_cache=cache)
                    r3["vs_all_valid"] = r3["certs_per_s"] / r2["certs_per_s"]
                    result["cert_stream_invalid"][f"N{N}"] = r3
                    if r3["parity"] != "ok":
                        result["parity"] = "FAIL"
                    r4 = run_cert_alternating(args, dev, stream, rank, world, N,
                                              args.cert_invalid, stream_cache=cache)
                    result.setdefault("cert_stream_alternating", {})[f"N{N}"] = r4
                    if r4["parity"] != "ok":
                        result["parity"] = "FAIL"
                cache.pop(N, None)
            for N in [int(x) for x in args.cert_payload_committees.split(",") if x]:
                rp, _ = run_cert(args, dev, stream, rank, world, N, stream_cache=cache,
                                 payload=args.cert_payload)
                result.setdefault("cert_stream_p32", {})[f"N{N}"] = rp
                if rp["parity"] != "ok":
                    result["parity"] = "FAIL"
                cache.pop((N, args.cert_payload), None)
        if not args.no_batch:
            r1, bsample = run_batch10k(args, dev, stream, rank, world)
            result["verify_batch_10k"] = r1
            if r1["parity"] != "ok":
                result["parity"] = "FAIL"
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                r1["cpu_baseline"] = cpu_baseline_batch(bsample, min(5.0, args.cpu_seconds))
        if not args.no_wire:
            rw = run_wire(args, dev, stream, rank, world)
            result["wire_ingest"] = rw
            if rw["parity"] != "ok":
                result["parity"] = "FAIL"
        # the latency legs are per process (one service / worker loop and its host threads):
        # at N > 1 rank 0 runs them while the other ranks wait at the final barrier, so that
        # N load generators do not compete for the node's cores
        if not args.no_worker and rank == 0:
            rwk = run_worker_latency(args, rank, world)
            result["worker_latency"] = rwk
            if rwk["parity"] != "ok":
                result["parity"] = "FAIL"
        if not args.no_service and rank == 0:
            result["service_latency"] = {}
            for N in [int(x) for x in args.service_committees.split(",") if x]:
                rs = run_service_latency(args, rank, world, N)
                result["service_latency"][f"N{N}"] = rs
                if rs["parity"] != "ok":
                    result["parity"] = "FAIL"
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cb, agree = cpu_baseline_strict(sample, args.cpu_seconds)
            result["cpu_baseline"] = cb
            if not agree:
                result["parity"] = "FAIL"
                log("oracle disagrees with GPU statuses on the cpu_baseline sample")
    elif args.workload == "cert":
        res, res_bad, res_alt, cache = {}, {}, {}, {}
        for N in [int(x) for x in args.committees.split(",") if x]:
            res[f"N{N}"] = run_cert(args, dev, stream, rank, world, N, stream_cache=cache)[0]
            if args.cert_invalid > 0:
                r3 = run_cert(args, dev, stream, rank, world, N, invalid=args.cert_invalid,
                              stream_cache=cache)[0]
                r3["vs_all_valid"] = r3["certs_per_s"] / res[f"N{N}"]["certs_per_s"]
                res_bad[f"N{N}"] = r3
                res_alt[f"N{N}"] = run_cert_alternating(args, dev, stream, rank, world, N,
                                                        args.cert_invalid, stream_cache=cache)
            cache.pop(N, None)
        res_p = {}
        for N in [int(x) for x in args.cert_payload_committees.split(",") if x]:
            res_p[f"N{N}"] = run_cert(args, dev, stream, rank, world, N, stream_cache=cache,
                                      payload=args.cert_payload)[0]
            cache.pop((N, args.cert_payload), None)
        last = list(res.values())[-1]
        result = {"metric": METRIC, "value": last["sig_checks_per_s"], "unit": "verifies/s",
                  "n_gpus": world, "steps": args.cert_steps, "warmup": 1,
                  "ms_per_step": last["ms_per_step"], "higher_is_better": True,
                  "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
                  "config": {"workload": "config2_certificate_stream",
                             "certs_per_gpu": args.certs, "parallelism": f"shard{world}"},
                  "cert_stream": res, "cert_stream_invalid": res_bad,
                  "cert_stream_alternating": res_alt, "cert_stream_p32": res_p,
                  "parity": "ok" if all(r["parity"] == "ok" for r in
                                        list(res.values()) + list(res_bad.values()) +
                                        list(res_alt.values()) + list(res_p.values()))
                  else "FAIL"}
    elif args.workload == "service":
        res = {f"N{N}": run_service_latency(args, rank, world, N)
               for N in [int(x) for x in args.service_committees.split(",") if x]}
        last = list(res.values())[-1]["loads"][-1]
        result = {"metric": METRIC, "value": last["achieved_certs_per_s"], "unit": "certs/s",
                  "n_gpus": world, "steps": 1, "warmup": 1, "ms_per_step": None,
                  "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                  "dtype": "u32", "data": "synthetic",
                  "config": {"workload": "certificate_service_latency",
                             "parallelism": f"shard{world}"},
                  "service_latency": res,
                  "parity": "ok" if all(r["parity"] == "ok" for r in res.values()) else "FAIL"}
    elif args.workload == "worker":
        rw = run_worker_latency(args, rank, world)
        last = rw["loads"][0]
        result = {"metric": METRIC, "value": last["achieved_batches_per_s"], "unit": "batches/s",
                  "n_gpus": world, "steps": 1, "warmup": 1, "ms_per_step": None,
                  "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                  "dtype": "u64", "data": "synthetic",
                  "config": {"workload": "worker_processor_latency",
                             "parallelism": f"shard{world}"},
                  "worker_latency": rw, "parity": rw["parity"]}
    elif args.workload == "batch":
        r1, bsample = run_batch10k(args, dev, stream, rank, world)
        result = {"metric": METRIC, "value": r1["verifies_per_s_resident"], "unit": "verifies/s",
                  "n_gpus": world, "steps": args.steps, "warmup": 1,
                  "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
                  "vs_baseline": None, "dtype": "u32", "data": "synthetic",
                  "config": {"workload": "config1_verify_batch_10k", "parallelism": f"shard{world}"},
                  "verify_batch_10k": r1, "parity": r1["parity"]}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline_batch(bsample, min(5.0, args.cpu_seconds))
    else:
        s = run_sha(args, dev, stream, rank, world)
        gbs = s["bytes"] * world / (s["elapsed"] / args.steps) / 1e9
        kgbs = s["bytes"] / (s["kernel_ms"] * 1e-3) / 1e9
        straffic, ssrc = pmc_traffic("k_sha512_digest32", s["n"])
        result = {
            "metric": METRIC, "value": gbs, "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": s["elapsed"] / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "config3_worker_batch_digests", "batches_per_gpu": s["n"],
                       "batch_bytes": W.BATCH_BYTES, "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": kgbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": kgbs / PEAK_HBM_GBS, "traffic": straffic,
                         "traffic_source": ssrc,
                         "kernel": "k_sha512_digest32", "kernel_ms": s["kernel_ms"]},
            "parity": "ok" if s["parity"] else "FAIL",
        }
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline_sha(s["sample"], min(3.0, args.cpu_seconds))
    result["summary"] = summary(result)
    if rank == 0:
        detail = write_detail(result)
        log(f"full per-leg record: {detail}")
        print(json.dumps(compact_line(result, detail), separators=(",", ":")), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if result.get("parity") != "ok":
        sys.exit(1)


if __name__ == "__main__":
    main()
