#!/usr/bin/env python3
"""Completion-stall probe (GPU box, diagnostics): a small GPU operation issued every ~100 us
on one stream for SECONDS, each completion awaited by polling its event, as the service's
completer does. Prints one JSON line per mode: the issue-to-completion latency percentiles
and every iteration above 1 ms with its time into the run.
    python tools/stall_probe.py [SECONDS] [MODE ...]
Modes: device  a trivial kernel on device memory (torch);
       pinned  the engine's SHA-512 kernel over 64 messages that live in pinned HOST memory
               (the kernel reads them across the bus, as the small-job kernel reads its
               inputs; nw_dev_sha512_digest32_many on the mapped pointer);
       copy    a 64 KB pinned-host -> device copy (DMA engine);
       mixed   the three in turn, each awaited on its own (same host conditions for all).
The certificate service showed rare 1-13 ms completion stalls (profiles/r05d-g) while a
clock-reading thread kept running; these modes separate the device, the bus and the DMA."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(secs, issue):
    s = torch.cuda.current_stream()
    lat, slow = [], []
    for _ in range(100):
        issue()
    s.synchronize()
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        if t0 - t_start > secs:
            break
        issue()
        ev = torch.cuda.Event()
        ev.record(s)
        while not ev.query():
            pass
        dt = time.perf_counter() - t0
        lat.append(dt)
        if dt > 1e-3:
            slow.append((round(t0 - t_start, 4), round(dt * 1e3, 3)))
        while time.perf_counter() - t0 < 1e-4:
            pass
    a = np.array(lat) * 1e3
    return {"iterations": len(a), "p50_ms": float(np.percentile(a, 50)),
            "p99_ms": float(np.percentile(a, 99)), "max_ms": float(a.max()), "over_1ms": slow}


def run_mixed(secs, issues):
    """The modes' operations in turn (one of each per ~300 us), each awaited on its own,
    so that all of them see the same host conditions."""
    s = torch.cuda.current_stream()
    names = list(issues)
    lat = {k: [] for k in names}
    slow = {k: [] for k in names}
    for _ in range(50):
        for k in names:
            issues[k]()
    s.synchronize()
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < secs:
        for k in names:
            t0 = time.perf_counter()
            issues[k]()
            ev = torch.cuda.Event()
            ev.record(s)
            while not ev.query():
                pass
            dt = time.perf_counter() - t0
            lat[k].append(dt)
            if dt > 1e-3:
                slow[k].append((round(t0 - t_start, 4), round(dt * 1e3, 3)))
            while time.perf_counter() - t0 < 1e-4:
                pass
    out = {}
    for k in names:
        a = np.array(lat[k]) * 1e3
        out[k] = {"iterations": len(a), "p50_ms": float(np.percentile(a, 50)),
                  "p99_ms": float(np.percentile(a, 99)), "max_ms": float(a.max()),
                  "over_1ms": slow[k]}
    return out


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    modes = sys.argv[2:] or ["device"]
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    mixed = "mixed" in modes
    if mixed:
        modes = ["device", "pinned", "copy"]
    issues = {}
    for mode in modes:
        if mode == "device":
            x = torch.zeros(64, device="cuda")
            issue = lambda x=x: x.add_(1)
        elif mode == "pinned":
            from narwhal_amd import _lib
            L = _lib.lib()
            assert L.nw_init() > 0 and L.nw_set_device(0) == 0
            n, ln = 64, 1024
            host = torch.zeros(n * ln, dtype=torch.uint8).pin_memory()
            offs = torch.arange(n, dtype=torch.int64, device="cuda") * ln
            lens = torch.full((n,), ln, dtype=torch.int64, device="cuda")
            out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
            P = ctypes.c_void_p
            sp = P(st.cuda_stream)

            def issue(host=host, offs=offs, lens=lens, out=out, L=L, n=n, sp=sp):
                rc = L.nw_dev_sha512_digest32_many(P(host.data_ptr()), P(offs.data_ptr()),
                                                   P(lens.data_ptr()), n, P(out.data_ptr()), sp)
                assert rc == 0, L.nw_last_error()
        elif mode == "copy":
            hcopy = torch.zeros(1 << 16, dtype=torch.uint8).pin_memory()
            dev = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
            issue = lambda dev=dev, hcopy=hcopy: dev.copy_(hcopy, non_blocking=True)
        else:
            raise SystemExit(f"unknown mode {mode}")
        issues[mode] = issue
        if not mixed:
            print(json.dumps({"mode": mode, **run(secs, issue)}), flush=True)
    if mixed:
        print(json.dumps({"mode": "mixed", **run_mixed(secs, issues)}), flush=True)


if __name__ == "__main__":
    main()
