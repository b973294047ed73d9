#!/usr/bin/env python3
"""Completion-stall probe (GPU box, diagnostics): a trivial kernel launched every ~100 us on
one stream for SECONDS, each completion awaited by polling its event, as the service's
completer does. Prints one JSON line: the launch-to-completion latency percentiles and every
iteration above 1 ms with its time into the run. If the rare 5-30 ms stalls of the
certificate service's timeline (profiles/r05d) show up here too, they are not the engine's.
    python tools/stall_probe.py [SECONDS]"""
import json
import sys
import time

import numpy as np
import torch


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    x = torch.zeros(64, device="cuda")
    s = torch.cuda.Stream()
    lat, slow = [], []
    t_start = time.perf_counter()
    with torch.cuda.stream(s):
        for _ in range(100):
            x.add_(1)
        s.synchronize()
        while True:
            t0 = time.perf_counter()
            if t0 - t_start > secs:
                break
            x.add_(1)
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
    print(json.dumps({"iterations": len(a), "p50_ms": float(np.percentile(a, 50)),
                      "p99_ms": float(np.percentile(a, 99)), "max_ms": float(a.max()),
                      "over_1ms": slow}))


if __name__ == "__main__":
    main()
