#!/usr/bin/env python3
"""Summarise an NW_SERVICE_DEBUG per-job timeline (diagnostics): per second of the run, the
jobs, certificates per job, and per job the microseconds from its first request to being
taken, the submit call (staging copy + launch: sub1 - sub0), the device (done - sub1) and the
callbacks (cb - done), mean and max. Shows which stage grows when a sustained load degrades.
    python tools/service_timeline.py TIMELINE.csv [--bin SECONDS]"""
import argparse
import json

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--bin", type=float, default=1.0)
    a = ap.parse_args()
    d = np.genfromtxt(a.csv, delimiter=",", names=True, dtype=np.int64)
    if d.size == 0:
        print(json.dumps({"csv": a.csv, "jobs": 0}))
        return
    t0 = d["first_ns"].min()
    stages = {"wait_us": d["taken_ns"] - d["first_ns"], "submit_us": d["sub1_ns"] - d["sub0_ns"],
              "device_us": d["done_ns"] - d["sub1_ns"], "callbacks_us": d["cb_ns"] - d["done_ns"]}
    b = ((d["first_ns"] - t0) / 1e9 / a.bin).astype(np.int64)
    rows = []
    for k in range(int(b.max()) + 1):
        m = b == k
        if not m.any():
            continue
        r = {"t_s": round(k * a.bin, 2), "jobs": int(m.sum()), "certs_per_job": round(float(d["n"][m].mean()), 1)}
        for name, v in stages.items():
            r[name] = [round(float(v[m].mean()) / 1e3, 1), round(float(v[m].max()) / 1e3, 1)]
        rows.append(r)
    tot = {name: {"p50": round(float(np.percentile(v, 50)) / 1e3, 1),
                  "p99": round(float(np.percentile(v, 99)) / 1e3, 1),
                  "max": round(float(v.max()) / 1e3, 1),
                  "sum_s": round(float(v.sum()) / 1e9, 3)} for name, v in stages.items()}
    print(json.dumps({"csv": a.csv, "jobs": int(d.size), "by_submitter": {str(h): int((d["how"] == h).sum()) for h in np.unique(d["how"])},
                      "stages_us": tot, "per_bin": rows}))


if __name__ == "__main__":
    main()
