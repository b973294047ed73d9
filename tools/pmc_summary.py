#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per nw:: kernel.

HBM traffic follows the MI355X guide's HBM/rocprofv3 section: FETCH_SIZE and WRITE_SIZE
are KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide coalesced stream, so the
read side is doubled (the SHA-512 kernel calibrates this: 2 x FETCH_SIZE == its message
bytes). Usage: python tools/pmc_summary.py <dir with fetch.csv write.csv sq.csv grbm.csv>
"""
import collections
import csv
import json
import os
import sys


def load(path):
    agg = collections.defaultdict(float)
    calls = collections.Counter()
    if not os.path.exists(path):
        return agg, calls
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith("nw::"):
            continue
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        calls[(k, r["Counter_Name"])] += 1
    return agg, calls


def summary(d):
    out = collections.defaultdict(dict)
    for name in ("fetch", "write", "sq", "grbm"):
        agg, calls = load(os.path.join(d, name + ".csv"))
        for (k, c), v in agg.items():
            out[k][c] = v
            out[k]["dispatches"] = calls[(k, c)]
    for k, v in out.items():
        if "FETCH_SIZE" in v:
            v["hbm_read_bytes_corrected"] = 2 * v["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in v:
            v["hbm_write_bytes"] = v["WRITE_SIZE"] * 1024
        if "SQ_INSTS_VALU" in v and "SQ_WAVES" in v and v["SQ_WAVES"]:
            v["valu_insts_per_wave"] = v["SQ_INSTS_VALU"] / v["SQ_WAVES"]
    return out


if __name__ == "__main__":
    print(json.dumps(summary(sys.argv[1] if len(sys.argv) > 1 else "profiles/r01_pmc"), indent=1))
