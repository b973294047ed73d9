#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_strict.sh / pmc_passes.sh output dirs).

    python tools/pmc_report.py DIR [KERNEL_SUBSTRING] [--items N]

Sums each counter over the dispatches of the matching kernel and prints per-wave VALU
instructions, the wave-cycle breakdown and HBM bytes (FETCH_SIZE doubled per the gfx950
correction in MI355X_MICROARCH.md; WRITE_SIZE as reported), per item when --items is given.
"""
import csv
import glob
import os
import sys


def collect(d, key):
    agg = {}
    for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if key not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return agg


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "k_verify_strict"
    items = int(sys.argv[sys.argv.index("--items") + 1]) if "--items" in sys.argv else 0
    a = collect(d, key)
    out = {"kernel": key, **a}
    waves = a.get("SQ_WAVES", 0)
    if waves:
        out["valu_insts_per_wave"] = a.get("SQ_INSTS_VALU", 0) / waves
        out["vmem_rd_per_wave"] = a.get("SQ_INSTS_VMEM_RD", 0) / waves
        if a.get("SQ_WAVE_CYCLES"):
            out["valu_active_frac_of_wave_cycles"] = (a.get("SQ_ACTIVE_INST_VALU", 0)
                                                      / a["SQ_WAVE_CYCLES"])
    if "FETCH_SIZE" in a:
        out["hbm_read_bytes"] = 2 * a["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in a:
        out["hbm_write_bytes"] = a["WRITE_SIZE"] * 1024
    if items:
        for k in ("hbm_read_bytes", "hbm_write_bytes"):
            if k in out:
                out[k + "_per_item"] = out[k] / items
    for k, v in out.items():
        print(f"{k:36s} {v:,.1f}" if isinstance(v, float) else f"{k:36s} {v}")


if __name__ == "__main__":
    main()
