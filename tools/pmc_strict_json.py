#!/usr/bin/env python3
"""The strict kernel's VALU mix and stall fractions as committed JSON
(profiles/<tag>/pmc_mix.json, stall_pmc.json) from tools/pmc_mix.sh / pmc_stall.sh output.

    python tools/pmc_strict_json.py MIXDIR STALLDIR OUTDIR [--items N]

Counters are summed over the config-4 launch's dispatches of the one-step bench run (the
two-pass path's k_strict_triage + k_verify_strict_pre + k_status_bitmap, or the one-pass
k_verify_strict)
(--items-per-gpu N, default 4,194,304). Lane-ops = instructions x 64 / items; the issue
budget prices INT64 (v_mad_u64_u32, 64-bit shifts), INT32 (half-rate 32-bit) and the rest
at the microbenchmarked rates (profiles/r01_ubench_valu_4wps.txt).
"""
import csv
import glob
import json
import os
import sys

RATES = {"int64": 32.39, "int32": 36.0, "other": 63.0}


STRICT = ("k_verify_strict", "k_strict_triage", "k_status_bitmap")


def collect(d, keys=STRICT):
    agg = {}
    for f in glob.glob(os.path.join(d, "**", "p_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Kernel_Name"] for k in keys):
                agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return agg


def main():
    mixd, stalld, out = sys.argv[1], sys.argv[2], sys.argv[3]
    items = int(sys.argv[sys.argv.index("--items") + 1]) if "--items" in sys.argv else 4194304
    os.makedirs(out, exist_ok=True)
    m = collect(mixd)
    if m:
        valu = m["SQ_INSTS_VALU"] * 64 / items
        i64 = m.get("SQ_INSTS_VALU_INT64", 0) * 64 / items
        i32 = m.get("SQ_INSTS_VALU_INT32", 0) * 64 / items
        lane = {"valu": valu, "int64": i64, "int32": i32, "other": valu - i64 - i32}
        ns = sum(lane[k] / (RATES[k] * 1e12) for k in RATES) * 1e9
        json.dump({"kernel": "config-4 launch (" + " + ".join(STRICT) + ")", "items": items,
                   "counters": m,
                   "per_verify_lane_ops": lane,
                   "issue_rates_T_lane_ops_s": {**RATES,
                                                "source": "profiles/r01_ubench_valu_4wps.txt"},
                   "issue_ns_per_verify": ns, "issue_peak_verifies_per_s": 1e9 / ns,
                   "source": "tools/pmc_mix.sh (one rocprofv3 --pmc pass)"},
                  open(os.path.join(out, "pmc_mix.json"), "w"), indent=4)
    s = collect(stalld)
    if s and s.get("SQ_WAVE_CYCLES"):
        wc = s["SQ_WAVE_CYCLES"]
        json.dump({"kernel": "k_verify_strict", "items": items, "counters": s,
                   "fractions_of_wave_cycles": {
                       "issuing_frac": s.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                       "wait_inst_any_frac": s.get("SQ_WAIT_INST_ANY", 0) / wc,
                       "waitcnt_frac": s.get("SQ_WAIT_ANY", 0) / wc},
                   "lds_insts_per_verify": s.get("SQ_ACTIVE_INST_LDS", 0) / items,
                   "source": "tools/pmc_stall.sh"},
                  open(os.path.join(out, "stall_pmc.json"), "w"), indent=4)


if __name__ == "__main__":
    main()
