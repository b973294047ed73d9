#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into committed profile files.

    python tools/profile_summary.py gpurun_out/prof_TAG profiles/TAG

Writes into profiles/TAG/:
  kernel_stats.csv     rocprofv3 --stats summary of the traced bench run (verbatim)
  kernels_by_grid.csv  the same trace grouped by (kernel, grid size): calls and mean/min/max
                       duration, plus the mean over the "large" calls (within 20 % of the
                       longest) = the bench-size launches, which is what bench.py's
                       kernel_ms is compared with
  pmc.json             PMC counters per (kernel, grid), largest dispatch, from the one-step
                       bench runs, with
                       HBM bytes per dispatch (FETCH_SIZE x 2 per the gfx950 correction in
                       MI355X_MICROARCH.md, WRITE_SIZE as reported; both in KiB)
  bench_traced.json    the bench line printed under the tracer
and refreshes profiles/traffic.json, the per-launch HBM traffic bench.py reports as
roofline.traffic for its dominant kernels (largest-grid dispatch of each).
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

# dominant kernels and the units one bench-default launch processes (bench.py defaults)
KERNELS = {"k_verify_strict": ("config4 strict verify launch", 12_500_000, "verifies"),
           "k_sha512_digest32": ("config3 SHA-512 launch", 65_536, "508,052-B batches")}
# the config-4 launch in two passes (NW_STRICT_TRIAGE): its kernels' largest dispatches summed
# (12.5M items are one slice: one dispatch of each per launch)
COMPOSITE = {"k_verify_strict": ("k_strict_triage", "k_verify_strict_pre", "k_status_bitmap")}


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:\(anonymous namespace\)::)?\w+)\(", name)
    base = m.group(1) if m else name.split("(")[0]
    base = re.sub(r"<[^<>]*>", "", base)   # k_verify_strict<false> -> k_verify_strict
    return base.split("::")[-1][:60]


def one(pattern):
    got = sorted(glob.glob(pattern, recursive=True))
    return got[0] if got else None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    tag = os.path.basename(os.path.normpath(dst))
    stats = one(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    trace = one(os.path.join(src, "trace", "**", "*kernel_trace.csv"))
    if trace:
        g = collections.defaultdict(list)
        for r in csv.DictReader(open(trace)):
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            g[(short(r["Kernel_Name"]), int(r["Grid_Size_X"] if "Grid_Size_X" in r else r["Grid_Size"]))].append(dur)
        with open(os.path.join(dst, "kernels_by_grid.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "grid", "calls", "mean_ms", "min_ms", "max_ms", "total_ms",
                        "large_calls", "large_mean_ms"])
            for (k, grid), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
                # the bench-size launches: calls within 20% of the longest (a persistent
                # kernel's grid does not change with the item count)
                big = [x for x in d if x >= 0.8 * max(d)]
                w.writerow([k, grid, len(d), f"{sum(d) / len(d) / 1e6:.4f}", f"{min(d) / 1e6:.4f}",
                            f"{max(d) / 1e6:.4f}", f"{sum(d) / 1e6:.3f}", len(big),
                            f"{sum(big) / len(big) / 1e6:.4f}"])
    bt = os.path.join(src, "bench_traced.json")
    if os.path.exists(bt) and os.path.getsize(bt):
        shutil.copy(bt, os.path.join(dst, "bench_traced.json"))
    # PMC: per dispatch, then per (kernel, grid) the LARGEST dispatch (the bench-size launch;
    # smaller launches of the same kernel and grid, e.g. the wire leg's, are other work)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            acc[(short(r["Kernel_Name"]), int(r["Grid_Size"]), int(r["Dispatch_Id"]),
                 r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, grid, _d, cn), v in acc.items():
            per[(k, grid)][cn].append(v)
    pmc = {}
    for (k, grid), cs in sorted(per.items()):
        e = {cn: max(v) for cn, v in cs.items()}
        e["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in e:
            e["hbm_read_bytes"] = 2 * e["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in e:
            e["hbm_write_bytes"] = e["WRITE_SIZE"] * 1024
        if e.get("SQ_WAVES"):
            e["valu_insts_per_wave"] = e.get("SQ_INSTS_VALU", 0) / e["SQ_WAVES"]
        if e.get("SQ_INSTS_LDS"):
            e["lds_bank_conflict_per_lds_inst"] = e.get("SQ_LDS_BANK_CONFLICT", 0) / e["SQ_INSTS_LDS"]
        pmc[f"{k}@grid{grid}"] = e
    if pmc:
        json.dump(pmc, open(os.path.join(dst, "pmc.json"), "w"), indent=1, sort_keys=True)
    # traffic for bench.py: the largest-grid dispatch of each dominant kernel
    tpath = os.path.join(os.path.dirname(os.path.normpath(dst)), "traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    def largest(k):
        cands = [(grid, e) for (kk, grid), _ in per.items() if kk == k
                 for e in [pmc[f"{kk}@grid{grid}"]] if "hbm_read_bytes" in e]
        return max(cands, key=lambda ge: ge[0]) if cands else (None, None)
    for k, (what, units, unit_name) in KERNELS.items():
        parts = [(kk,) + largest(kk) for kk in COMPOSITE.get(k, ())]
        parts = [p for p in parts if p[2] is not None]
        if parts and any(p[0] != "k_status_bitmap" for p in parts):
            e = {"hbm_read_bytes": sum(p[2]["hbm_read_bytes"] for p in parts),
                 "hbm_write_bytes": sum(p[2].get("hbm_write_bytes") or 0 for p in parts)}
            grid = {p[0]: p[1] for p in parts}
            what = what + " (" + " + ".join(p[0] for p in parts) + ")"
        else:
            grid, e = largest(k)
        if e is None:
            continue
        traffic[k] = {"grid": grid, "hbm_read_bytes": e["hbm_read_bytes"],
                      "hbm_write_bytes": e.get("hbm_write_bytes"),
                      "hbm_bytes": e["hbm_read_bytes"] + (e.get("hbm_write_bytes") or 0),
                      "units": units, "unit": unit_name,
                      "what": what, "source": f"profiles/{tag}/pmc.json"}
    json.dump(traffic, open(tpath, "w"), indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
