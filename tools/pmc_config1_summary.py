"""Summarise tools/pmc_config1.sh: per config-1 kernel, the median over its dispatches of each
counter, HBM bytes per dispatch (FETCH_SIZE x 2 + WRITE_SIZE, KiB -> bytes, the gfx950
correction of MI355X_MICROARCH.md) and the L2 hit rate.
    python tools/pmc_config1_summary.py OUTDIR profiles/TAG   (writes config1_pmc.json)"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

KERNELS = ("k_pip_points_sorted", "k_pip_tail_fused")


def main():
    src, dst = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in glob.glob(os.path.join(src, "*", "**", "*counter_collection.csv"), recursive=True):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
            k = next((x for x in KERNELS if x in name), None)
            if k:
                acc[(k, int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, d, cn), v in acc.items():
            per[k][cn][d] = v
    out = {}
    for k, cs in per.items():
        e = {cn: statistics.median(list(v.values())) for cn, v in cs.items()}
        e["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_read_bytes"] = 2 * e["FETCH_SIZE"] * 1024
            e["hbm_write_bytes"] = e["WRITE_SIZE"] * 1024
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if e.get("TCC_HIT_sum") is not None and e.get("TCC_MISS_sum") is not None:
            tot = e["TCC_HIT_sum"] + e["TCC_MISS_sum"]
            e["l2_hit_rate"] = e["TCC_HIT_sum"] / tot if tot else None
        if e.get("SQ_WAVE_CYCLES"):
            e["issue_stall_frac"] = e.get("SQ_WAIT_INST_ANY", 0) / e["SQ_WAVE_CYCLES"]
        out[k] = e
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, "config1_pmc.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
