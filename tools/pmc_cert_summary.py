#!/usr/bin/env python3
"""Summarise tools/pmc_cert.sh output into profiles/<tag>/cert_pmc.json.

    python tools/pmc_cert_summary.py gpurun_out/pmc_cert_TAG profiles/TAG

Per (mode, committee size) and per kernel, per bench call (warmup + timed call run the
same dispatches, so half of each kernel's totals): trace time, and from the PMC passes: HBM bytes (FETCH_SIZE x 2 per the gfx950 correction in
MI355X_MICROARCH.md + WRITE_SIZE), TCC hit rate, VALU instructions, the issue / wait split
(SQ_WAIT_INST_ANY, SQ_WAIT_ANY over SQ_WAVE_CYCLES) and per-vote figures (nvotes of one
bench call = 1M certificates x q).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

Q = {4: 3, 10: 7, 50: 34, 100: 67}
NCERT = 1_000_000


def short(name):
    m = re.match(r"(?:void )?([\w:]+(?:\(anonymous namespace\)::)?\w+)\(", name)
    base = m.group(1) if m else name.split("(")[0]
    return base.split("::")[-1][:60]


def one(pattern):
    got = sorted(glob.glob(pattern, recursive=True))
    return got[0] if got else None


def counters(d):
    """kernel -> counter -> sum over its dispatches / 2 (the bench's warmup call and timed
    call run the same dispatches; large calls are split into slices, so one dispatch is not
    one call). Corpus-building kernels (k_sign, k_keypair, k_btab_build, k_key_*) are
    outside the calls and their figures are not per call."""
    f = one(os.path.join(d, "**", "*counter_collection.csv"))
    if not f:
        return {}
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        acc[(short(r["Kernel_Name"]), int(r["Dispatch_Id"]), r["Counter_Name"])] += \
            float(r["Counter_Value"])
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for (k, disp, cn), v in acc.items():
        per[k][disp][cn] = v
    out = {}
    for k, disps in per.items():
        tot = collections.defaultdict(float)
        for c in disps.values():
            for cn, v in c.items():
                tot[cn] += v / 2
        out[k] = dict(tot)
    return out


def trace(d):
    """kernel -> (calls, total ms) over the whole traced run, plus the per-call split: the
    bench does one warmup call and one timed call, so half of each kernel's dispatches."""
    f = one(os.path.join(d, "**", "*kernel_trace.csv"))
    if not f:
        return {}
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        g[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: {"dispatches": len(v), "total_ms": sum(v) / 1e6} for k, v in g.items()}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    res = {}
    for tdir in sorted(glob.glob(os.path.join(src, "*_trace"))):
        tag = os.path.basename(tdir)[: -len("_trace")]
        mode, n = tag.split("_n")
        N = int(n)
        nv = NCERT * Q[N]
        tr = trace(tdir)
        pm = {}
        for p in ("fetch", "write", "tcc", "sq", "grbm"):
            for k, c in counters(os.path.join(src, f"{tag}_{p}")).items():
                pm.setdefault(k, {}).update(c)
        bench = {}
        try:
            bench = json.load(open(os.path.join(src, f"{tag}_trace.json")))["cert_stream"][f"N{N}"]
        except (OSError, ValueError, KeyError):
            pass
        kern = {}
        for k in sorted(set(tr) | set(pm), key=lambda k: -tr.get(k, {}).get("total_ms", 0)):
            e = {}
            if k in tr:
                e.update(tr[k])
                e["per_call_ms"] = tr[k]["total_ms"] / 2   # warmup + timed call
            c = pm.get(k, {})
            if "FETCH_SIZE" in c:
                e["hbm_read_bytes"] = 2 * c["FETCH_SIZE"] * 1024
            if "WRITE_SIZE" in c:
                e["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
            if "hbm_read_bytes" in e:
                e["hbm_bytes_per_vote"] = (e["hbm_read_bytes"] + e.get("hbm_write_bytes", 0)) / nv
            if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
                tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
                e["tcc_hit_rate"] = c["TCC_HIT_sum"] / tot if tot else None
                e["tcc_requests_per_vote"] = tot / nv
            if c.get("SQ_WAVE_CYCLES"):
                wc = c["SQ_WAVE_CYCLES"]
                e["wait_inst_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / wc
                e["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / wc
                e["issue_frac"] = 1 - e["wait_inst_frac"] - e["wait_any_frac"]
            if "SQ_INSTS_VALU" in c:
                e["valu_lane_ops_per_vote"] = c["SQ_INSTS_VALU"] * 64 / nv
            if c.get("SQ_INSTS_LDS"):
                e["lds_bank_conflict_per_lds_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"]
            e["counters"] = c
            kern[k] = e
        res[tag] = {"mode": mode, "committee": N, "votes_per_call": nv,
                    "certs_per_s": bench.get("certs_per_s"), "ms_per_step": bench.get("ms_per_step"),
                    "kernels": kern}
    out = os.path.join(dst, "cert_pmc.json")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    # per committee size: HBM bytes per vote of one certificate call (the call's kernels
    # only), for bench.py's cert_stream roofline (profiles/cert_traffic.json)
    setup = ("k_sign", "k_keypair", "k_btab_build", "k_key_", "direct_copy", "elementwise",
             "vectorized", "__amd_rocclr")
    tr = {}
    for tag, r in res.items():
        if r["mode"] != "keyed":
            continue
        call_k = {k: e for k, e in r["kernels"].items()
                  if k.startswith("k_") and not k.startswith(setup)}   # library kernels
        per = list(call_k.values())
        if not per or any("hbm_read_bytes" not in e for e in per):
            continue
        tr[f"N{r['committee']}"] = {
            "hbm_bytes_per_vote": sum(e["hbm_bytes_per_vote"] for e in per),
            "kernels": sorted(call_k),
            "source": os.path.join(dst, "cert_pmc.json")}
    json.dump(tr, open(os.path.join(dst, "cert_traffic.json"), "w"), indent=1, sort_keys=True)
    for tag, r in res.items():
        print(f"== {tag}: {r['certs_per_s'] and r['certs_per_s'] / 1e6:.2f} M certs/s, "
              f"{r['ms_per_step']:.1f} ms/call")
        for k, e in list(r["kernels"].items())[:8]:
            print(f"  {k:28s} {e.get('per_call_ms', 0):8.2f} ms  "
                  f"B/vote {e.get('hbm_bytes_per_vote', 0):8.0f}  hit {e.get('tcc_hit_rate') or 0:.3f}  "
                  f"issue {e.get('issue_frac', 0):.2f} waitI {e.get('wait_inst_frac', 0):.2f} "
                  f"waitA {e.get('wait_any_frac', 0):.2f}  valu/vote {e.get('valu_lane_ops_per_vote', 0):8.0f}")


if __name__ == "__main__":
    main()
