#!/usr/bin/env python3
"""Per-phase split of k_verify_strict's VALU work from the PMC passes of
tools/strict_phases_pmc.sh: the full kernel and the phase-cut builds (nw_strict.hpp
NW_STRICT_STOP = 1..6) over the same 1,048,576-item config-4 launch. Lane-ops per verify =
instructions x 64 / items; a phase's work = the difference of consecutive cuts. Beside each
phase: its field-operation count (squarings S, products M) and the lane-ops those would cost
at the kernel's own instruction counts per operation (fe_sq / fe_mul as compiled, ISA
listing of tools/fe_asm.hip: ~103 / ~150 VALU instructions, 58 / 104 of them
v_mad_u64_u32), i.e. how far each
phase sits above its arithmetic.

    python tools/strict_phases_summary.py gpurun_out/strict_phases OUT.json [--items N]
"""
import csv
import glob
import json
import os
import sys

# (name, cut, field ops per verify at the kernel's algorithm: S squarings, M products,
#  note). Windows W ~= 33.2 per wave (66 % of lanes need 33, 0.35 % 34, the
# wave takes its maximum), 4 doublings per window after the first.
PHASES = [
    ("decompress A and R (two (p-5)/8 powers, sqrt_ratio_i)", 1, 2 * 255, 2 * 18, ""),
    ("per-lane tables j*A, j*R (1 doubling + 6 additions each, packed stores)", 2,
     2 * 4, 2 * 66, ""),
    ("SHA-512 of R||A||M and Barrett mod l", 3, 0, 0,
     "~4,200 32-bit ops per SHA-512 block + ~300 MACs (not field ops)"),
    ("half-size split (Lehmer), w = -v s mod l, recodings", 4, 0, 0, "scalar arithmetic"),
    ("ladder doublings (4 per window, ~129)", 5, 129 * 4, 129 * 3 + 33, ""),
    ("ladder A and R additions (~62, cached, table unpack)", 6, 0, 62 * 8, ""),
    ("ladder B additions (11, affine niels from the 2.15 GB tables) + final check", 0, 0,
     11 * 7 + 2, ""),
]
VALU_PER_S, VALU_PER_M = 103, 150   # tools/fe_asm.hip + asm_mix.py: 105 / 152 incl. ~2 address ops


def collect(d, key="k_verify_strict"):
    agg = {}
    for f in glob.glob(os.path.join(d, "**", "p_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return agg


def main():
    src, out = sys.argv[1], sys.argv[2]
    items = int(sys.argv[sys.argv.index("--items") + 1]) if "--items" in sys.argv else 1 << 20
    per = {}
    for v in ["stop1", "stop2", "stop3", "stop4", "stop5", "stop6", "full"]:
        c = collect(os.path.join(src, v))
        if not c:
            print(f"no counters for {v}", file=sys.stderr)
            continue
        per[v] = {k: c.get(k, 0.0) * 64 / items for k in
                  ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_INT32")}
    rows, prev = [], {"SQ_INSTS_VALU": 0.0, "SQ_INSTS_VALU_INT64": 0.0, "SQ_INSTS_VALU_INT32": 0.0}
    for name, cut, S, M, note in PHASES:
        v = f"stop{cut}" if cut else "full"
        if v not in per:
            continue
        cur = per[v]
        d = {k: cur[k] - prev[k] for k in cur}
        arith = S * VALU_PER_S + M * VALU_PER_M
        rows.append({"phase": name, "cut": v, "valu_lane_ops": round(d["SQ_INSTS_VALU"]),
                     "int64_lane_ops": round(d["SQ_INSTS_VALU_INT64"]),
                     "int32_lane_ops": round(d["SQ_INSTS_VALU_INT32"]),
                     "field_ops": {"S": S, "M": M}, "field_op_lane_ops": arith or None,
                     "excess_over_field_ops": (round(d["SQ_INSTS_VALU"] / arith, 3)
                                               if arith else None),
                     "note": note})
        prev = cur
    total = per.get("full", {}).get("SQ_INSTS_VALU")
    for r in rows:
        r["share"] = round(r["valu_lane_ops"] / total, 4) if total else None
    res = {"kernel": "k_verify_strict<false> (config 4)", "items": items,
           "valu_lane_ops_per_verify": round(total) if total else None,
           "method": "SQ_INSTS_VALU (+ INT64 / INT32) x 64 / items of phase-cut builds "
                     "(NW_STRICT_STOP, tools/strict_phases.sh + strict_phases_pmc.sh); a phase "
                     "= difference of consecutive cuts. field_op_lane_ops prices the phase's "
                     "squarings / products at ~103 / ~150 VALU instructions (the compiled "
                     "fe_sq / fe_mul).",
           "cuts": per, "phases": rows}
    json.dump(res, open(out, "w"), indent=2)
    for r in rows:
        print(f"{r['valu_lane_ops']:8d} {r['share'] or 0:6.3f} x{r['excess_over_field_ops'] or 0:5.2f} "
              f"{r['phase']}")
    print("total", res["valu_lane_ops_per_verify"])


if __name__ == "__main__":
    main()
