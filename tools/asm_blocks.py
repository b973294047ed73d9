#!/usr/bin/env python3
"""Per-basic-block summary of one kernel in a hipcc -S listing: size, v_mad_u64_u32,
s_nop, scratch / global / LDS ops and the block's branches (loop back-edges show which
blocks are loop bodies).   python tools/asm_blocks.py listing.s KERNEL_SUBSTRING [MINSIZE]"""
import collections
import re
import sys

path, key = sys.argv[1], sys.argv[2]
minsize = int(sys.argv[3]) if len(sys.argv) > 3 else 0
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + key + r"\w*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".size"))
blocks, cur, label = [], [], "entry"
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        blocks.append((label, cur))
        label, cur = m.group(1), []
        continue
    t = l.strip()
    if t and not t.startswith((".", ";")) and l.startswith("\t"):
        cur.append(t)
blocks.append((label, cur))
for lab, ins in blocks:
    if len(ins) < minsize:
        continue
    ops = collections.Counter(x.split()[0] for x in ins)
    scr = sum(v for k, v in ops.items() if k.startswith("scratch_"))
    glb = sum(v for k, v in ops.items() if k.startswith("global_"))
    lds = sum(v for k, v in ops.items() if k.startswith("ds_"))
    br = [x.split()[1] for x in ins if x.startswith("s_cbranch") or x.startswith("s_branch")]
    print(f"{lab:10s} n={len(ins):5d} mad={ops['v_mad_u64_u32']:4d} nop={ops['s_nop']:3d} "
          f"scr={scr:3d} glb={glb:3d} lds={lds:3d} -> {' '.join(br)}")
