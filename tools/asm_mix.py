#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing, per basic block and in total.

    python tools/asm_mix.py listing.s KERNEL_SUBSTRING [--blocks N]

Prints the kernel's total instruction count by opcode, then the N largest basic blocks
(label, size, scratch/global/LDS ops, v_mad_u64_u32 count) so the hot loop bodies and
their spill traffic can be read off without a GPU.
"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    nblocks = int(sys.argv[sys.argv.index("--blocks") + 1]) if "--blocks" in sys.argv else 12
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + key + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".size"))
    body = lines[start:end]
    total = collections.Counter()
    blocks, cur, label = [], collections.Counter(), "entry"
    for l in body:
        if re.match(r"^\.LBB\w+:", l):
            blocks.append((label, cur))
            label, cur = l.split(":")[0], collections.Counter()
            continue
        t = l.strip()
        if not t or t.startswith((".", ";")) or not l.startswith("\t"):
            continue
        op = t.split()[0]
        total[op] += 1
        cur[op] += 1
    blocks.append((label, cur))
    n = sum(total.values())
    print(f"{key}: {n} instructions")
    for op, c in total.most_common(40):
        print(f"  {op:28s} {c:7d}")
    print("largest basic blocks:")
    for label, c in sorted(blocks, key=lambda b: -sum(b[1].values()))[:nblocks]:
        sz = sum(c.values())
        scr = sum(v for k, v in c.items() if k.startswith("scratch_"))
        glb = sum(v for k, v in c.items() if k.startswith("global_"))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        print(f"  {label:14s} {sz:6d}  mad64={c['v_mad_u64_u32']:5d} scratch={scr:4d} "
              f"global={glb:4d} lds={lds:4d} accvgpr={c['v_accvgpr_read_b32'] + c['v_accvgpr_write_b32']:4d}")


if __name__ == "__main__":
    main()
