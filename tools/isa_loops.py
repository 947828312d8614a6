#!/usr/bin/env python3
"""Instruction mix per loop of one kernel in a gfx950 assembly listing (hipcc --cuda-device-only -S).

    python tools/isa_loops.py large.s persist_kernelILi0  [--blocks]

Basic blocks are grouped by the innermost loop header the compiler annotates ("in Loop: Header=...
Depth=d"); for each loop it prints the count of each instruction class (VALU, SALU, MFMA, LDS, VMEM,
v_readlane/v_writelane = SGPR spill traffic, s_waitcnt, s_nop) in the blocks of that loop, not
counting nested loops."""
import re
import sys
from collections import Counter, defaultdict


def classify(op):
    if op.startswith("v_mfma"):
        return "MFMA"
    if op in ("v_readlane_b32", "v_writelane_b32"):
        return "lane(spill)"
    if op.startswith("v_readfirstlane"):
        return "readfirstlane"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "VMEM"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    return "other"


def main():
    path, kern = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(kern) + r"\S*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    loop_of = {}
    cur_block, cur_loop = "entry", "none"
    counts = defaultdict(Counter)
    ops = defaultdict(Counter)
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\S+):(.*)$", l)
        if m:
            cur_block = m.group(1)
            c = m.group(2)
            h = re.search(r"Header=(\S+) Depth=(\d+)", c)
            if "Loop Header" in c:
                d = re.search(r"Depth=(\d+)", c).group(1)
                cur_loop = f"{cur_block} (d{d})"
            elif h:
                cur_loop = f".L{h.group(1)} (d{h.group(2)})"
            else:
                cur_loop = "none"
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        counts[cur_loop][classify(op)] += 1
        ops[cur_loop][op] += 1
    for loop, c in counts.items():
        tot = sum(c.values())
        print(f"{loop}: {tot} instructions: " + ", ".join(f"{k} {v}" for k, v in c.most_common()))
        if "--ops" in sys.argv:
            print("   ", ", ".join(f"{k} {v}" for k, v in ops[loop].most_common(40)))


if __name__ == "__main__":
    main()
